// fd_api.hip — the C-ABI (include/dvc.h) of the frame-differencing worker.
//
// Host side of one camera feed: owns the device state the reference keeps in
// Python locals (prev_gray fd:75-77,133; accumulated_mask fd:81,107), the
// contour-filter scratch, and the launch sequence of fd_kernels.hip for one
// frame (the body of the loop at frame_differencing.py:85-138).
#include <hip/hip_runtime.h>
#include <cstdlib>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/dvc.h"
#include "fd_kernels.h"
#include "host_common.h"

namespace dvc_host {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

const char* last_error() { return g_err.c_str(); }

// getGaussianKernelBitExact in double (OpenCV 4.11): the small binomial tables
// for sigma <= 0 and n <= 7, else exp(-x^2 / 2 sigma^2) normalised with the
// centre tap 1/sum. The float kernels of getGaussianKernel(CV_32F) are these
// values cast to float.
void gauss_f64(int n, double sigma, double* k)
{
    if (sigma <= 0 && n <= 7) {
        static const double t1[] = {1.0};
        static const double t3[] = {0.25, 0.5, 0.25};
        static const double t5[] = {0.0625, 0.25, 0.375, 0.25, 0.0625};
        static const double t7[] = {0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125};
        const double* t = n == 1 ? t1 : n == 3 ? t3 : n == 5 ? t5 : t7;
        for (int i = 0; i < n; ++i) k[i] = t[i];
        return;
    }
    double sx = sigma > 0 ? sigma : std::fma((double)n, 0.15, 0.35);
    double scale2X = -0.125 / (sx * sx);
    int n2 = (n - 1) / 2;
    double vals[64], sum = 0.0;
    for (int i = 0, x = 1 - n; i < n2; ++i, x += 2) {
        vals[i] = std::exp((double)(x * x) * scale2X);
        sum += vals[i];
    }
    sum = sum * 2.0 + 1.0;
    double mul1 = 1.0 / sum;
    for (int i = 0; i < n2; ++i) k[i] = k[n - 1 - i] = vals[i] * mul1;
    k[n2] = mul1;
}

void dct_matrix(int B, dvc::DctMat& M)
{
    const double PI = 3.14159265358979323846;
    for (int k = 0; k < B; ++k)
        for (int n = 0; n < B; ++n) {
            double c = k == 0 ? std::sqrt(1.0 / B) : std::sqrt(2.0 / B);
            M.m[k * B + n] = M.mt[n * B + k] = (float)(c * std::cos(PI * (2 * n + 1) * k / (2.0 * B)));
        }
}

}  // namespace dvc_host

namespace {

using dvc_host::fail;
using dvc_host::dct_matrix;

// getGaussianKernelBitExact + getGaussianKernelFixedPoint_ED (8 fraction bits):
// the taps OpenCV's 8U GaussianBlur uses (fd:77, fd:93).
int gauss_taps(int n, double sigma, uint16_t* taps)
{
    if (n < 1 || n > 63 || (n & 1) == 0) return -1;
    double k[64];
    dvc_host::gauss_f64(n, sigma, k);
    int n2 = n / 2;
    double err = 0.0;
    long long s = 0;
    for (int i = 0; i < n2; ++i) {
        double adj = k[i] * 256.0 + err;
        double v0 = std::nearbyint(adj);
        err = adj - v0;
        taps[i] = taps[n - 1 - i] = (uint16_t)v0;
        s += (long long)v0;
    }
    taps[n2] = (uint16_t)(256 - 2 * s);
    return 0;
}

}  // namespace

// Buffers of one batch in flight (max_batch frames): motion masks, contour-
// filter scratch, kept masks and the dilate -> accumulate -> out bit fields.
struct Slot {
    dvc::CclBufs c{};
    uint64_t *dblk = nullptr, *rblk = nullptr, *sbits = nullptr;   // k_dilate -> k_acc -> k_out bits
    hipEvent_t ev_front = nullptr, ev_ccl = nullptr, ev_acc = nullptr, ev_out = nullptr;
    bool recorded = false;  // the events hold a batch that the next user of the slot must wait for
};

// Batches in flight: three slots.
constexpr int NSLOT = 3;

struct dvc_fd {
    dvc_fd_params p{};
    int device = 0;
    hipStream_t stream = nullptr;  // prime + contour filter (internal)
    hipStream_t user = nullptr;    // the caller's stream (create's hip_stream; NULL = legacy default)
    bool has_user = false;         // join `user` (hip_stream given, or DVC_FLAG_JOIN_STREAM)
    hipEvent_t ev_user = nullptr, ev_join_out = nullptr, ev_join_acc = nullptr;
    hipStream_t s_front = nullptr;       // blur/threshold front (previous-gray recurrence)
    hipStream_t s_acc = nullptr;         // dilate + accumulate (accumulated-mask recurrence)
    hipStream_t s_out = nullptr;         // overlay + compressed frames
    dvc::RowGeom g{};
    dvc::GaussTaps kprime{};
    dvc::DctMat M{};
    bool primed = false;
    int max_batch = 1;
    int SW = 0;          // 64-block words per block row
    size_t sstride = 0;  // static-block bit words per frame
    uint64_t frames = 0, seq = 0;  // frames stepped, batches launched
    int last_n = 0;                // frames of the last batch
    Slot slot[NSLOT];
    // device state
    uint8_t* gray[2] = {nullptr, nullptr};  // previous blurred gray (fd:77, 133): gray[gcur]
    int gcur = 0;
    uint8_t* acc = nullptr;        // accumulated mask (fd:81, 107)
    uint64_t* dbg_dil = nullptr;
    uint32_t* tmp32 = nullptr;
    uint8_t* gtmp = nullptr;
    unsigned long long* stats = nullptr;
    // host-pointer staging (max_batch frames)
    uint8_t *d_in = nullptr, *d_ov = nullptr, *d_cp = nullptr;
    uint8_t *h_in = nullptr, *h_ov = nullptr, *h_cp = nullptr, *h_acc = nullptr;
    // dominant-kernel timing
    std::vector<hipEvent_t> ev;
    size_t ev_used = 0;
};

static void free_all(dvc_fd* h)
{
    for (Slot& s : h->slot) {
        void* dev[] = {s.c.mbits, s.c.fbits, s.c.kbits, s.c.rs, s.c.re, s.c.nfg, s.c.fpar, s.c.gpar, s.c.area2, s.c.gE,
                       s.dblk, s.rblk, s.sbits};
        for (void* p : dev)
            if (p) (void)hipFree(p);
        for (hipEvent_t e : {s.ev_front, s.ev_ccl, s.ev_acc, s.ev_out})
            if (e) (void)hipEventDestroy(e);
    }
    void* dev[] = {h->gray[0], h->gray[1], h->acc, h->dbg_dil, h->tmp32, h->gtmp, h->stats, h->d_in, h->d_ov, h->d_cp};
    for (void* p : dev)
        if (p) (void)hipFree(p);
    void* pin[] = {h->h_in, h->h_ov, h->h_cp, h->h_acc};
    for (void* p : pin)
        if (p) (void)hipHostFree(p);
    for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
    for (hipEvent_t e : {h->ev_user, h->ev_join_out, h->ev_join_acc})
        if (e) (void)hipEventDestroy(e);
    for (hipStream_t st : {h->s_front, h->s_acc, h->s_out, h->stream})
        if (st) (void)hipStreamDestroy(st);
}

template <typename T>
static hipError_t dalloc(T** p, size_t bytes)
{
    return hipMalloc(reinterpret_cast<void**>(p), bytes ? bytes : 16);
}

// The caller's stream (if any) -> every internal stream: work the caller queued
// before this call (e.g. the copy that produced the frames, or reads of the
// previous outputs) happens before the call's kernels.
static hipError_t wait_user(dvc_fd* h)
{
    if (!h->has_user) return hipSuccess;
    hipError_t e = hipEventRecord(h->ev_user, h->user);
    for (hipStream_t st : {h->stream, h->s_front, h->s_acc, h->s_out})
        if (e == hipSuccess) e = hipStreamWaitEvent(st, h->ev_user, 0);
    return e;
}

// Internal streams -> the caller's stream: work the caller queues after this
// call sees its outputs (overlay/compressed on s_out, acc_out on s_acc).
static hipError_t join_user(dvc_fd* h)
{
    if (!h->has_user) return hipSuccess;
    hipError_t e = hipEventRecord(h->ev_join_out, h->s_out);
    if (e == hipSuccess) e = hipEventRecord(h->ev_join_acc, h->s_acc);
    if (e == hipSuccess) e = hipStreamWaitEvent(h->user, h->ev_join_out, 0);
    if (e == hipSuccess) e = hipStreamWaitEvent(h->user, h->ev_join_acc, 0);
    return e;
}

static hipError_t sync_all(dvc_fd* h)
{
    hipError_t e = hipStreamSynchronize(h->stream);
    for (hipStream_t st : {h->s_front, h->s_acc, h->s_out})
        if (e == hipSuccess && st) e = hipStreamSynchronize(st);
    return e;
}

extern "C" {

int dvc_abi_version(void) { return DVC_ABI_VERSION; }

const char* dvc_last_error(void) { return dvc_host::last_error(); }

int dvc_device_count(int* count)
{
    if (!count) return fail(DVC_E_INVALID, "count is NULL");
    HIP_OK(hipGetDeviceCount(count));
    return DVC_OK;
}

int dvc_gaussian_taps_q8(int n, double sigma, uint16_t* taps)
{
    if (!taps || gauss_taps(n, sigma, taps) != 0) return fail(DVC_E_INVALID, "kernel size must be odd, 1..63");
    return DVC_OK;
}

int dvc_fd_create(const dvc_fd_params* prm, int device, void* hip_stream, dvc_fd** out)
{
    if (!prm || !out) return fail(DVC_E_INVALID, "NULL argument");
    const dvc_fd_params& p = *prm;
    if (p.width < 16 || p.height < 16 || p.width > 65520)
        return fail(DVC_E_INVALID, "frame %dx%d outside 16..65520 x >=16", p.width, p.height);
    if (p.block != 4 && p.block != 8)
        return fail(DVC_E_UNSUPPORTED, "block_size %d: the GPU path implements 4 and 8", p.block);
    if (p.width % p.block || p.height % p.block)
        return fail(DVC_E_UNSUPPORTED, "frame %dx%d is not a multiple of block_size %d", p.width, p.height, p.block);
    if (p.ksize < 1 || p.ksize > 63 || p.anchor < 0 || p.anchor >= p.ksize)
        return fail(DVC_E_INVALID, "dilation kernel %d (anchor %d) outside 1..63", p.ksize, p.anchor);
    if (p.ithresh < -1 || p.ithresh > 255) return fail(DVC_E_INVALID, "ithresh %d outside -1..255", p.ithresh);
    if (!(p.quant == p.quant) || p.quant == 0.0f) return fail(DVC_E_INVALID, "quantization_level must be nonzero");
    const int mb = p.max_batch == 0 ? 1 : (int)p.max_batch;
    if (p.max_batch > DVC_MAX_BATCH) return fail(DVC_E_INVALID, "max_batch %u outside 1..%d", p.max_batch, DVC_MAX_BATCH);
    dvc_fd* h = new dvc_fd();
    h->p = p;
    h->device = device;
    h->max_batch = mb;
    h->g.W = p.width;
    h->g.H = p.height;
    h->g.WW = (p.width + 63) / 64;
    h->g.CAP = p.width / 2 + 1;
    h->SW = (p.width / p.block + 63) / 64;
    h->sstride = (size_t)(p.height / p.block) * h->SW;
    if (gauss_taps(p.prime_ksize, p.prime_sigma, h->kprime.t) != 0) {
        delete h;
        return fail(DVC_E_INVALID, "prime blur size %d must be odd, 1..63", p.prime_ksize);
    }
    h->kprime.n = p.prime_ksize;
    dct_matrix(p.block, h->M);
    auto bad = [&](hipError_t e, const char* what) {
        int rc = fail(e == hipErrorOutOfMemory ? DVC_E_NOMEM : DVC_E_HIP, "%s: %s", what, hipGetErrorString(e));
        free_all(h);
        delete h;
        return rc;
    };
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return bad(e, "hipSetDevice");
    h->user = (hipStream_t)hip_stream;
    h->has_user = hip_stream != nullptr || (p.flags & DVC_FLAG_JOIN_STREAM);
    // four internal streams — contour filter, front, accumulate, output —
    // within the default 4 hardware queues (a queue shared by two stages
    // serialises them); priorities: the latency-bound contour filter and
    // accumulate chains high, the VALU-bound front low. The caller's stream (if
    // any) is only joined: each call waits for the work queued on it before the
    // call, and work queued on it after the call waits for the call's outputs.
    int plo = 0, phi = 0;
    (void)hipDeviceGetStreamPriorityRange(&plo, &phi);
    auto mk = [](hipStream_t* st, int prio) { return hipStreamCreateWithPriority(st, hipStreamNonBlocking, prio); };
    if ((e = mk(&h->stream, phi)) != hipSuccess) return bad(e, "hipStreamCreate");
    for (hipEvent_t* ev : {&h->ev_user, &h->ev_join_out, &h->ev_join_acc})
        if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    for (auto sp : {std::make_pair(&h->s_front, plo), std::make_pair(&h->s_acc, phi), std::make_pair(&h->s_out, 0)})
        if ((e = mk(sp.first, sp.second)) != hipSuccess) return bad(e, "hipStreamCreate");
    const size_t W = p.width, H = p.height, N = W * H, WW = h->g.WW;
    for (Slot& s : h->slot) {
        size_t sz[10];
        dvc::CclBufs::sizes(h->g, mb, sz);
        void** ptrs[10] = {(void**)&s.c.mbits, (void**)&s.c.fbits, (void**)&s.c.rs, (void**)&s.c.re,
                           (void**)&s.c.nfg, (void**)&s.c.fpar, (void**)&s.c.gpar, (void**)&s.c.gE,
                           (void**)&s.c.area2, (void**)&s.c.kbits};
        for (int i = 0; i < 10; ++i)
            if ((e = dalloc(ptrs[i], sz[i])) != hipSuccess) return bad(e, "hipMalloc");
        // block fields: (W/B)(H/B) x B*B bits = W*H/8 bytes per frame <= 8*H*WW
        if ((e = dalloc(&s.dblk, 8 * H * WW * (size_t)mb)) != hipSuccess) return bad(e, "hipMalloc");
        if ((e = dalloc(&s.rblk, 8 * H * WW * (size_t)mb)) != hipSuccess) return bad(e, "hipMalloc");
        if ((e = dalloc(&s.sbits, 8 * h->sstride * (size_t)mb)) != hipSuccess) return bad(e, "hipMalloc");
        for (hipEvent_t* ev : {&s.ev_front, &s.ev_ccl, &s.ev_acc, &s.ev_out})
            if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    }
    struct { void** ptr; size_t bytes; } allocs[] = {
        {(void**)&h->gray[0], N}, {(void**)&h->gray[1], N}, {(void**)&h->acc, N}, {(void**)&h->stats, 8 * 4 * 64},
    };
    for (auto& a : allocs)
        if ((e = dalloc(a.ptr, a.bytes)) != hipSuccess) return bad(e, "hipMalloc");
    for (Slot& s : h->slot) s.c.stats = h->stats;
    if (p.flags & DVC_FLAG_KEEP_PLANES) {
        if ((e = dalloc(&h->dbg_dil, 8 * H * WW)) != hipSuccess) return bad(e, "hipMalloc");
    }
    if (!(p.flags & DVC_FLAG_DEVICE_PTRS)) {
        const size_t F = 3 * N * (size_t)mb;
        if ((e = dalloc(&h->d_in, F)) != hipSuccess) return bad(e, "hipMalloc");
        if ((e = dalloc(&h->d_ov, F)) != hipSuccess) return bad(e, "hipMalloc");
        if ((e = dalloc(&h->d_cp, F)) != hipSuccess) return bad(e, "hipMalloc");
        if ((e = hipHostMalloc((void**)&h->h_in, F)) != hipSuccess) return bad(e, "hipHostMalloc");
        if ((e = hipHostMalloc((void**)&h->h_ov, F)) != hipSuccess) return bad(e, "hipHostMalloc");
        if ((e = hipHostMalloc((void**)&h->h_cp, F)) != hipSuccess) return bad(e, "hipHostMalloc");
        if ((e = hipHostMalloc((void**)&h->h_acc, N)) != hipSuccess) return bad(e, "hipHostMalloc");
    }
    if ((e = hipMemsetAsync(h->stats, 0, 8 * 4 * 64, h->stream)) != hipSuccess) return bad(e, "hipMemset");
    // the OUTSIDE gap node of every frame slice is its own root before any
    // k_band runs (its over-budget path may walk through it)
    for (Slot& s : h->slot) {
        size_t sz[10];
        dvc::CclBufs::sizes(h->g, mb, sz);
        if ((e = hipMemsetAsync(s.c.gpar, 0, sz[6], h->stream)) != hipSuccess) return bad(e, "hipMemset");
    }
    if ((e = hipStreamSynchronize(h->stream)) != hipSuccess) return bad(e, "hipStreamSynchronize");
    *out = h;
    return DVC_OK;
}

int dvc_fd_prime(dvc_fd* h, const uint8_t* bgr, size_t pitch)
{
    if (!h || !bgr) return fail(DVC_E_INVALID, "NULL argument");
    if (pitch < 3 * (size_t)h->p.width || pitch % 4) return fail(DVC_E_INVALID, "pitch %zu invalid", pitch);
    HIP_OK(hipSetDevice(h->device));
    const size_t W = h->p.width, H = h->p.height, N = W * H;
    if (!h->tmp32) {
        HIP_OK(dalloc(&h->tmp32, 4 * N));
        HIP_OK(dalloc(&h->gtmp, N));
    }
    HIP_OK(sync_all(h));  // no batch of a previous run may still be in flight
    HIP_OK(wait_user(h));
    const uint8_t* d = bgr;
    int dp = (int)pitch;
    if (!(h->p.flags & DVC_FLAG_DEVICE_PTRS)) {
        for (size_t y = 0; y < H; ++y) std::memcpy(h->h_in + y * 3 * W, bgr + y * pitch, 3 * W);
        HIP_OK(hipMemcpyAsync(h->d_in, h->h_in, 3 * N, hipMemcpyHostToDevice, h->stream));
        d = h->d_in;
        dp = (int)(3 * W);
    }
    HIP_OK(dvc::launch_prime(d, dp, h->gtmp, h->tmp32, h->gray[h->gcur], h->p.width, h->p.height, h->kprime, h->stream));
    HIP_OK(hipMemsetAsync(h->acc, 0, N, h->stream));
    HIP_OK(hipMemsetAsync(h->stats, 0, 8 * 4 * 64, h->stream));
    HIP_OK(hipStreamSynchronize(h->stream));
    for (Slot& s : h->slot) s.recorded = false;
    h->frames = 0;
    h->seq = 0;
    h->last_n = 0;
    h->primed = true;
    return DVC_OK;
}

}  // extern "C"

// Enqueue one batch i of n <= max_batch device-resident frames, slot S = i % 3
// (j = i - 3 = the slot's previous batch):
//   s_front:         [wait ccl(j)]            front(i) -> ev_front   (S.mbits free)
//   stream:          [wait ev_front, acc(j)]  contour filter(i) -> ev_ccl (S.kbits free)
//   s_acc:           [wait ev_ccl, out(j)]    dilate + accumulate(i) -> ev_acc (S bits free)
//   s_out:           [wait ev_acc]            k_out(i) -> ev_out
// so front(i+2), the contour filter of i+1, the accumulation of i and the
// output of i-1 can all be in flight; the two recurrences (previous gray,
// accumulated mask) are serial, each on its own stream.
static int enqueue_batch(dvc_fd* h, const uint8_t* d, int dp, size_t fstride, int n, uint8_t* ov, uint8_t* cp,
                         size_t ostride)
{
    Slot& S = h->slot[h->seq % NSLOT];
    hipStream_t s_ccl = h->stream;
    if (S.recorded) HIP_OK(hipStreamWaitEvent(h->s_front, S.ev_ccl, 0));
    HIP_OK(dvc::launch_front(d, dp, fstride, n, h->gray[h->gcur], h->gray[h->gcur ^ 1], S.c.mbits, h->g,
                             h->p.ithresh, h->s_front));
    HIP_OK(hipEventRecord(S.ev_front, h->s_front));
    h->gcur ^= 1;
    HIP_OK(hipStreamWaitEvent(s_ccl, S.ev_front, 0));
    if (S.recorded) HIP_OK(hipStreamWaitEvent(s_ccl, S.ev_acc, 0));
    HIP_OK(dvc::launch_ccl(S.c, h->g, n, h->p.min_area2, s_ccl));
    HIP_OK(hipEventRecord(S.ev_ccl, s_ccl));
    HIP_OK(hipStreamWaitEvent(h->s_acc, S.ev_ccl, 0));
    if (S.recorded) HIP_OK(hipStreamWaitEvent(h->s_acc, S.ev_out, 0));
    dvc::BackArgs a{};
    a.g = h->g;
    a.bgr = d;
    a.pitch = dp;
    a.fstride = fstride;
    a.acc = h->acc;
    a.overlay = ov;
    a.compressed = cp;
    a.opitch = 3 * h->p.width;
    a.ostride = ostride;
    a.kbits = S.c.kbits;
    a.dblk = S.dblk;
    a.rblk = S.rblk;
    a.sbits = S.sbits;
    a.SW = h->SW;
    a.sstride = h->sstride;
    a.n = n;
    a.ksize = h->p.ksize;
    a.anchor = h->p.anchor;
    a.alpha = h->p.alpha;
    a.beta = h->p.beta;
    a.gamma = h->p.gamma;
    a.quant = h->p.quant;
    a.qinv = 1.0 / (double)h->p.quant;
    {
        const float z = std::rint(std::fmaf(0.0f, h->p.alpha, std::fmaf(0.0f, h->p.beta, h->p.gamma)));
        a.acc0_fixed = z < 0.5f && z > -0.5f;  // saturate_cast<uchar>(0) == 0 (NaN/negatives excluded)
    }
    a.M = h->M;
    a.stats = h->stats;
    a.dbg_dil = h->dbg_dil;
    // KTIMING: events around k_out (the HBM-bound kernel) on s_out
    const bool timed = h->p.flags & DVC_FLAG_KTIMING;
    if (timed) {
        while (h->ev.size() < h->ev_used + 2) {
            hipEvent_t e;
            HIP_OK(hipEventCreate(&e));
            h->ev.push_back(e);
        }
    }
    HIP_OK(dvc::launch_accumulate(a, h->p.block, h->s_acc));
    HIP_OK(hipEventRecord(S.ev_acc, h->s_acc));
    HIP_OK(hipStreamWaitEvent(h->s_out, S.ev_acc, 0));
    if (timed) HIP_OK(hipEventRecord(h->ev[h->ev_used], h->s_out));
    HIP_OK(dvc::launch_out(a, h->p.block, h->s_out));
    if (timed) {
        HIP_OK(hipEventRecord(h->ev[h->ev_used + 1], h->s_out));
        h->ev_used += 2;
    }
    HIP_OK(hipEventRecord(S.ev_out, h->s_out));
    S.recorded = true;
    h->seq++;
    h->frames += (uint64_t)n;
    h->last_n = n;
    return DVC_OK;
}

// n frames in chunks of max_batch; host pointers are staged through the pinned
// buffers (each chunk completes before the call returns).
static int run_frames(dvc_fd* h, const uint8_t* bgr, size_t pitch, size_t fstride, int n, uint8_t* overlay,
                      uint8_t* compressed, size_t ostride, uint8_t* acc_out)
{
    if (!h || !bgr) return fail(DVC_E_INVALID, "NULL argument");
    if (!h->primed) return fail(DVC_E_STATE, "step before dvc_fd_prime");
    if (n < 0) return fail(DVC_E_INVALID, "negative frame count");
    const size_t W = h->p.width, H = h->p.height, N = W * H, row = 3 * W;
    if (pitch < row || pitch % 4) return fail(DVC_E_INVALID, "pitch %zu invalid", pitch);
    if (n > 1 && (fstride < pitch * (H - 1) + row || fstride % 4))
        return fail(DVC_E_INVALID, "frame stride %zu invalid", fstride);
    if (n > 1 && (overlay || compressed) && (ostride < 3 * N || ostride % 4))
        return fail(DVC_E_INVALID, "output frame stride %zu invalid", ostride);
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(wait_user(h));
    const bool devp = h->p.flags & DVC_FLAG_DEVICE_PTRS;
    for (int f0 = 0; f0 < n; f0 += h->max_batch) {
        const int m = std::min(h->max_batch, n - f0);
        const uint8_t* in = bgr + (size_t)f0 * fstride;
        uint8_t* ov = overlay ? overlay + (size_t)f0 * ostride : nullptr;
        uint8_t* cp = compressed ? compressed + (size_t)f0 * ostride : nullptr;
        if (devp) {
            int rc = enqueue_batch(h, in, (int)pitch, fstride, m, ov, cp, ostride);
            if (rc) return rc;
            continue;
        }
        for (int t = 0; t < m; ++t)
            for (size_t y = 0; y < H; ++y)
                std::memcpy(h->h_in + (size_t)t * 3 * N + y * row, in + (size_t)t * fstride + y * pitch, row);
        HIP_OK(hipMemcpyAsync(h->d_in, h->h_in, (size_t)m * 3 * N, hipMemcpyHostToDevice, h->s_front));
        int rc = enqueue_batch(h, h->d_in, (int)row, 3 * N, m, ov ? h->d_ov : nullptr, cp ? h->d_cp : nullptr, 3 * N);
        if (rc) return rc;
        if (ov) HIP_OK(hipMemcpyAsync(h->h_ov, h->d_ov, (size_t)m * 3 * N, hipMemcpyDeviceToHost, h->s_out));
        if (cp) HIP_OK(hipMemcpyAsync(h->h_cp, h->d_cp, (size_t)m * 3 * N, hipMemcpyDeviceToHost, h->s_out));
        HIP_OK(sync_all(h));
        for (int t = 0; t < m; ++t) {
            if (ov) std::memcpy(ov + (size_t)t * ostride, h->h_ov + (size_t)t * 3 * N, 3 * N);
            if (cp) std::memcpy(cp + (size_t)t * ostride, h->h_cp + (size_t)t * 3 * N, 3 * N);
        }
    }
    if (acc_out) {
        if (devp) {
            HIP_OK(hipMemcpyAsync(acc_out, h->acc, N, hipMemcpyDeviceToDevice, h->s_acc));
        } else {
            HIP_OK(hipMemcpyAsync(h->h_acc, h->acc, N, hipMemcpyDeviceToHost, h->s_acc));
            HIP_OK(hipStreamSynchronize(h->s_acc));
            std::memcpy(acc_out, h->h_acc, N);
        }
    }
    HIP_OK(join_user(h));
    return DVC_OK;
}

extern "C" {

int dvc_fd_step(dvc_fd* h, const uint8_t* bgr, size_t pitch, uint8_t* overlay, uint8_t* compressed,
                uint8_t* acc_out)
{
    return run_frames(h, bgr, pitch, 0, 1, overlay, compressed, 0, acc_out);
}

int dvc_fd_step_batch(dvc_fd* h, const uint8_t* bgr, size_t pitch, size_t frame_stride, int n, uint8_t* overlay,
                      uint8_t* compressed, size_t out_stride)
{
    return run_frames(h, bgr, pitch, frame_stride, n, overlay, compressed, out_stride, nullptr);
}

int dvc_fd_sync(dvc_fd* h)
{
    if (!h) return fail(DVC_E_INVALID, "NULL handle");
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(sync_all(h));
    return DVC_OK;
}

int dvc_fd_get_stats(dvc_fd* h, dvc_fd_stats* out)
{
    if (!h || !out) return fail(DVC_E_INVALID, "NULL argument");
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(sync_all(h));
    unsigned long long slots[64 * 4], s[4] = {0, 0, 0, 0};
    HIP_OK(hipMemcpy(slots, h->stats, sizeof(slots), hipMemcpyDeviceToHost));
    for (int i = 0; i < 64 * 4; ++i) s[i % 4] += slots[i];
    out->frames = h->frames;
    out->motion_px = s[1];
    out->components = s[2];
    out->static_blocks = s[3];
    return DVC_OK;
}

int dvc_fd_read_plane(dvc_fd* h, int plane, uint8_t* dst)
{
    if (!h || !dst) return fail(DVC_E_INVALID, "NULL argument");
    if (!h->frames) return fail(DVC_E_STATE, "no frame stepped yet");
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(sync_all(h));
    const size_t W = h->p.width, H = h->p.height, N = W * H, WW = h->g.WW;
    if (plane == DVC_PLANE_GRAY || plane == DVC_PLANE_ACC) {
        HIP_OK(hipMemcpy(dst, plane == DVC_PLANE_GRAY ? h->gray[h->gcur] : h->acc, N, hipMemcpyDeviceToHost));
        return DVC_OK;
    }
    // the last frame of the last batch
    const dvc::CclBufs c = h->slot[(h->seq - 1) % NSLOT].c.frame((size_t)h->last_n - 1, h->g);
    const uint64_t* src = plane == DVC_PLANE_MOTION ? c.mbits
                        : plane == DVC_PLANE_FILTERED ? c.kbits
                        : plane == DVC_PLANE_DILATED ? h->dbg_dil : nullptr;
    if (plane != DVC_PLANE_MOTION && plane != DVC_PLANE_FILTERED && plane != DVC_PLANE_DILATED)
        return fail(DVC_E_INVALID, "unknown plane %d", plane);
    if (!src) return fail(DVC_E_STATE, "plane %d needs DVC_FLAG_KEEP_PLANES", plane);
    std::vector<uint64_t> bits(H * WW);
    HIP_OK(hipMemcpy(bits.data(), src, 8 * H * WW, hipMemcpyDeviceToHost));
    for (size_t y = 0; y < H; ++y)
        for (size_t x = 0; x < W; ++x) dst[y * W + x] = ((bits[y * WW + x / 64] >> (x % 64)) & 1) ? 255 : 0;
    return DVC_OK;
}

int dvc_fd_ktime(dvc_fd* h, double* total_ms, uint64_t* launches, int reset)
{
    if (!h) return fail(DVC_E_INVALID, "NULL handle");
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(sync_all(h));
    double t = 0.0;
    for (size_t i = 0; i + 1 < h->ev_used; i += 2) {
        float ms = 0.f;
        HIP_OK(hipEventElapsedTime(&ms, h->ev[i], h->ev[i + 1]));
        t += ms;
    }
    if (total_ms) *total_ms = t;
    if (launches) *launches = h->ev_used / 2;
    if (reset) h->ev_used = 0;
    return DVC_OK;
}

void dvc_fd_destroy(dvc_fd* h)
{
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)sync_all(h);
    free_all(h);
    delete h;
}

int dvc_contour_filter(const uint8_t* mask, int width, int height, int64_t min_area2, int device,
                       uint8_t* filtered, uint64_t* components)
{
    if (!mask || !filtered) return fail(DVC_E_INVALID, "NULL argument");
    if (width < 4 || height < 4 || width % 4 || height % 4 || width > 65520)
        return fail(DVC_E_INVALID, "mask %dx%d: sides must be multiples of 4", width, height);
    HIP_OK(hipSetDevice(device));
    dvc::RowGeom g{width, height, (width + 63) / 64, width / 2 + 1};
    const size_t W = width, H = height, N = W * H, WW = g.WW, CAP = g.CAP;
    std::vector<uint64_t> bits(H * WW, 0);
    for (size_t y = 0; y < H; ++y)
        for (size_t x = 0; x < W; ++x)
            if (mask[y * W + x]) bits[y * WW + x / 64] |= 1ull << (x % 64);
    std::vector<void*> owned;
    auto alloc = [&](size_t bytes) -> void* {
        void* p = nullptr;
        if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) return nullptr;
        owned.push_back(p);
        return p;
    };
    uint64_t* mbits = (uint64_t*)alloc(8 * H * WW);
    uint64_t* fbits = (uint64_t*)alloc(8 * H * WW);
    uint64_t* kept = (uint64_t*)alloc(8 * H * WW);
    uint16_t* rs = (uint16_t*)alloc(2 * H * CAP);
    uint16_t* re = (uint16_t*)alloc(2 * H * CAP);
    uint32_t* nfg = (uint32_t*)alloc(4 * H);
    uint32_t* fpar = (uint32_t*)alloc(4 * H * CAP);
    uint32_t* gpar = (uint32_t*)alloc(4 * (1 + H * (CAP + 1)));
    uint8_t* gE = (uint8_t*)alloc(H * (CAP + 1));
    uint32_t* area2 = (uint32_t*)alloc(4 * H * CAP);
    unsigned long long* stats = (unsigned long long*)alloc(8 * 4 * 64);
    int rc = DVC_OK;
    auto done = [&]() { for (void* p : owned) (void)hipFree(p); };
    for (void* p : owned)
        if (!p) { done(); return fail(DVC_E_NOMEM, "hipMalloc failed"); }
    hipStream_t s = nullptr;
    hipError_t e = hipMemcpy(mbits, bits.data(), 8 * H * WW, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(stats, 0, 8 * 4 * 64);
    if (e == hipSuccess) e = hipMemset(gpar, 0, 4 * (1 + H * (CAP + 1)));
    if (e == hipSuccess) {
        dvc::CclBufs c{mbits, fbits, rs, re, nfg, fpar, gpar, gE, area2, kept, stats};
        e = dvc::launch_ccl(c, g, 1, min_area2, s);
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    unsigned long long st[4] = {0, 0, 0, 0}, slots[64 * 4];
    if (e == hipSuccess) e = hipMemcpy(bits.data(), kept, 8 * H * WW, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(slots, stats, sizeof(slots), hipMemcpyDeviceToHost);
    for (int i = 0; i < 64 * 4; ++i) st[i % 4] += slots[i];
    if (e != hipSuccess) rc = fail(DVC_E_HIP, "contour filter: %s", hipGetErrorString(e));
    done();
    if (rc) return rc;
    for (size_t y = 0; y < H; ++y)
        for (size_t x = 0; x < W; ++x) filtered[y * W + x] = ((bits[y * WW + x / 64] >> (x % 64)) & 1) ? 255 : 0;
    if (components) *components = st[2];
    return DVC_OK;
}

}  // extern "C"
