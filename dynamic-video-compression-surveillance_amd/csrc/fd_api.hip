// fd_api.hip — the C-ABI (include/dvc.h) of the frame-differencing worker.
//
// Host side of one camera feed: owns the device state the reference keeps in
// Python locals (prev_gray fd:75-77,133; accumulated_mask fd:81,107), the
// contour-filter scratch, and the launch sequence of fd_kernels.hip for one
// frame (the body of the loop at frame_differencing.py:85-138).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/dvc.h"
#include "fd_kernels.h"

namespace {

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

#define HIP_OK(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(DVC_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),     \
                        __FILE__, __LINE__);                                                  \
    } while (0)

// getGaussianKernelBitExact + getGaussianKernelFixedPoint_ED (8 fraction bits):
// the taps OpenCV's 8U GaussianBlur uses (fd:77, fd:93).
int gauss_taps(int n, double sigma, uint16_t* taps)
{
    if (n < 1 || n > 63 || (n & 1) == 0) return -1;
    double k[64];
    if (sigma <= 0 && n <= 7) {
        static const double t1[] = {1.0};
        static const double t3[] = {0.25, 0.5, 0.25};
        static const double t5[] = {0.0625, 0.25, 0.375, 0.25, 0.0625};
        static const double t7[] = {0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125};
        const double* t = n == 1 ? t1 : n == 3 ? t3 : n == 5 ? t5 : t7;
        for (int i = 0; i < n; ++i) k[i] = t[i];
    } else {
        double sx = sigma > 0 ? sigma : std::fma((double)n, 0.15, 0.35);
        double scale2X = -0.125 / (sx * sx);
        int n2 = (n - 1) / 2;
        double vals[32], sum = 0.0;
        for (int i = 0, x = 1 - n; i < n2; ++i, x += 2) {
            vals[i] = std::exp((double)(x * x) * scale2X);
            sum += vals[i];
        }
        sum = sum * 2.0 + 1.0;
        double mul1 = 1.0 / sum;
        for (int i = 0; i < n2; ++i) k[i] = k[n - 1 - i] = vals[i] * mul1;
        k[n2] = mul1;
    }
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

void dct_matrix(int B, float* M)
{
    const double PI = 3.14159265358979323846;
    for (int k = 0; k < B; ++k)
        for (int n = 0; n < B; ++n) {
            double c = k == 0 ? std::sqrt(1.0 / B) : std::sqrt(2.0 / B);
            M[k * B + n] = (float)(c * std::cos(PI * (2 * n + 1) * k / (2.0 * B)));
        }
}

}  // namespace

struct dvc_fd {
    dvc_fd_params p{};
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    dvc::RowGeom g{};
    dvc::GaussTaps kprime{};
    dvc::DctMat M{};
    bool primed = false;
    int cur = 0;              // gray[cur] = previous blurred gray
    uint64_t frames = 0;
    // device state
    uint8_t* gray[2] = {nullptr, nullptr};
    uint8_t* acc = nullptr;
    uint64_t *mbits = nullptr, *fbits = nullptr, *dbg_kept = nullptr, *dbg_dil = nullptr;
    uint16_t *rs = nullptr, *re = nullptr;
    uint32_t *nfg = nullptr, *fpar = nullptr, *gpar = nullptr, *area2 = nullptr, *tmp32 = nullptr;
    uint8_t *gE = nullptr, *gtmp = nullptr;
    unsigned long long* stats = nullptr;
    // host-pointer staging
    uint8_t *d_frame = nullptr, *d_ov = nullptr, *d_cp = nullptr;
    uint8_t *h_in = nullptr, *h_ov = nullptr, *h_cp = nullptr, *h_acc = nullptr;
    // dominant-kernel timing
    std::vector<hipEvent_t> ev;
    size_t ev_used = 0;
    // hipGraph of a captured frame sequence
    bool capturing = false;
    int cap_cur = 0;
    uint64_t cap_frames = 0;
    hipGraph_t graph = nullptr;
    hipGraphExec_t gexec = nullptr;
};

static void free_all(dvc_fd* h)
{
    void* dev[] = {h->gray[0], h->gray[1], h->acc, h->mbits, h->fbits, h->dbg_kept, h->dbg_dil, h->rs, h->re,
                   h->nfg, h->fpar, h->gpar, h->area2, h->tmp32, h->gE, h->gtmp, h->stats, h->d_frame,
                   h->d_ov, h->d_cp};
    for (void* p : dev)
        if (p) (void)hipFree(p);
    void* pin[] = {h->h_in, h->h_ov, h->h_cp, h->h_acc};
    for (void* p : pin)
        if (p) (void)hipHostFree(p);
    for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
    if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
    if (h->graph) (void)hipGraphDestroy(h->graph);
    if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
}

template <typename T>
static hipError_t dalloc(T** p, size_t bytes)
{
    return hipMalloc(reinterpret_cast<void**>(p), bytes ? bytes : 16);
}

extern "C" {

int dvc_abi_version(void) { return DVC_ABI_VERSION; }

const char* dvc_last_error(void) { return g_err.c_str(); }

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
    dvc_fd* h = new dvc_fd();
    h->p = p;
    h->device = device;
    h->g.W = p.width;
    h->g.H = p.height;
    h->g.WW = (p.width + 63) / 64;
    h->g.CAP = p.width / 2 + 1;
    if (gauss_taps(p.prime_ksize, p.prime_sigma, h->kprime.t) != 0) {
        delete h;
        return fail(DVC_E_INVALID, "prime blur size %d must be odd, 1..63", p.prime_ksize);
    }
    h->kprime.n = p.prime_ksize;
    dct_matrix(p.block, h->M.m);
    auto bad = [&](hipError_t e, const char* what) {
        int rc = fail(e == hipErrorOutOfMemory ? DVC_E_NOMEM : DVC_E_HIP, "%s: %s", what, hipGetErrorString(e));
        free_all(h);
        delete h;
        return rc;
    };
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return bad(e, "hipSetDevice");
    if (hip_stream) {
        h->stream = (hipStream_t)hip_stream;
    } else {
        e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
        if (e != hipSuccess) return bad(e, "hipStreamCreate");
        h->own_stream = true;
    }
    const size_t W = p.width, H = p.height, N = W * H, WW = h->g.WW, CAP = h->g.CAP;
    struct { void** ptr; size_t bytes; } allocs[] = {
        {(void**)&h->gray[0], N}, {(void**)&h->gray[1], N}, {(void**)&h->acc, N},
        {(void**)&h->mbits, 8 * H * WW}, {(void**)&h->fbits, 8 * H * WW},
        {(void**)&h->rs, 2 * H * CAP}, {(void**)&h->re, 2 * H * CAP}, {(void**)&h->nfg, 4 * H},
        {(void**)&h->fpar, 4 * H * CAP}, {(void**)&h->gpar, 4 * (1 + H * (CAP + 1))},
        {(void**)&h->gE, H * (CAP + 1)}, {(void**)&h->area2, 4 * H * CAP},
        {(void**)&h->stats, 8 * 4},
    };
    for (auto& a : allocs) {
        e = dalloc(a.ptr, a.bytes);
        if (e != hipSuccess) return bad(e, "hipMalloc");
    }
    if (p.flags & DVC_FLAG_KEEP_PLANES) {
        if ((e = dalloc(&h->dbg_kept, 8 * H * WW)) != hipSuccess) return bad(e, "hipMalloc");
        if ((e = dalloc(&h->dbg_dil, 8 * H * WW)) != hipSuccess) return bad(e, "hipMalloc");
    }
    if (!(p.flags & DVC_FLAG_DEVICE_PTRS)) {
        if ((e = dalloc(&h->d_frame, 3 * N)) != hipSuccess) return bad(e, "hipMalloc");
        if ((e = dalloc(&h->d_ov, 3 * N)) != hipSuccess) return bad(e, "hipMalloc");
        if ((e = dalloc(&h->d_cp, 3 * N)) != hipSuccess) return bad(e, "hipMalloc");
        if ((e = hipHostMalloc((void**)&h->h_in, 3 * N)) != hipSuccess) return bad(e, "hipHostMalloc");
        if ((e = hipHostMalloc((void**)&h->h_ov, 3 * N)) != hipSuccess) return bad(e, "hipHostMalloc");
        if ((e = hipHostMalloc((void**)&h->h_cp, 3 * N)) != hipSuccess) return bad(e, "hipHostMalloc");
        if ((e = hipHostMalloc((void**)&h->h_acc, N)) != hipSuccess) return bad(e, "hipHostMalloc");
    }
    if ((e = hipMemsetAsync(h->stats, 0, 32, h->stream)) != hipSuccess) return bad(e, "hipMemset");
    *out = h;
    return DVC_OK;
}

// Stage a host frame (any pitch) into the compact device frame buffer.
static int stage_in(dvc_fd* h, const uint8_t* bgr, size_t pitch, const uint8_t** dptr, int* dpitch)
{
    const size_t W = h->p.width, H = h->p.height;
    if (h->p.flags & DVC_FLAG_DEVICE_PTRS) {
        *dptr = bgr;
        *dpitch = (int)pitch;
        return DVC_OK;
    }
    for (size_t y = 0; y < H; ++y) std::memcpy(h->h_in + y * 3 * W, bgr + y * pitch, 3 * W);
    HIP_OK(hipMemcpyAsync(h->d_frame, h->h_in, 3 * W * H, hipMemcpyHostToDevice, h->stream));
    *dptr = h->d_frame;
    *dpitch = (int)(3 * W);
    return DVC_OK;
}

int dvc_fd_prime(dvc_fd* h, const uint8_t* bgr, size_t pitch)
{
    if (!h || !bgr) return fail(DVC_E_INVALID, "NULL argument");
    if (pitch < 3 * (size_t)h->p.width || pitch % 4) return fail(DVC_E_INVALID, "pitch %zu invalid", pitch);
    HIP_OK(hipSetDevice(h->device));
    const size_t N = (size_t)h->p.width * h->p.height;
    if (!h->tmp32) {
        HIP_OK(dalloc(&h->tmp32, 4 * N));
        HIP_OK(dalloc(&h->gtmp, N));
    }
    const uint8_t* d;
    int dp;
    int rc = stage_in(h, bgr, pitch, &d, &dp);
    if (rc) return rc;
    HIP_OK(dvc::launch_prime(d, dp, h->gtmp, h->tmp32, h->gray[h->cur], h->p.width, h->p.height, h->kprime,
                             h->stream));
    HIP_OK(hipMemsetAsync(h->acc, 0, N, h->stream));
    HIP_OK(hipMemsetAsync(h->stats, 0, 32, h->stream));
    if (!(h->p.flags & DVC_FLAG_DEVICE_PTRS)) HIP_OK(hipStreamSynchronize(h->stream));
    h->frames = 0;
    h->primed = true;
    return DVC_OK;
}

int dvc_fd_step(dvc_fd* h, const uint8_t* bgr, size_t pitch, uint8_t* overlay, uint8_t* compressed,
                uint8_t* acc_out)
{
    if (!h || !bgr) return fail(DVC_E_INVALID, "NULL argument");
    if (!h->primed) return fail(DVC_E_STATE, "dvc_fd_step before dvc_fd_prime");
    if (pitch < 3 * (size_t)h->p.width || pitch % 4) return fail(DVC_E_INVALID, "pitch %zu invalid", pitch);
    HIP_OK(hipSetDevice(h->device));
    const bool devp = h->p.flags & DVC_FLAG_DEVICE_PTRS;
    const size_t W = h->p.width, H = h->p.height, N = W * H;
    const uint8_t* d;
    int dp;
    int rc = stage_in(h, bgr, pitch, &d, &dp);
    if (rc) return rc;
    uint8_t* prev = h->gray[h->cur];
    uint8_t* cur = h->gray[h->cur ^ 1];
    HIP_OK(dvc::launch_front(d, dp, prev, cur, h->mbits, h->g, h->p.ithresh, h->stream));
    dvc::CclBufs c{h->mbits, h->fbits, h->rs, h->re, h->nfg, h->fpar, h->gpar, h->gE, h->area2, h->stats};
    HIP_OK(dvc::launch_ccl(c, h->g, h->stream));
    dvc::BackArgs a{};
    a.g = h->g;
    a.bgr = d;
    a.pitch = dp;
    a.acc = h->acc;
    a.overlay = devp ? overlay : (overlay ? h->d_ov : nullptr);
    a.compressed = devp ? compressed : (compressed ? h->d_cp : nullptr);
    a.opitch = (int)(3 * W);
    a.rs = h->rs;
    a.re = h->re;
    a.nfg = h->nfg;
    a.fpar = h->fpar;
    a.gE = h->gE;
    a.area2 = h->area2;
    a.min_area2 = h->p.min_area2;
    a.ksize = h->p.ksize;
    a.anchor = h->p.anchor;
    a.alpha = h->p.alpha;
    a.beta = h->p.beta;
    a.gamma = h->p.gamma;
    a.quant = h->p.quant;
    a.M = h->M;
    a.stats = h->stats;
    a.dbg_kept = h->dbg_kept;
    a.dbg_dil = h->dbg_dil;
    const bool timed = (h->p.flags & DVC_FLAG_KTIMING) && !h->capturing;
    if (timed) {
        while (h->ev.size() < h->ev_used + 2) {
            hipEvent_t e;
            HIP_OK(hipEventCreate(&e));
            h->ev.push_back(e);
        }
        HIP_OK(hipEventRecord(h->ev[h->ev_used], h->stream));
    }
    HIP_OK(dvc::launch_back(a, h->p.block, h->stream));
    if (timed) {
        HIP_OK(hipEventRecord(h->ev[h->ev_used + 1], h->stream));
        h->ev_used += 2;
    }
    if (acc_out && devp) HIP_OK(hipMemcpyAsync(acc_out, h->acc, N, hipMemcpyDeviceToDevice, h->stream));
    h->cur ^= 1;
    h->frames++;
    if (!devp) {
        if (overlay) HIP_OK(hipMemcpyAsync(h->h_ov, h->d_ov, 3 * N, hipMemcpyDeviceToHost, h->stream));
        if (compressed) HIP_OK(hipMemcpyAsync(h->h_cp, h->d_cp, 3 * N, hipMemcpyDeviceToHost, h->stream));
        if (acc_out) HIP_OK(hipMemcpyAsync(h->h_acc, h->acc, N, hipMemcpyDeviceToHost, h->stream));
        HIP_OK(hipStreamSynchronize(h->stream));
        if (overlay) std::memcpy(overlay, h->h_ov, 3 * N);
        if (compressed) std::memcpy(compressed, h->h_cp, 3 * N);
        if (acc_out) std::memcpy(acc_out, h->h_acc, N);
    }
    return DVC_OK;
}

int dvc_fd_graph_begin(dvc_fd* h)
{
    if (!h) return fail(DVC_E_INVALID, "NULL handle");
    if (!(h->p.flags & DVC_FLAG_DEVICE_PTRS)) return fail(DVC_E_STATE, "graph capture needs DVC_FLAG_DEVICE_PTRS");
    if (!h->primed) return fail(DVC_E_STATE, "graph capture before dvc_fd_prime");
    if (h->capturing) return fail(DVC_E_STATE, "already capturing");
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(hipStreamBeginCapture(h->stream, hipStreamCaptureModeRelaxed));
    h->capturing = true;
    h->cap_cur = h->cur;
    h->cap_frames = h->frames;
    return DVC_OK;
}

int dvc_fd_graph_end(dvc_fd* h)
{
    if (!h || !h->capturing) return fail(DVC_E_STATE, "not capturing");
    HIP_OK(hipSetDevice(h->device));
    hipGraph_t g = nullptr;
    h->capturing = false;
    HIP_OK(hipStreamEndCapture(h->stream, &g));
    uint64_t n = h->frames - h->cap_frames;
    // the captured steps only enqueued work: restore the host-side state
    h->frames = h->cap_frames;
    if (h->cur != h->cap_cur) {
        (void)hipGraphDestroy(g);
        h->cur = h->cap_cur;
        return fail(DVC_E_INVALID, "captured %llu frames: the sequence must be even", (unsigned long long)n);
    }
    if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
    if (h->graph) (void)hipGraphDestroy(h->graph);
    h->graph = g;
    h->gexec = nullptr;
    HIP_OK(hipGraphInstantiate(&h->gexec, g, nullptr, nullptr, 0));
    h->cap_frames = n;
    return DVC_OK;
}

int dvc_fd_graph_launch(dvc_fd* h)
{
    if (!h || !h->gexec) return fail(DVC_E_STATE, "no captured graph");
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(hipGraphLaunch(h->gexec, h->stream));
    h->frames += h->cap_frames;
    return DVC_OK;
}

int dvc_fd_sync(dvc_fd* h)
{
    if (!h) return fail(DVC_E_INVALID, "NULL handle");
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(hipStreamSynchronize(h->stream));
    return DVC_OK;
}

int dvc_fd_get_stats(dvc_fd* h, dvc_fd_stats* out)
{
    if (!h || !out) return fail(DVC_E_INVALID, "NULL argument");
    HIP_OK(hipSetDevice(h->device));
    unsigned long long s[4];
    HIP_OK(hipMemcpyAsync(s, h->stats, sizeof(s), hipMemcpyDeviceToHost, h->stream));
    HIP_OK(hipStreamSynchronize(h->stream));
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
    const size_t W = h->p.width, H = h->p.height, N = W * H, WW = h->g.WW;
    if (plane == DVC_PLANE_GRAY || plane == DVC_PLANE_ACC) {
        HIP_OK(hipMemcpyAsync(dst, plane == DVC_PLANE_GRAY ? h->gray[h->cur] : h->acc, N, hipMemcpyDeviceToHost,
                              h->stream));
        HIP_OK(hipStreamSynchronize(h->stream));
        return DVC_OK;
    }
    const uint64_t* src = plane == DVC_PLANE_MOTION ? h->mbits
                        : plane == DVC_PLANE_FILTERED ? h->dbg_kept
                        : plane == DVC_PLANE_DILATED ? h->dbg_dil : nullptr;
    if (plane != DVC_PLANE_MOTION && plane != DVC_PLANE_FILTERED && plane != DVC_PLANE_DILATED)
        return fail(DVC_E_INVALID, "unknown plane %d", plane);
    if (!src) return fail(DVC_E_STATE, "plane %d needs DVC_FLAG_KEEP_PLANES", plane);
    std::vector<uint64_t> bits(H * WW);
    HIP_OK(hipMemcpyAsync(bits.data(), src, 8 * H * WW, hipMemcpyDeviceToHost, h->stream));
    HIP_OK(hipStreamSynchronize(h->stream));
    for (size_t y = 0; y < H; ++y)
        for (size_t x = 0; x < W; ++x) dst[y * W + x] = ((bits[y * WW + x / 64] >> (x % 64)) & 1) ? 255 : 0;
    return DVC_OK;
}

int dvc_fd_ktime(dvc_fd* h, double* total_ms, uint64_t* launches, int reset)
{
    if (!h) return fail(DVC_E_INVALID, "NULL handle");
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(hipStreamSynchronize(h->stream));
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
    if (h->stream) (void)hipStreamSynchronize(h->stream);
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
    unsigned long long* stats = (unsigned long long*)alloc(32);
    uint8_t* frame = (uint8_t*)alloc(3 * N);
    uint8_t* acc = (uint8_t*)alloc(N);
    int rc = DVC_OK;
    auto done = [&]() { for (void* p : owned) (void)hipFree(p); };
    for (void* p : owned)
        if (!p) { done(); return fail(DVC_E_NOMEM, "hipMalloc failed"); }
    hipStream_t s = nullptr;
    hipError_t e = hipMemcpy(mbits, bits.data(), 8 * H * WW, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(stats, 0, 32);
    if (e == hipSuccess) e = hipMemset(frame, 0, 3 * N);
    if (e == hipSuccess) e = hipMemset(acc, 0, N);
    if (e == hipSuccess) {
        dvc::CclBufs c{mbits, fbits, rs, re, nfg, fpar, gpar, gE, area2, stats};
        e = dvc::launch_ccl(c, g, s);
    }
    if (e == hipSuccess) {
        dvc::BackArgs a{};
        a.g = g; a.bgr = frame; a.pitch = width * 3; a.acc = acc; a.opitch = width * 3;
        a.rs = rs; a.re = re; a.nfg = nfg; a.fpar = fpar; a.gE = gE; a.area2 = area2;
        a.min_area2 = min_area2; a.ksize = 1; a.anchor = 0; a.alpha = 0.5f; a.beta = 0.5f; a.quant = 100.f;
        dct_matrix(4, a.M.m);
        a.stats = stats; a.dbg_kept = kept;
        e = dvc::launch_back(a, 4, s);
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    unsigned long long st[4] = {0, 0, 0, 0};
    if (e == hipSuccess) e = hipMemcpy(bits.data(), kept, 8 * H * WW, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(st, stats, 32, hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = fail(DVC_E_HIP, "contour filter: %s", hipGetErrorString(e));
    done();
    if (rc) return rc;
    for (size_t y = 0; y < H; ++y)
        for (size_t x = 0; x < W; ++x) filtered[y * W + x] = ((bits[y * WW + x / 64] >> (x % 64)) & 1) ? 255 : 0;
    if (components) *components = st[2];
    return DVC_OK;
}

}  // extern "C"
