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

// Contour-filter scratch of one frame in flight.
struct Slot {
    uint64_t *mbits = nullptr, *fbits = nullptr, *kbits = nullptr;
    uint16_t *rs = nullptr, *re = nullptr;
    uint32_t *nfg = nullptr, *fpar = nullptr, *gpar = nullptr, *area2 = nullptr;
    uint8_t* gE = nullptr;
    hipStream_t s_ccl = nullptr;
    hipEvent_t ev_front = nullptr, ev_ccl = nullptr, ev_back = nullptr;
    bool recorded = false;  // ev_ccl / ev_back hold a frame that later frames must wait for
    hipGraphNode_t node_ccl = nullptr, node_back = nullptr;  // graph building: last frame of this slot
};

constexpr int MAX_DEPTH = 8;

struct dvc_fd {
    dvc_fd_params p{};
    int device = 0;
    hipStream_t stream = nullptr;  // the caller's stream: prime, sequential mode, capture origin
    bool own_stream = false;
    dvc::RowGeom g{};
    dvc::GaussTaps kprime{};
    dvc::DctMat M{};
    bool primed = false;
    int cur = 0;                   // gray[cur] = previous blurred gray
    uint64_t frames = 0;
    // pipelining: `depth` frames in flight; front and back chains on their own
    // streams, the contour filter of frame t on slot[t % depth].s_ccl
    int depth = 1;
    uint64_t seq = 0;
    Slot slot[MAX_DEPTH];
    hipStream_t s_front = nullptr, s_back = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join[2 + MAX_DEPTH] = {};
    // device state
    uint8_t* gray[2] = {nullptr, nullptr};
    uint8_t* acc = nullptr;
    uint64_t* dbg_dil = nullptr;
    uint32_t* tmp32 = nullptr;
    uint8_t* gtmp = nullptr;
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
    uint64_t cap_frames = 0, cap_seq = 0;
    hipGraph_t graph = nullptr;
    hipGraphExec_t gexec = nullptr;
    bool eager_dirty = false;  // pipelined eager steps since the last graph launch
    bool graph_dirty = false;  // a graph launch since the last pipelined eager step
    hipStream_t cap_stream = nullptr;  // private stream the stages are captured on
    hipGraphNode_t last_front = nullptr, last_back = nullptr;
};

static void free_all(dvc_fd* h)
{
    for (Slot& s : h->slot) {
        void* dev[] = {s.mbits, s.fbits, s.kbits, s.rs, s.re, s.nfg, s.fpar, s.gpar, s.area2, s.gE};
        for (void* p : dev)
            if (p) (void)hipFree(p);
        for (hipEvent_t e : {s.ev_front, s.ev_ccl, s.ev_back})
            if (e) (void)hipEventDestroy(e);
        if (s.s_ccl && s.s_ccl != h->stream) (void)hipStreamDestroy(s.s_ccl);
    }
    void* dev[] = {h->gray[0], h->gray[1], h->acc, h->dbg_dil, h->tmp32, h->gtmp, h->stats, h->d_frame,
                   h->d_ov, h->d_cp};
    for (void* p : dev)
        if (p) (void)hipFree(p);
    void* pin[] = {h->h_in, h->h_ov, h->h_cp, h->h_acc};
    for (void* p : pin)
        if (p) (void)hipHostFree(p);
    for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
    if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
    for (hipEvent_t e : h->ev_join)
        if (e) (void)hipEventDestroy(e);
    if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
    if (h->graph) (void)hipGraphDestroy(h->graph);
    if (h->cap_stream) (void)hipStreamDestroy(h->cap_stream);
    if (h->s_front && h->s_front != h->stream) (void)hipStreamDestroy(h->s_front);
    if (h->s_back && h->s_back != h->stream) (void)hipStreamDestroy(h->s_back);
    if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
}

template <typename T>
static hipError_t dalloc(T** p, size_t bytes)
{
    return hipMalloc(reinterpret_cast<void**>(p), bytes ? bytes : 16);
}

// every stream the handle may have work on
static int all_streams(dvc_fd* h, hipStream_t* out)
{
    int n = 0;
    out[n++] = h->stream;
    if (h->depth > 1) {
        out[n++] = h->s_front;
        out[n++] = h->s_back;
        for (int i = 0; i < h->depth; ++i) out[n++] = h->slot[i].s_ccl;
    }
    return n;
}

static hipError_t sync_all(dvc_fd* h)
{
    hipStream_t s[2 + MAX_DEPTH];
    int n = all_streams(h, s);
    for (int i = 0; i < n; ++i) {
        hipError_t e = hipStreamSynchronize(s[i]);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
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
    const int depth = p.pipeline <= 1 ? 1 : (int)p.pipeline;
    if (depth > MAX_DEPTH) return fail(DVC_E_INVALID, "pipeline depth %d outside 1..%d", depth, MAX_DEPTH);
    if (depth > 1 && !(p.flags & DVC_FLAG_DEVICE_PTRS))
        return fail(DVC_E_INVALID, "a pipeline depth > 1 needs DVC_FLAG_DEVICE_PTRS");
    dvc_fd* h = new dvc_fd();
    h->p = p;
    h->device = device;
    h->depth = depth;
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
    for (int i = 0; i < depth; ++i) {
        Slot& s = h->slot[i];
        struct { void** ptr; size_t bytes; } allocs[] = {
            {(void**)&s.mbits, 8 * H * WW}, {(void**)&s.fbits, 8 * H * WW}, {(void**)&s.kbits, 8 * H * WW},
            {(void**)&s.rs, 2 * H * CAP}, {(void**)&s.re, 2 * H * CAP}, {(void**)&s.nfg, 4 * H},
            {(void**)&s.fpar, 4 * H * CAP}, {(void**)&s.gpar, 4 * (1 + H * (CAP + 1))},
            {(void**)&s.gE, H * (CAP + 1)}, {(void**)&s.area2, 4 * H * CAP},
        };
        for (auto& a : allocs)
            if ((e = dalloc(a.ptr, a.bytes)) != hipSuccess) return bad(e, "hipMalloc");
        if (depth > 1) {
            if ((e = hipStreamCreateWithFlags(&s.s_ccl, hipStreamNonBlocking)) != hipSuccess)
                return bad(e, "hipStreamCreate");
            for (hipEvent_t* ev : {&s.ev_front, &s.ev_ccl, &s.ev_back})
                if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess)
                    return bad(e, "hipEventCreate");
        } else {
            s.s_ccl = h->stream;
        }
    }
    if (depth > 1) {
        for (hipStream_t* st : {&h->s_front, &h->s_back})
            if ((e = hipStreamCreateWithFlags(st, hipStreamNonBlocking)) != hipSuccess) return bad(e, "hipStreamCreate");
        if ((e = hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming)) != hipSuccess)
            return bad(e, "hipEventCreate");
        for (hipEvent_t& ev : h->ev_join)
            if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    } else {
        h->s_front = h->s_back = h->stream;
    }
    struct { void** ptr; size_t bytes; } allocs[] = {
        {(void**)&h->gray[0], N}, {(void**)&h->gray[1], N}, {(void**)&h->acc, N}, {(void**)&h->stats, 8 * 4 * 64},
    };
    for (auto& a : allocs)
        if ((e = dalloc(a.ptr, a.bytes)) != hipSuccess) return bad(e, "hipMalloc");
    if (p.flags & DVC_FLAG_KEEP_PLANES) {
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
    if ((e = hipMemsetAsync(h->stats, 0, 8 * 4 * 64, h->stream)) != hipSuccess) return bad(e, "hipMemset");
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
    if (h->capturing) return fail(DVC_E_STATE, "prime during graph capture");
    if (pitch < 3 * (size_t)h->p.width || pitch % 4) return fail(DVC_E_INVALID, "pitch %zu invalid", pitch);
    HIP_OK(hipSetDevice(h->device));
    const size_t N = (size_t)h->p.width * h->p.height;
    if (!h->tmp32) {
        HIP_OK(dalloc(&h->tmp32, 4 * N));
        HIP_OK(dalloc(&h->gtmp, N));
    }
    HIP_OK(sync_all(h));  // no frame of a previous run may still be in flight
    const uint8_t* d;
    int dp;
    int rc = stage_in(h, bgr, pitch, &d, &dp);
    if (rc) return rc;
    HIP_OK(dvc::launch_prime(d, dp, h->gtmp, h->tmp32, h->gray[h->cur], h->p.width, h->p.height, h->kprime,
                             h->stream));
    HIP_OK(hipMemsetAsync(h->acc, 0, N, h->stream));
    HIP_OK(hipMemsetAsync(h->stats, 0, 8 * 4 * 64, h->stream));
    if (!(h->p.flags & DVC_FLAG_DEVICE_PTRS) || h->depth > 1) HIP_OK(hipStreamSynchronize(h->stream));
    for (Slot& s : h->slot) s.recorded = false;
    h->frames = 0;
    h->seq = 0;
    h->primed = true;
    return DVC_OK;
}

}  // extern "C"

// The three stages of one frame, each enqueued on one stream.
static hipError_t stage_front(dvc_fd* h, Slot& S, const uint8_t* d, int dp, hipStream_t s)
{
    return dvc::launch_front(d, dp, h->gray[h->cur], h->gray[h->cur ^ 1], S.mbits, h->g, h->p.ithresh, s);
}

static hipError_t stage_ccl(dvc_fd* h, Slot& S, hipStream_t s)
{
    dvc::CclBufs c{S.mbits, S.fbits, S.rs, S.re, S.nfg, S.fpar, S.gpar, S.gE, S.area2, S.kbits, h->stats};
    return dvc::launch_ccl(c, h->g, h->p.min_area2, s);
}

static dvc::BackArgs back_args(dvc_fd* h, Slot& S, const uint8_t* d, int dp, uint8_t* ov, uint8_t* cp)
{
    dvc::BackArgs a{};
    a.g = h->g;
    a.bgr = d;
    a.pitch = dp;
    a.acc = h->acc;
    a.overlay = ov;
    a.compressed = cp;
    a.opitch = 3 * h->p.width;
    a.kbits = S.kbits;
    a.ksize = h->p.ksize;
    a.anchor = h->p.anchor;
    a.alpha = h->p.alpha;
    a.beta = h->p.beta;
    a.gamma = h->p.gamma;
    a.quant = h->p.quant;
    a.M = h->M;
    a.stats = h->stats;
    a.dbg_dil = h->dbg_dil;
    return a;
}

// Graph building: capture one stage on the private capture stream and add it as
// a child-graph node that depends on `deps` (single-stream captures only).
template <typename F>
static int add_stage_node(dvc_fd* h, F&& enqueue, const hipGraphNode_t* deps, size_t ndeps, hipGraphNode_t* node)
{
    hipGraph_t child = nullptr;
    HIP_OK(hipStreamBeginCapture(h->cap_stream, hipStreamCaptureModeRelaxed));
    hipError_t e = enqueue(h->cap_stream);
    hipError_t e2 = hipStreamEndCapture(h->cap_stream, &child);
    if (e != hipSuccess) {
        if (child) (void)hipGraphDestroy(child);
        return fail(DVC_E_HIP, "stage capture: %s", hipGetErrorString(e));
    }
    HIP_OK(e2);
    hipError_t e3 = hipGraphAddChildGraphNode(node, h->graph, deps, ndeps, child);
    (void)hipGraphDestroy(child);
    HIP_OK(e3);
    return DVC_OK;
}

extern "C" {

int dvc_fd_step(dvc_fd* h, const uint8_t* bgr, size_t pitch, uint8_t* overlay, uint8_t* compressed,
                uint8_t* acc_out)
{
    if (!h || !bgr) return fail(DVC_E_INVALID, "NULL argument");
    if (!h->primed) return fail(DVC_E_STATE, "dvc_fd_step before dvc_fd_prime");
    if (pitch < 3 * (size_t)h->p.width || pitch % 4) return fail(DVC_E_INVALID, "pitch %zu invalid", pitch);
    HIP_OK(hipSetDevice(h->device));
    const bool devp = h->p.flags & DVC_FLAG_DEVICE_PTRS;
    const bool pipe = h->depth > 1;
    const size_t W = h->p.width, H = h->p.height, N = W * H;
    const uint8_t* d;
    int dp;
    int rc = stage_in(h, bgr, pitch, &d, &dp);
    if (rc) return rc;
    Slot& S = h->slot[h->seq % h->depth];
    dvc::BackArgs a = back_args(h, S, d, dp, devp ? overlay : (overlay ? h->d_ov : nullptr),
                                devp ? compressed : (compressed ? h->d_cp : nullptr));

    if (h->capturing) {
        // frame t = graph nodes F_t, C_t, B_t with the edges of the pipeline:
        //   F_t <- F_{t-1} (gray chain), C_{t-D} (mask slot reuse)
        //   C_t <- F_t, B_{t-D} (kept-mask slot reuse)
        //   B_t <- C_t, B_{t-1} (accumulated-mask chain)
        if (acc_out) return fail(DVC_E_UNSUPPORTED, "acc_out is not captured into graphs");
        hipGraphNode_t deps[2];
        size_t nd = 0;
        if (h->last_front) deps[nd++] = h->last_front;
        if (S.node_ccl) deps[nd++] = S.node_ccl;
        hipGraphNode_t nf, nc, nb;
        rc = add_stage_node(h, [&](hipStream_t s) { return stage_front(h, S, d, dp, s); }, deps, nd, &nf);
        if (rc) return rc;
        nd = 0;
        deps[nd++] = nf;
        if (S.node_back) deps[nd++] = S.node_back;
        rc = add_stage_node(h, [&](hipStream_t s) { return stage_ccl(h, S, s); }, deps, nd, &nc);
        if (rc) return rc;
        nd = 0;
        deps[nd++] = nc;
        if (h->last_back) deps[nd++] = h->last_back;
        rc = add_stage_node(h, [&](hipStream_t s) { return dvc::launch_back(a, h->p.block, s); }, deps, nd, &nb);
        if (rc) return rc;
        h->last_front = nf;
        h->last_back = nb;
        S.node_ccl = nc;
        S.node_back = nb;
        h->cur ^= 1;
        h->frames++;
        h->seq++;
        return DVC_OK;
    }

    if (pipe) {
        if (h->graph_dirty) {  // order after the replayed graph on the origin stream
            HIP_OK(hipEventRecord(h->ev_fork, h->stream));
            hipStream_t s[2 + MAX_DEPTH];
            int n = all_streams(h, s);
            for (int i = 1; i < n; ++i) HIP_OK(hipStreamWaitEvent(s[i], h->ev_fork, 0));
            h->graph_dirty = false;
        }
        h->eager_dirty = true;
    }
    // front(t): its mask slot must have been released by the contour filter of frame t - depth
    if (pipe && S.recorded) HIP_OK(hipStreamWaitEvent(h->s_front, S.ev_ccl, 0));
    HIP_OK(stage_front(h, S, d, dp, h->s_front));
    if (pipe) {
        HIP_OK(hipEventRecord(S.ev_front, h->s_front));
        // contour filter(t): after front(t), and after back(t - depth) released the kept mask
        HIP_OK(hipStreamWaitEvent(S.s_ccl, S.ev_front, 0));
        if (S.recorded) HIP_OK(hipStreamWaitEvent(S.s_ccl, S.ev_back, 0));
    }
    HIP_OK(stage_ccl(h, S, S.s_ccl));
    if (pipe) {
        HIP_OK(hipEventRecord(S.ev_ccl, S.s_ccl));
        HIP_OK(hipStreamWaitEvent(h->s_back, S.ev_ccl, 0));
    }
    // back(t): after the contour filter of t; the back chain is ordered on s_back (acc)
    const bool timed = h->p.flags & DVC_FLAG_KTIMING;
    if (timed) {
        while (h->ev.size() < h->ev_used + 2) {
            hipEvent_t e;
            HIP_OK(hipEventCreate(&e));
            h->ev.push_back(e);
        }
        HIP_OK(hipEventRecord(h->ev[h->ev_used], h->s_back));
    }
    HIP_OK(dvc::launch_back(a, h->p.block, h->s_back));
    if (timed) {
        HIP_OK(hipEventRecord(h->ev[h->ev_used + 1], h->s_back));
        h->ev_used += 2;
    }
    if (pipe) HIP_OK(hipEventRecord(S.ev_back, h->s_back));
    S.recorded = true;
    if (acc_out && devp) HIP_OK(hipMemcpyAsync(acc_out, h->acc, N, hipMemcpyDeviceToDevice, h->s_back));
    h->cur ^= 1;
    h->frames++;
    h->seq++;
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
    // earlier eager frames must be complete: the graph waits on nothing outside itself
    HIP_OK(sync_all(h));
    h->eager_dirty = false;
    if (!h->cap_stream) HIP_OK(hipStreamCreateWithFlags(&h->cap_stream, hipStreamNonBlocking));
    if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
    if (h->graph) (void)hipGraphDestroy(h->graph);
    h->gexec = nullptr;
    h->graph = nullptr;
    HIP_OK(hipGraphCreate(&h->graph, 0));
    h->last_front = h->last_back = nullptr;
    for (Slot& s : h->slot) {
        s.node_ccl = s.node_back = nullptr;
        s.recorded = false;
    }
    h->capturing = true;
    h->cap_cur = h->cur;
    h->cap_frames = h->frames;
    h->cap_seq = h->seq;
    return DVC_OK;
}

int dvc_fd_graph_end(dvc_fd* h)
{
    if (!h || !h->capturing) return fail(DVC_E_STATE, "not capturing");
    HIP_OK(hipSetDevice(h->device));
    h->capturing = false;
    uint64_t n = h->frames - h->cap_frames;
    // building the graph only recorded work: restore the host-side state
    h->frames = h->cap_frames;
    const bool ok = n > 0 && h->cur == h->cap_cur && n % (uint64_t)h->depth == 0;
    h->cur = h->cap_cur;
    h->seq = h->cap_seq;
    if (!ok) {
        (void)hipGraphDestroy(h->graph);
        h->graph = nullptr;
        return fail(DVC_E_INVALID, "graph of %llu frames: must be a nonzero multiple of 2 and of the pipeline "
                    "depth %d", (unsigned long long)n, h->depth);
    }
    HIP_OK(hipGraphInstantiate(&h->gexec, h->graph, nullptr, nullptr, 0));
    h->cap_frames = n;
    return DVC_OK;
}

int dvc_fd_graph_launch(dvc_fd* h)
{
    if (!h || !h->gexec) return fail(DVC_E_STATE, "no captured graph");
    HIP_OK(hipSetDevice(h->device));
    if (h->eager_dirty) {  // eager steps on the internal streams must finish first
        HIP_OK(sync_all(h));
        h->eager_dirty = false;
    }
    HIP_OK(hipGraphLaunch(h->gexec, h->stream));
    h->graph_dirty = h->depth > 1;
    for (Slot& s : h->slot) s.recorded = false;
    h->frames += h->cap_frames;
    return DVC_OK;
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
        HIP_OK(hipMemcpy(dst, plane == DVC_PLANE_GRAY ? h->gray[h->cur] : h->acc, N, hipMemcpyDeviceToHost));
        return DVC_OK;
    }
    const Slot& S = h->slot[(h->seq + h->depth - 1) % h->depth];  // the last stepped frame
    const uint64_t* src = plane == DVC_PLANE_MOTION ? S.mbits
                        : plane == DVC_PLANE_FILTERED ? S.kbits
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
    if (e == hipSuccess) {
        dvc::CclBufs c{mbits, fbits, rs, re, nfg, fpar, gpar, gE, area2, kept, stats};
        e = dvc::launch_ccl(c, g, min_area2, s);
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
