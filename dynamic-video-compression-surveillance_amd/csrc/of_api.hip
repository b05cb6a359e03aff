// of_api.hip — the C-ABI (include/dvc.h, dvc_of_*) of the optical-flow worker.
//
// Host side of one camera feed of motion_compression_opt.py: the state the
// reference keeps in Python locals (prev_gray of:60,101; mask_queue of:61,84)
// lives on the device as per-level polynomial-expansion rings, the raw-mask
// ring and the per-pixel vote counts. The per-level geometry (pyramid sizes,
// smoothing kernels, INTER_LINEAR tables, FarnebackPrepareGaussian) is derived
// here with the same expressions as oracle/of_oracle.c.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <cstdio>

#include <cfloat>
#include <cmath>
#include <cstring>
#include <algorithm>
#include <vector>

#include "../../include/dvc.h"
#include "host_common.h"
#include "yuv_kernels.h"
#include "of_kernels.h"
#include "tune.h"

using dvc_host::fail;

namespace {

// FarnebackPrepareGaussian (optflowgf.cpp; oc_poly_gauss): float taps, and the
// needed entries of the inverse moment matrix (Cholesky, double).
void poly_coef(int n, double sigma, dvc::PolyCoef& pc)
{
    float g[2 * dvc::OF_MAX_POLY_N + 1], xg[2 * dvc::OF_MAX_POLY_N + 1], xxg[2 * dvc::OF_MAX_POLY_N + 1];
    if (sigma < FLT_EPSILON) sigma = n * 0.3;
    double s = 0.;
    for (int x = -n; x <= n; ++x) {
        g[x + n] = (float)std::exp(-x * x / (2 * sigma * sigma));
        s += g[x + n];
    }
    s = 1. / s;
    for (int x = -n; x <= n; ++x) {
        g[x + n] = (float)(g[x + n] * s);
        xg[x + n] = (float)(x * g[x + n]);
        xxg[x + n] = (float)(x * x * g[x + n]);
    }
    double G[6][6];
    std::memset(G, 0, sizeof(G));
    for (int y = -n; y <= n; ++y)
        for (int x = -n; x <= n; ++x) {
            G[0][0] += g[y + n] * g[x + n];
            G[1][1] += g[y + n] * g[x + n] * x * x;
            G[3][3] += g[y + n] * g[x + n] * x * x * x * x;
            G[5][5] += g[y + n] * g[x + n] * x * x * y * y;
        }
    G[2][2] = G[0][3] = G[0][4] = G[3][0] = G[4][0] = G[1][1];
    G[4][4] = G[3][3];
    G[3][4] = G[4][3] = G[5][5];
    double L[6][6];
    std::memset(L, 0, sizeof(L));
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j <= i; ++j) {
            double v = G[i][j];
            for (int k = 0; k < j; ++k) v -= L[i][k] * L[j][k];
            L[i][j] = (i == j) ? std::sqrt(v) : v / L[j][j];
        }
    double inv[6][6];
    for (int c = 0; c < 6; ++c) {
        double z[6], xv[6];
        for (int i = 0; i < 6; ++i) {
            double v = (i == c) ? 1.0 : 0.0;
            for (int k = 0; k < i; ++k) v -= L[i][k] * z[k];
            z[i] = v / L[i][i];
        }
        for (int i = 5; i >= 0; --i) {
            double v = z[i];
            for (int k = i + 1; k < 6; ++k) v -= L[k][i] * xv[k];
            xv[i] = v / L[i][i];
        }
        for (int i = 0; i < 6; ++i) inv[i][c] = xv[i];
    }
    pc.n = n;
    for (int i = 0; i < 2 * n + 1; ++i) {
        pc.g[i] = g[i];
        pc.xg[i] = xg[i];
        pc.xxg[i] = xxg[i];
    }
    pc.ig11 = inv[1][1];
    pc.ig03 = inv[0][3];
    pc.ig33 = inv[3][3];
    pc.ig55 = inv[5][5];
}

// INTER_LINEAR source taps of a resize sw -> dw (oc_resize_linear_f32, one axis).
void lin_taps(int sw, int dw, std::vector<dvc::LinTap>& out)
{
    out.resize(dw);
    const double sc = (double)sw / dw;
    for (int d = 0; d < dw; ++d) {
        float f = (float)((d + 0.5) * sc - 0.5);
        int s = (int)std::floor(f);
        f -= (float)s;
        if (s < 0) { f = 0.f; s = 0; }
        if (s >= sw - 1) { f = 0.f; s = sw - 1; }
        const int s1 = s + 1 < sw ? s + 1 : sw - 1;
        out[d] = dvc::LinTap{s, s1, 1.f - f, f};
    }
}

// getStructuringElement(MORPH_ELLIPSE, (k, k)) (of:62; oc_ellipse_element) as
// per-row column ranges relative to the anchor (k/2, k/2): row i covers
// dx = mlo[i] .. mhi[i] (mlo > mhi: empty row).
void ellipse_rows(int k, dvc::OfGeom& g)
{
    const int r = k / 2, c = k / 2;
    const double inv_r2 = r ? 1. / ((double)r * r) : 0;
    g.mk = k;
    for (int i = 0; i < k; ++i) {
        const int dy = i - r;
        int j1 = 0, j2 = 0;
        if (std::abs(dy) <= r) {
            const int dx = (int)std::lrint(c * std::sqrt((r * r - dy * dy) * inv_r2));
            j1 = std::max(c - dx, 0);
            j2 = std::min(c + dx + 1, k);
        }
        g.mlo[i] = (int8_t)(j1 < j2 ? j1 - c : 1);
        g.mhi[i] = (int8_t)(j1 < j2 ? j2 - 1 - c : 0);
    }
}

// smallest c with c*255 >= alpha*L*255 in float64 (of:86; oc_vote_threshold)
int vote_threshold(double alpha, int L)
{
    const double thr = alpha * L * 255;
    int c = 0;
    while (c <= L && !((double)(c * 255) >= thr)) ++c;
    return c;
}

}  // namespace

// Events of one batch in flight; two slots alternate (batch i waits on i-2).
struct OfSlot {
    hipEvent_t ev_pyr = nullptr, ev_flow = nullptr, ev_mask = nullptr;
    hipEvent_t ev_l1 = nullptr, ev_l0a = nullptr;   // flow: coarse levels done / level 0's first iteration done
    bool recorded = false;
    uint8_t* fin = nullptr;   // staged input: YUV frames converted to BGR, or BGR frames the kernels
                              // cannot read in place, re-pitched (rows of ip), read by the pyramid
                              // and by k_of_out
};

struct dvc_of {
    dvc_of_params p{};
    int device = 0;
    hipStream_t stream = nullptr;  // prime + pyramid stage (s_pyr), internal
    hipStream_t user = nullptr;    // the caller's stream (create's hip_stream; NULL = legacy default)
    bool has_user = false;         // join `user` (hip_stream given, or DVC_FLAG_JOIN_STREAM)
    hipEvent_t ev_user = nullptr, ev_join = nullptr;
    // batch i: s_pyr [wait flow(i-2)] pyramid(i); s_flow [wait pyramid(i),
    // mask(i-2)] flow(i); s_mask [wait flow(i)] vote/morphology/rects + out(i)
    hipStream_t s_pyr = nullptr, s_flow = nullptr, s_mask = nullptr;
    // pyramid levels 2..L beside level 1 (of_launch_pyramid) on s_flow, idle
    // while the batch's pyramid is built (its flow waits for it); the fork /
    // join events. (A fifth stream would share one of the 4 hardware queues
    // with another stage and serialise it: measured, experiments/README.md.)
    hipEvent_t ev_gray = nullptr, ev_side = nullptr;
    OfSlot slot[2];
    uint64_t seq = 0;
    dvc::OfGeom g{};
    dvc::Level lv[dvc::OF_MAX_LEVELS]{};
    dvc::OfBufs b{};
    dvc::DctMat M{};
    int max_batch = 1;
    int ip = 0;                          // row pitch the kernels read BGR frames with: 3 * roundup(W, 4)
    int fmt = DVC_FMT_BGR, crows = 0;   // frame format handed to prime/step (DVC_FMT_*)
    long long a_next = 1;
    bool primed = false;
    uint64_t frames = 0;
    int last_n = 0;
    std::vector<void*> dev;  // every device allocation
    uint8_t *d_in = nullptr, *d_mask = nullptr, *d_cp = nullptr;
    uint8_t *h_in = nullptr, *h_mask = nullptr, *h_cp = nullptr;
    std::vector<hipEvent_t> ev;
    size_t ev_used = 0;
    unsigned int epoch = 0;   // k_flow_scan launches so far (hand-off flags carry it)
    int l0_kernel = -1;       // the level-0 flow kernel of the last batch (DVC_KTIME_FLOW*)
    // DVC_OF_FAULT=scan_abort at create (fault injection, tests/test_of_gpu.py):
    // every batch starts with the scan hand-off's abort flag raised, so each
    // strip that polls fails at once and the launch drains; the next sync
    // reports the error (the path a hand-off timeout takes)
    bool fault_abort = false;
};

static void of_free(dvc_of* h)
{
    for (void* p : h->dev)
        if (p) (void)hipFree(p);
    h->dev.clear();
    for (void* p : {(void*)h->h_in, (void*)h->h_mask, (void*)h->h_cp})
        if (p) (void)hipHostFree(p);
    for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
    for (OfSlot& sl : h->slot)
        for (hipEvent_t e : {sl.ev_pyr, sl.ev_flow, sl.ev_mask, sl.ev_l1, sl.ev_l0a})
            if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : {h->ev_user, h->ev_join, h->ev_gray, h->ev_side})
        if (e) (void)hipEventDestroy(e);
    for (hipStream_t st : {h->s_flow, h->s_mask, h->stream})
        if (st) (void)hipStreamDestroy(st);
}

// The caller's stream (if any) -> the internal streams, before a call's work;
// the internal streams -> the caller's stream after it (outputs on s_mask).
static hipError_t of_wait_user(dvc_of* h)
{
    if (!h->has_user) return hipSuccess;
    hipError_t e = hipEventRecord(h->ev_user, h->user);
    for (hipStream_t st : {h->stream, h->s_flow, h->s_mask})
        if (e == hipSuccess) e = hipStreamWaitEvent(st, h->ev_user, 0);
    return e;
}

static hipError_t of_join_user(dvc_of* h)
{
    if (!h->has_user) return hipSuccess;
    hipError_t e = hipEventRecord(h->ev_join, h->s_mask);
    if (e == hipSuccess) e = hipStreamWaitEvent(h->user, h->ev_join, 0);
    return e;
}

static hipError_t of_sync_all(dvc_of* h)
{
    hipError_t e = hipStreamSynchronize(h->stream);
    for (hipStream_t st : {h->s_flow, h->s_mask})
        if (e == hipSuccess && st) e = hipStreamSynchronize(st);
    return e;
}

// After a sync: did a k_flow_scan hand-off wait time out? (never in a correct run)
static int of_check_abort(dvc_of* h)
{
    unsigned int ab = 0;
    HIP_OK(hipMemcpy(&ab, h->b.scan_abort, 4, hipMemcpyDeviceToHost));
    if (ab) return fail(DVC_E_HIP, "k_flow_scan: a strip hand-off wait timed out");
    return DVC_OK;
}

template <typename T>
static hipError_t of_alloc(dvc_of* h, T** p, size_t bytes)
{
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, bytes ? bytes : 16);
    if (e == hipSuccess) {
        h->dev.push_back(q);
        *p = reinterpret_cast<T*>(q);
    }
    return e;
}

extern "C" {

// Frames handed to prime/step: BGR rows of `pitch` (>= 3W), or 4:2:0
// surfaces (luma pitch >= W; I420: even).
static bool of_pitch_ok(const dvc_of* h, size_t pitch)
{
    const size_t W = h->p.width;
    if (h->fmt == DVC_FMT_BGR) return pitch >= 3 * W;
    return pitch >= W && (h->fmt != DVC_FMT_I420 || pitch % 2 == 0);
}

// Can the kernels read these BGR device frames in place? Dword rows reaching
// whole 4-px quads (3 * roundup(W, 4) bytes), aligned base and frame stride;
// anything else is re-pitched into the slot's staging frames first. W % 4 == 0:
// a frame's last row then ends exactly at its last quad, so a buffer sized to
// the frame span (pitch * (H - 1) + 3W, what the step checks) is never read
// past its end.
static bool of_direct(const dvc_of* h, const uint8_t* p, size_t pitch, size_t fstride, int n)
{
    return h->p.width % 4 == 0 && pitch % 4 == 0 && pitch >= (size_t)h->ip && ((uintptr_t)p & 3) == 0 &&
           (n <= 1 || fstride % 4 == 0);
}

// Can k_of_front0 / k_of_out read these 4:2:0 surfaces in place? Dword luma
// rows (pitch % 4 == 0, so rows reach whole quads), aligned base and stride,
// W % 4 == 0 (the last luma and chroma rows end at a whole quad's bytes).
// DVC_OF_YUV_DIRECT=0 forces the staged conversion (A/B).
static bool of_direct_yuv(const dvc_of* h, const uint8_t* p, size_t pitch, size_t fstride, int n)
{
    static const int on = [] { const char* e = dvc::tune_env("DVC_OF_YUV_DIRECT"); return e ? atoi(e) : 1; }();
    return on && h->p.width % 4 == 0 && pitch % 4 == 0 && ((uintptr_t)p & 3) == 0 && (n <= 1 || fstride % 4 == 0);
}

// The frames the kernels read for a batch in slot S: the caller's device
// frames in place (BGR rows the kernels can read, or 4:2:0 surfaces converted
// per pixel as they load: *sf says which), or (re-pitch needed, surfaces not
// readable in place) converted / copied into S.fin on stream `st` once the
// slot's previous batch is done with it.
static int of_stage(dvc_of* h, OfSlot& S, const uint8_t* d, int dp, size_t fstride, int n, int crows, hipStream_t st,
                    const uint8_t** kd, int* kp, size_t* kfs, dvc::SrcFmt* sf)
{
    const size_t W = h->p.width, H = h->p.height, FS = (size_t)h->ip * H;
    *sf = dvc::SrcFmt{DVC_FMT_BGR, 0, 0, 0};
    if (h->fmt == DVC_FMT_BGR && of_direct(h, d, (size_t)dp, fstride, n)) {
        *kd = d;
        *kp = dp;
        *kfs = fstride;
        return DVC_OK;
    }
    if (h->fmt != DVC_FMT_BGR && of_direct_yuv(h, d, (size_t)dp, fstride, n)) {
        const dvc::YuvLayout L = dvc::yuv_layout(d, dp, h->fmt, crows, fstride);
        *sf = dvc::SrcFmt{h->fmt, L.uoff, L.voff, L.cpitch};
        *kd = d;
        *kp = dp;
        *kfs = fstride;
        return DVC_OK;
    }
    if (!S.fin) HIP_OK(of_alloc(h, &S.fin, FS * h->max_batch));
    if (S.recorded) HIP_OK(hipStreamWaitEvent(st, S.ev_mask, 0));   // batch i-2's k_of_out read S.fin
    if (h->fmt != DVC_FMT_BGR) {   // cvtColor of the decoded surfaces (what cap.read() returns, of:54,66)
        HIP_OK(dvc::launch_yuv420_to_bgr(dvc::yuv_layout(d, dp, h->fmt, crows, fstride), (int)W, (int)H, n, S.fin,
                                         h->ip, FS, st));
    } else if (n == 1 || fstride == (size_t)dp * H) {
        HIP_OK(hipMemcpy2DAsync(S.fin, h->ip, d, dp, 3 * W, H * n, hipMemcpyDeviceToDevice, st));
    } else {
        for (int t = 0; t < n; ++t)
            HIP_OK(hipMemcpy2DAsync(S.fin + t * FS, h->ip, d + t * fstride, dp, 3 * W, H, hipMemcpyDeviceToDevice, st));
    }
    *kd = S.fin;
    *kp = h->ip;
    *kfs = FS;
    return DVC_OK;
}

static size_t of_frame_span(const dvc_of* h, size_t pitch)
{
    if (h->fmt == DVC_FMT_BGR) return pitch * (h->p.height - 1) + 3 * (size_t)h->p.width;
    return dvc::yuv_frame_bytes(pitch, h->crows);
}

// A host frame into pinned staging in the layout the device copy is read with
// (BGR rows of ip; YUV: luma rows of W and the chroma plane(s) right after).
static void of_pack_host(const dvc_of* h, const uint8_t* src, size_t pitch, uint8_t* dst)
{
    const size_t W = h->p.width, H = h->p.height;
    if (h->fmt == DVC_FMT_BGR) {
        for (size_t y = 0; y < H; ++y) std::memcpy(dst + y * h->ip, src + y * pitch, 3 * W);
        return;
    }
    const dvc::YuvLayout L = dvc::yuv_layout(src, pitch, h->fmt, h->crows, 0);
    const dvc::YuvLayout C = dvc::yuv_layout(dst, W, h->fmt, (int)H, 0);
    for (size_t y = 0; y < H; ++y) std::memcpy(dst + y * W, src + y * pitch, W);
    const size_t cb = h->fmt == DVC_FMT_NV12 ? W : W / 2;
    for (size_t y = 0; y < H / 2; ++y) {
        std::memcpy(dst + C.uoff + y * C.cpitch, src + L.uoff + y * L.cpitch, cb);
        if (h->fmt == DVC_FMT_I420) std::memcpy(dst + C.voff + y * C.cpitch, src + L.voff + y * L.cpitch, cb);
    }
}

int dvc_of_create(const dvc_of_params* prm, int device, void* hip_stream, dvc_of** out)
{
    if (!prm || !out) return fail(DVC_E_INVALID, "NULL argument");
    const dvc_of_params& p = *prm;
    if (p.width < 8 || p.height < 8 || p.width > 65520)
        return fail(DVC_E_INVALID, "frame %dx%d outside 8..65520 x >=8", p.width, p.height);
    if (p.morph_kernel < 1 || p.morph_kernel > dvc::OF_MAX_MORPH)
        return fail(DVC_E_UNSUPPORTED, "morph_kernel %d outside 1..%d", p.morph_kernel, dvc::OF_MAX_MORPH);
    if (p.window < 1 || p.window > 255) return fail(DVC_E_UNSUPPORTED, "window_size %d outside 1..255", p.window);
    if (p.poly_n != 5 && p.poly_n != 7) return fail(DVC_E_UNSUPPORTED, "poly_n %d: 5 or 7", p.poly_n);
    if (p.winsize < 1 || p.winsize / 2 > dvc::OF_MAX_BOX_M)
        return fail(DVC_E_UNSUPPORTED, "winsize %d outside 1..%d", p.winsize, 2 * dvc::OF_MAX_BOX_M + 1);
    if (p.iterations < 1) return fail(DVC_E_INVALID, "iterations must be >= 1");
    if (!(p.pyr_scale > 0 && p.pyr_scale < 1)) return fail(DVC_E_INVALID, "pyr_scale must be in (0, 1)");
    if (p.levels < 0) return fail(DVC_E_INVALID, "levels must be >= 0");
    if (!(p.quant == p.quant) || p.quant == 0.0f) return fail(DVC_E_INVALID, "quant must be nonzero");
    if (p.max_batch > DVC_MAX_BATCH) return fail(DVC_E_INVALID, "max_batch %u outside 1..%d", p.max_batch, DVC_MAX_BATCH);
    if (p.in_format != DVC_FMT_BGR && p.in_format != DVC_FMT_I420 && p.in_format != DVC_FMT_NV12)
        return fail(DVC_E_INVALID, "in_format %d unknown", p.in_format);
    if (p.in_format != DVC_FMT_BGR && p.chroma_rows && (p.chroma_rows < p.height || (p.chroma_rows & 1)))
        return fail(DVC_E_INVALID, "chroma_rows %d: even and >= the frame height %d", p.chroma_rows, p.height);
    // pyramid depth (oc_fb_levels: min size 32)
    int L = 0;
    {
        double scale = 1;
        for (L = 0; L < p.levels; ++L) {
            scale *= p.pyr_scale;
            if (p.width * scale < 32 || p.height * scale < 32) break;
        }
    }
    if (L >= dvc::OF_MAX_LEVELS) return fail(DVC_E_UNSUPPORTED, "%d pyramid levels (max %d)", L + 1, dvc::OF_MAX_LEVELS);

    dvc_of* h = new dvc_of();
    h->p = p;
    h->device = device;
    h->max_batch = p.max_batch == 0 ? 1 : (int)p.max_batch;
    h->fmt = p.in_format;
    h->crows = p.chroma_rows ? p.chroma_rows : p.height;
    const int mb = h->max_batch;
    dvc::OfGeom& g = h->g;
    g.W = p.width;
    g.H = p.height;
    g.GP = (p.width + 3) & ~3;
    h->ip = 3 * g.GP;
    g.WW = (p.width + 63) / 64;
    g.CAP = p.width / 2 + 1;
    g.L = L;
    // rings sized for two batches in flight: the pyramid of batch i+1 and the
    // flow of batch i (R: frames a0-1 .. a0+2n-1), the flow of batch i+1 and
    // the vote of batch i (raw bits: frames a0-window .. a0+2n-1)
    g.RS = 2 * mb + 1;
    g.RB = p.window + 2 * mb;
    g.iters = p.iterations;
    g.m = p.winsize / 2;
    g.box_scale = 1. / (p.winsize * p.winsize);
    g.up = (float)(1. / p.pyr_scale);
    g.flow_thr = p.flow_threshold;
    // box sums: 0 direct per pixel (k_flow), 1 OpenCV's running order by the
    // barrier-phased scan, 2 by the pipelined scan where it applies (winsize 9;
    // of_launch_flow). DVC_OF_SCAN2=0 at create selects 1 (read per handle:
    // tests compare the two scans, tests/test_of_gpu.py)
    {
        const char* e = getenv("DVC_OF_SCAN2");
        g.sliding = (p.flags & DVC_FLAG_OF_DIRECT_SUMS) ? 0 : (e && atoi(e) == 0 ? 1 : 2);
    }
    poly_coef(p.poly_n, p.poly_sigma, g.pc);   // FarnebackPolyExp(I, R, polyN, ...): n = poly_n
    dvc_host::dct_matrix(8, h->M);
    ellipse_rows(p.morph_kernel, g);           // of:62
    {   // the mask stage's morph rows + halo in LDS: a large element on a wide frame may not fit
        int lds = 160 * 1024;
        if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) != hipSuccess) lds = 160 * 1024;
        if (dvc::of_mask_min_lds(g) > (size_t)lds) {
            const size_t need = dvc::of_mask_min_lds(g);
            delete h;
            return fail(DVC_E_UNSUPPORTED, "morph_kernel %d at width %d: the mask stage needs %zu B of LDS (max %d)",
                        p.morph_kernel, p.width, need, lds);
        }
    }

    auto bad = [&](hipError_t e, const char* what) {
        int rc = fail(e == hipErrorOutOfMemory ? DVC_E_NOMEM : DVC_E_HIP, "%s: %s", what, hipGetErrorString(e));
        of_free(h);
        delete h;
        return rc;
    };
    auto unsupported = [&](const char* what, int v) {
        int rc = fail(DVC_E_UNSUPPORTED, what, v);
        of_free(h);
        delete h;
        return rc;
    };
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return bad(e, "hipSetDevice");
    h->user = (hipStream_t)hip_stream;
    h->has_user = hip_stream != nullptr || (p.flags & DVC_FLAG_JOIN_STREAM);
    // three internal streams (pyramid, flow, mask/output): within the default 4
    // hardware queues beside the framework's stream, so no two stages share a
    // queue (a shared queue serialises them); the caller's stream is only joined
    // equal priorities: the flow and pyramid stages alternate as the critical
    // chain (interleaved sweep after the packed M phase: equal 16.15 k, flow +
    // mask high / pyramid low 15.88 k Mpx/s)
    if ((e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking)) != hipSuccess) return bad(e, "hipStreamCreate");
    for (hipEvent_t* ev : {&h->ev_user, &h->ev_join, &h->ev_gray, &h->ev_side})
        if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    h->s_pyr = h->stream;
    {
        // DVC_OF_PRIO=<flow><mask> (experiments): h / n / l stream priority each
        const char* pe = dvc::tune_env("DVC_OF_PRIO");
        int lo = 0, hi = 0;
        (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
        auto prio = [&](int i) {
            const char c = pe && (int)strlen(pe) > i ? pe[i] : 'n';
            return c == 'h' ? hi : (c == 'l' ? lo : 0);
        };
        hipStream_t* ss[2] = {&h->s_flow, &h->s_mask};
        for (int i = 0; i < 2; ++i)
            if ((e = hipStreamCreateWithPriority(ss[i], hipStreamNonBlocking, prio(i))) != hipSuccess)
                return bad(e, "hipStreamCreate");
    }
    for (OfSlot& sl : h->slot)
        for (hipEvent_t* ev : {&sl.ev_pyr, &sl.ev_flow, &sl.ev_mask, &sl.ev_l1, &sl.ev_l0a})
            if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    const size_t W = p.width, H = p.height, N = W * H, WW = g.WW, CAP = g.CAP;
    // levels (oc_fb_level_poly geometry)
    std::vector<dvc::LinTap> tabs;   // all tables, uploaded once
    struct TabRef { size_t xt, yt, ux, uy; } tr[dvc::OF_MAX_LEVELS];
    for (int k = 0; k <= L; ++k) {
        dvc::Level& lv = h->lv[k];
        double scale = 1;
        for (int i = 0; i < k; ++i) scale *= p.pyr_scale;
        const double sigma = (1. / scale - 1) * 0.5;
        int sz = ((int)std::lrint(sigma * 5)) | 1;
        if (sz < 3) sz = 3;
        if (sz > dvc::OF_MAX_BLUR) return unsupported("pyramid smoothing kernel of %d taps (max 63)", sz);
        lv.w = (int)std::lrint(p.width * scale);
        lv.h = (int)std::lrint(p.height * scale);
        lv.r = sz / 2;
        double kd[64];
        dvc_host::gauss_f64(sz, sigma, kd);
        for (int i = 0; i < sz; ++i) lv.kf[i] = (float)kd[i];
        std::vector<dvc::LinTap> t;
        tr[k].xt = tabs.size();
        lin_taps(p.width, lv.w, t);
        tabs.insert(tabs.end(), t.begin(), t.end());
        tr[k].yt = tabs.size();
        lin_taps(p.height, lv.h, t);
        tabs.insert(tabs.end(), t.begin(), t.end());
        tr[k].ux = tr[k].uy = 0;
    }
    for (int k = 0; k < L; ++k) {
        std::vector<dvc::LinTap> t;
        tr[k].ux = tabs.size();
        lin_taps(h->lv[k + 1].w, h->lv[k].w, t);
        tabs.insert(tabs.end(), t.begin(), t.end());
        tr[k].uy = tabs.size();
        lin_taps(h->lv[k + 1].h, h->lv[k].h, t);
        tabs.insert(tabs.end(), t.begin(), t.end());
        // k_flow_up_lds stages the coarse rows a workgroup's up_per rows read
        // in LDS when they fit (the row taps are monotone: first row's s0 ..
        // last row's s1); 8 rows a workgroup beat 4 by 0.7% OF and 16 by 0.3%
        // (3-round same-box A/B), halving the staging per output row
        const int up_per = [] {   // read per handle (tests vary it)
            const char* e = getenv("DVC_OF_UP_ROWS");
            const int v = e ? atoi(e) : dvc::FU_ROWS_LDS;
            return v >= 1 && v <= 64 ? v : dvc::FU_ROWS_LDS;
        }();
        h->lv[k].up_rows = 0;
        // DVC_OF_UP_GATHER (read per handle: tests compare the forms): the gather
        // form k_flow_up on every level (up_rows = 0)
        const bool gather = getenv("DVC_OF_UP_GATHER") != nullptr;
        for (int per = gather ? 0 : up_per; per >= 1 && !h->lv[k].up_rows;
             per = per > dvc::FU_ROWS ? dvc::FU_ROWS : 0) {
            int rows = 0;
            for (int y0 = 0; y0 < h->lv[k].h; y0 += per) {
                const int ye = std::min(y0 + per, h->lv[k].h) - 1;
                rows = std::max(rows, t[ye].s1 - t[y0].s0 + 1);
            }
            if ((size_t)rows * h->lv[k + 1].w * 8 <= dvc::FU_LDS_MAX) {
                h->lv[k].up_rows = rows;
                h->lv[k].up_per = per;
            }
        }
    }
    dvc::LinTap* dtab = nullptr;
    if ((e = of_alloc(h, &dtab, sizeof(dvc::LinTap) * tabs.size())) != hipSuccess) return bad(e, "hipMalloc");
    if ((e = hipMemcpy(dtab, tabs.data(), sizeof(dvc::LinTap) * tabs.size(), hipMemcpyHostToDevice)) != hipSuccess)
        return bad(e, "hipMemcpy");
    for (int k = 0; k <= L; ++k) {
        dvc::Level& lv = h->lv[k];
        const size_t px = (size_t)lv.w * lv.h;
        lv.xt = dtab + tr[k].xt;
        lv.yt = dtab + tr[k].yt;
        lv.ux = k < L ? dtab + tr[k].ux : nullptr;
        lv.uy = k < L ? dtab + tr[k].uy : nullptr;
        if ((e = of_alloc(h, &lv.R, 20 * px * g.RS)) != hipSuccess) return bad(e, "hipMalloc");
        for (int q = 0; q < 2; ++q)
            if ((e = of_alloc(h, &lv.flow[q], 8 * px * mb)) != hipSuccess) return bad(e, "hipMalloc");
        if (k > 0 && (e = of_alloc(h, &lv.tmpc, 4 * H * 2 * (size_t)lv.w * mb)) != hipSuccess) return bad(e, "hipMalloc");
        if (k > 0 && (e = of_alloc(h, &lv.vtmp, 4 * 2 * (size_t)lv.h * 2 * lv.w * mb)) != hipSuccess)
            return bad(e, "hipMalloc");
    }
    dvc::OfBufs& b = h->b;
    struct { void** ptr; size_t bytes; } allocs[] = {
        {(void**)&b.gray, (size_t)g.GP * H * mb},
        {(void**)&b.mring, 8 * H * WW * g.RB},
        {(void**)&b.cnt, 64 * H * WW},
        {(void**)&b.vthr, 2 * 256},
        {(void**)&b.sbits, 8 * H * WW * mb},
        {(void**)&b.obits, 8 * H * WW * mb},
        {(void**)&b.rbits, 8 * H * WW * mb},
        {(void**)&b.rs, 2 * H * CAP * mb},
        {(void**)&b.re, 2 * H * CAP * mb},
        {(void**)&b.nfg, 4 * H * mb},
        {(void**)&b.fpar, 4 * H * CAP * mb},
        {(void**)&b.bx0, 4 * H * CAP * mb},
        {(void**)&b.bx1, 4 * H * CAP * mb},
        {(void**)&b.by0, 4 * H * CAP * mb},
        {(void**)&b.by1, 4 * H * CAP * mb},
        {(void**)&b.roots, 4 * H * CAP * mb},
        {(void**)&b.nroots, 4 * (size_t)mb},
        {(void**)&b.stats, 8 * 4 * 64},
        {(void**)&b.scan_ctr, 4 * 8 * (size_t)(L + 1) * std::max(1, g.iters)},   // SCAN_Q counters a scan launch
        {(void**)&b.scan_abort, 4},
    };
    for (auto& a : allocs)
        if ((e = of_alloc(h, a.ptr, a.bytes)) != hipSuccess) return bad(e, "hipMalloc");
    if (p.flags & DVC_FLAG_KEEP_PLANES)
        if ((e = of_alloc(h, &b.dbg_flow, 8 * N)) != hipSuccess) return bad(e, "hipMalloc");
    if (g.sliding) {   // k_flow_scan hand-off slots, sized for the largest level
        size_t slots = 0;
        for (int k = 0; k <= L; ++k) slots = std::max(slots, dvc::of_scan_slots(g, h->lv[k].w, h->lv[k].h));
        // tags start at 0, below every launch's epoch (>= 1): no slot reads as published
        if ((e = of_alloc(h, &b.scan_g, 16 * slots * mb)) != hipSuccess) return bad(e, "hipMalloc");
        if ((e = hipMemset(b.scan_g, 0, 16 * slots * mb)) != hipSuccess) return bad(e, "hipMemset");
    }
    if ((e = hipMemset(b.scan_abort, 0, 4)) != hipSuccess) return bad(e, "hipMemset");
    {
        const char* fe = getenv("DVC_OF_FAULT");
        h->fault_abort = fe && std::strcmp(fe, "scan_abort") == 0;
    }
    uint16_t vt[256];
    std::memset(vt, 0, sizeof(vt));
    for (int l = 1; l <= p.window; ++l) vt[l] = (uint16_t)vote_threshold(p.alpha_fraction, l);   // <= l + 1 <= 256
    if ((e = hipMemcpy((void*)b.vthr, vt, sizeof(vt), hipMemcpyHostToDevice)) != hipSuccess) return bad(e, "hipMemcpy");
    const size_t FS = (size_t)h->ip * H;   // one staged / packed BGR frame
    if (h->fmt != DVC_FMT_BGR)   // BGR device frames: allocated on first use (of_stage), when re-pitched
        for (OfSlot& sl : h->slot)
            if ((e = of_alloc(h, &sl.fin, FS * mb)) != hipSuccess) return bad(e, "hipMalloc");
    if (!(p.flags & DVC_FLAG_DEVICE_PTRS)) {
        const size_t FI = h->fmt == DVC_FMT_BGR ? FS : 3 * N;   // packed host frame (YUV: 1.5 N bytes used)
        if ((e = of_alloc(h, &h->d_in, FI * mb)) != hipSuccess) return bad(e, "hipMalloc");
        if ((e = of_alloc(h, &h->d_mask, N * mb)) != hipSuccess) return bad(e, "hipMalloc");
        if ((e = of_alloc(h, &h->d_cp, 3 * N * mb)) != hipSuccess) return bad(e, "hipMalloc");
        if ((e = hipHostMalloc((void**)&h->h_in, FI * mb)) != hipSuccess) return bad(e, "hipHostMalloc");
        if ((e = hipHostMalloc((void**)&h->h_mask, N * mb)) != hipSuccess) return bad(e, "hipHostMalloc");
        if ((e = hipHostMalloc((void**)&h->h_cp, 3 * N * mb)) != hipSuccess) return bad(e, "hipHostMalloc");
    }
    if ((e = hipMemsetAsync(b.stats, 0, 8 * 4 * 64, h->stream)) != hipSuccess) return bad(e, "hipMemset");
    if ((e = hipStreamSynchronize(h->stream)) != hipSuccess) return bad(e, "hipStreamSynchronize");
    *out = h;
    return DVC_OK;
}

int dvc_of_prime(dvc_of* h, const uint8_t* bgr, size_t pitch)
{
    if (!h || !bgr) return fail(DVC_E_INVALID, "NULL argument");
    if (!of_pitch_ok(h, pitch)) return fail(DVC_E_INVALID, "pitch %zu invalid", pitch);
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(of_sync_all(h));   // no batch of a previous run may still be in flight
    HIP_OK(of_wait_user(h));
    const size_t W = h->p.width, H = h->p.height, WW = h->g.WW;
    const uint8_t* d = bgr;
    int dp = (int)pitch, crows = h->crows;
    if (!(h->p.flags & DVC_FLAG_DEVICE_PTRS)) {
        of_pack_host(h, bgr, pitch, h->h_in);
        const size_t fb = h->fmt == DVC_FMT_BGR ? (size_t)h->ip * H : dvc::yuv_frame_bytes(W, (int)H);
        HIP_OK(hipMemcpyAsync(h->d_in, h->h_in, fb, hipMemcpyHostToDevice, h->stream));
        d = h->d_in;
        dp = (int)(h->fmt == DVC_FMT_BGR ? h->ip : W);
        crows = (int)H;
    }
    for (OfSlot& sl : h->slot) sl.recorded = false;   // synced above: no batch in flight
    const uint8_t* kd = nullptr;
    int kp = 0;
    size_t kfs = 0;
    dvc::SrcFmt sf{};
    int rc = of_stage(h, h->slot[0], d, dp, 0, 1, crows, h->stream, &kd, &kp, &kfs, &sf);
    if (rc) return rc;
    HIP_OK(dvc::of_launch_pyramid(h->g, h->lv, h->b, kd, kp, kfs, sf, 0, 1, h->stream));   // of:60
    HIP_OK(hipMemsetAsync(h->b.mring, 0, 8 * H * WW * h->g.RB, h->stream));            // of:61 deque()
    HIP_OK(hipMemsetAsync(h->b.cnt, 0, 64 * H * WW, h->stream));
    HIP_OK(hipMemsetAsync(h->b.stats, 0, 8 * 4 * 64, h->stream));
    // a new run: a hand-off timeout of an earlier run (reported by its sync)
    // does not poison this one
    HIP_OK(hipMemsetAsync(h->b.scan_abort, 0, 4, h->stream));
    HIP_OK(hipStreamSynchronize(h->stream));
    for (OfSlot& sl : h->slot) sl.recorded = false;
    h->seq = 0;
    h->a_next = 1;
    h->frames = 0;
    h->last_n = 0;
    h->primed = true;
    return DVC_OK;
}

// Resume a feed (checkpoint / resume) from the state the
// reference carries across frames: the previous gray (of:60,101) and the raw
// |flow| masks of the last n frames, oldest first (the deque, of:61,84;
// nonzero = motion; n > window keeps the newest window). Host planes of H x W
// bytes, as dvc_of_read_plane exports them (DVC_OF_PLANE_GRAY, _RAW). The
// previous frame's pyramid is rebuilt from the gray exactly: a BGR frame with
// B = G = R = gray grays back to itself ((1868 + 9617 + 4899) * g + 2^13 >> 14
// = g), so the prime path runs on it. Counters are reset, as by dvc_of_prime.
int dvc_of_set_state(dvc_of* h, const uint8_t* prev_gray, const uint8_t* raw_masks, int n)
{
    if (!h || !prev_gray || (n > 0 && !raw_masks) || n < 0) return fail(DVC_E_INVALID, "NULL argument / bad count");
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(of_sync_all(h));
    HIP_OK(of_wait_user(h));
    const size_t W = h->p.width, H = h->p.height, WW = h->g.WW, window = (size_t)h->p.window;
    if ((size_t)n > window) {
        raw_masks += ((size_t)n - window) * W * H;
        n = (int)window;
    }
    // the previous frame as gray-replicated BGR rows of ip, through the prime path
    std::vector<uint8_t> bgr((size_t)h->ip * H, 0);
    for (size_t y = 0; y < H; ++y)
        for (size_t x = 0; x < W; ++x) {
            const uint8_t g = prev_gray[y * W + x];
            uint8_t* p = &bgr[y * h->ip + 3 * x];
            p[0] = p[1] = p[2] = g;
        }
    uint8_t* d = nullptr;
    HIP_OK(of_alloc(h, &d, bgr.size()));
    HIP_OK(hipMemcpy(d, bgr.data(), bgr.size(), hipMemcpyHostToDevice));
    // frames 1..n are the window's masks; the previous frame is a = n
    std::vector<uint64_t> bits(H * WW * std::max(n, 1), 0);
    std::vector<uint8_t> cnt(64 * H * WW, 0);   // bytes, rows of 64 WW (k_vote's counters)
    for (int k = 0; k < n; ++k)
        for (size_t y = 0; y < H; ++y)
            for (size_t x = 0; x < W; ++x)
                if (raw_masks[((size_t)k * H + y) * W + x]) {
                    bits[((size_t)k * H + y) * WW + x / 64] |= 1ull << (x % 64);
                    cnt[y * 64 * WW + x]++;
                }
    HIP_OK(hipMemsetAsync(h->b.mring, 0, 8 * H * WW * h->g.RB, h->stream));
    for (int k = 0; k < n; ++k)
        HIP_OK(hipMemcpyAsync(h->b.mring + (size_t)((k + 1) % h->g.RB) * H * WW, bits.data() + (size_t)k * H * WW,
                              8 * H * WW, hipMemcpyHostToDevice, h->stream));
    HIP_OK(hipMemcpyAsync(h->b.cnt, cnt.data(), cnt.size(), hipMemcpyHostToDevice, h->stream));
    for (OfSlot& sl : h->slot) sl.recorded = false;
    HIP_OK(dvc::of_launch_pyramid(h->g, h->lv, h->b, d, h->ip, (size_t)h->ip * H, dvc::SrcFmt{}, n, 1, h->stream));
    HIP_OK(hipMemsetAsync(h->b.stats, 0, 8 * 4 * 64, h->stream));
    HIP_OK(hipMemsetAsync(h->b.scan_abort, 0, 4, h->stream));
    HIP_OK(hipStreamSynchronize(h->stream));
    // the temporary frame is released now (no kernel reads it any more)
    for (size_t i = 0; i < h->dev.size(); ++i)
        if (h->dev[i] == d) {
            (void)hipFree(d);
            h->dev.erase(h->dev.begin() + (long)i);
            break;
        }
    h->seq = 0;
    h->a_next = n + 1;
    h->frames = 0;
    h->last_n = 0;
    h->primed = true;
    return DVC_OK;
}

}  // extern "C"

static int of_enqueue(dvc_of* h, const uint8_t* d, int dp, size_t fstride, int n, uint8_t* mask, size_t mstride,
                      uint8_t* cp, size_t ostride, int crows)
{
    const long long a0 = h->a_next;
    const bool timed = h->p.flags & DVC_FLAG_KTIMING;
    // slot S last held batch i-2: with RS = 2 mb + 1 the pyramid of batch i
    // overwrites R slots that only flow(i-2) reads; with RB = window + 2 mb the
    // raw bits flow(i) writes are the evictions only vote(i-2) reads
    OfSlot& S = h->slot[h->seq & 1];
#ifdef DVC_ABLATION
    // DVC_OF_SKIP (stage ablation for profiling only, results are wrong when
    // set): bit 1 flow, 2 vote + mask morphology / rectangles, 3 k_of_out (the
    // pyramid always runs: the flow kernels index R by the flow). Only in the
    // ablation build (tools/build_variant.sh <out> -DDVC_ABLATION).
    static const int skip = [] {
        const char* e = getenv("DVC_OF_SKIP");
        const int v = e ? atoi(e) : 0;
        if (v) std::fprintf(stderr, "dvc: DVC_OF_SKIP=%d set: stages skipped, outputs are wrong (profiling only)\n", v);
        return v;
    }();
#else
    constexpr int skip = 0;
#endif
    if (S.recorded) HIP_OK(hipStreamWaitEvent(h->s_pyr, S.ev_flow, 0));
    // The pyramid of batch i also waits for the flow of batch i-1 (not only
    // i-2, whose R slots it overwrites): a scan launch needs whole CUs (two of
    // its workgroups fill a CU's register file), so k_of_front0 beside the
    // coarse levels' latency-bound wavefronts starved both — level 2's first
    // iteration took ~3 ms beside it for 1.7 % of the pixels. Serial: +4 % (3
    // rounds, one box). DVC_OF_SERIAL=0 restores the overlap; =2 also holds
    // the flow of batch i until the mask stage of batch i-1 is done.
    static const int serial = [] { const char* e = dvc::tune_env("DVC_OF_SERIAL"); return e ? atoi(e) : 1; }();
    OfSlot& Sp = h->slot[(h->seq + 1) & 1];   // batch i-1
    // (experiments) =3: wait only for batch i-1's coarse levels, =4: for its
    // level 0's first iteration — the pyramid then fills the CUs the level-0
    // scan frees in its tail
    if (serial >= 1 && Sp.recorded)
        HIP_OK(hipStreamWaitEvent(h->s_pyr, serial == 3 ? Sp.ev_l1 : serial == 4 ? Sp.ev_l0a : Sp.ev_flow, 0));
    dvc::SrcFmt sf{};
    {   // 4:2:0 surfaces read in place, or -> BGR (of:66,145) / re-pitched BGR in
        // the slot's frames, read by the pyramid and by k_of_out
        const uint8_t* kd = nullptr;
        int kp = 0;
        size_t kfs = 0;
        int rc = of_stage(h, S, d, dp, fstride, n, crows, h->s_pyr, &kd, &kp, &kfs, &sf);
        if (rc) return rc;
        d = kd;
        dp = kp;
        fstride = kfs;
    }
    HIP_OK(dvc::of_launch_pyramid(h->g, h->lv, h->b, d, dp, fstride, sf, a0, n, h->s_pyr, h->s_flow, h->ev_gray,
                                  h->ev_side));
    HIP_OK(hipEventRecord(S.ev_pyr, h->s_pyr));
    HIP_OK(hipStreamWaitEvent(h->s_flow, S.ev_pyr, 0));
    if (S.recorded) HIP_OK(hipStreamWaitEvent(h->s_flow, S.ev_mask, 0));
    if (serial >= 2 && Sp.recorded) HIP_OK(hipStreamWaitEvent(h->s_flow, Sp.ev_mask, 0));
    if (timed) {
        while (h->ev.size() < h->ev_used + 2) {
            hipEvent_t e;
            HIP_OK(hipEventCreate(&e));
            h->ev.push_back(e);
        }
    }
    if (h->fault_abort) HIP_OK(hipMemsetAsync(h->b.scan_abort, 0xff, 4, h->s_flow));
    if (!(skip & 2)) HIP_OK(dvc::of_launch_flow(h->g, h->lv, h->b, a0, n, h->g.L, 1, h->s_flow, &h->epoch));
    HIP_OK(hipEventRecord(S.ev_l1, h->s_flow));
    if (timed) HIP_OK(hipEventRecord(h->ev[h->ev_used], h->s_flow));
    if (!(skip & 2))
        HIP_OK(dvc::of_launch_flow(h->g, h->lv, h->b, a0, n, 0, 0, h->s_flow, &h->epoch, serial == 4 ? S.ev_l0a : nullptr,
                                   &h->l0_kernel));
    if (timed) {
        HIP_OK(hipEventRecord(h->ev[h->ev_used + 1], h->s_flow));
        h->ev_used += 2;
    }
    HIP_OK(hipEventRecord(S.ev_flow, h->s_flow));
    HIP_OK(hipStreamWaitEvent(h->s_mask, S.ev_flow, 0));
    if (!(skip & 4)) HIP_OK(dvc::of_launch_mask(h->g, h->b, a0, h->p.window, n, h->s_mask));
    dvc::OfOutArgs o{};
    o.bgr = d;
    o.pitch = dp;
    o.fstride = fstride;
    o.mask = mask;
    o.mstride = mstride;
    o.compressed = cp;
    o.ostride = ostride;
    o.quant = h->p.quant;
    o.qinv = 1.0 / (double)h->p.quant;
    o.M = h->M;
    o.sf = sf;
    if (!(skip & 8)) HIP_OK(dvc::of_launch_out(h->g, h->b, o, n, h->s_mask));
    HIP_OK(hipEventRecord(S.ev_mask, h->s_mask));
    S.recorded = true;
    h->seq++;
    h->a_next += n;
    h->frames += (uint64_t)n;
    h->last_n = n;
    return DVC_OK;
}

static int of_run(dvc_of* h, const uint8_t* bgr, size_t pitch, size_t fstride, int n, uint8_t* mask, size_t mstride,
                  uint8_t* compressed, size_t ostride)
{
    if (!h || !bgr) return fail(DVC_E_INVALID, "NULL argument");
    if (!h->primed) return fail(DVC_E_STATE, "step before dvc_of_prime");
    if (n < 0) return fail(DVC_E_INVALID, "negative frame count");
    const size_t W = h->p.width, H = h->p.height, N = W * H;
    const bool yuv = h->fmt != DVC_FMT_BGR;
    if (!of_pitch_ok(h, pitch)) return fail(DVC_E_INVALID, "pitch %zu invalid", pitch);
    if (n > 1 && fstride < of_frame_span(h, pitch)) return fail(DVC_E_INVALID, "frame stride %zu invalid", fstride);
    if (n > 1 && mask && mstride < N) return fail(DVC_E_INVALID, "mask stride %zu invalid", mstride);
    if (n > 1 && compressed && ostride < 3 * N) return fail(DVC_E_INVALID, "output frame stride %zu invalid", ostride);
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(of_wait_user(h));
    const bool devp = h->p.flags & DVC_FLAG_DEVICE_PTRS;
    for (int f0 = 0; f0 < n; f0 += h->max_batch) {
        const int m = std::min(h->max_batch, n - f0);
        const uint8_t* in = bgr + (size_t)f0 * fstride;
        uint8_t* mk = mask ? mask + (size_t)f0 * mstride : nullptr;
        uint8_t* cp = compressed ? compressed + (size_t)f0 * ostride : nullptr;
        if (devp) {
            int rc = of_enqueue(h, in, (int)pitch, fstride, m, mk, mstride, cp, ostride, h->crows);
            if (rc) return rc;
            continue;
        }
        const size_t FI = yuv ? 3 * N : (size_t)h->ip * H;   // packed frame slot (of_pack_host)
        for (int t = 0; t < m; ++t) of_pack_host(h, in + (size_t)t * fstride, pitch, h->h_in + (size_t)t * FI);
        HIP_OK(hipMemcpyAsync(h->d_in, h->h_in, (size_t)m * FI, hipMemcpyHostToDevice, h->s_pyr));
        int rc = of_enqueue(h, h->d_in, (int)(yuv ? W : h->ip), FI, m, mk ? h->d_mask : nullptr, N,
                            cp ? h->d_cp : nullptr, 3 * N, (int)H);
        if (rc) return rc;
        if (mk) HIP_OK(hipMemcpyAsync(h->h_mask, h->d_mask, (size_t)m * N, hipMemcpyDeviceToHost, h->s_mask));
        if (cp) HIP_OK(hipMemcpyAsync(h->h_cp, h->d_cp, (size_t)m * 3 * N, hipMemcpyDeviceToHost, h->s_mask));
        HIP_OK(of_sync_all(h));
        for (int t = 0; t < m; ++t) {
            if (mk) std::memcpy(mk + (size_t)t * mstride, h->h_mask + (size_t)t * N, N);
            if (cp) std::memcpy(cp + (size_t)t * ostride, h->h_cp + (size_t)t * 3 * N, 3 * N);
        }
    }
    HIP_OK(of_join_user(h));
    return devp ? DVC_OK : of_check_abort(h);
}

extern "C" {

int dvc_of_step(dvc_of* h, const uint8_t* bgr, size_t pitch, uint8_t* mask, uint8_t* compressed)
{
    return of_run(h, bgr, pitch, 0, 1, mask, 0, compressed, 0);
}

int dvc_of_step_batch(dvc_of* h, const uint8_t* bgr, size_t pitch, size_t frame_stride, int n, uint8_t* mask,
                      size_t mask_stride, uint8_t* compressed, size_t out_stride)
{
    return of_run(h, bgr, pitch, frame_stride, n, mask, mask_stride, compressed, out_stride);
}

int dvc_of_sync(dvc_of* h)
{
    if (!h) return fail(DVC_E_INVALID, "NULL handle");
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(of_sync_all(h));
    return of_check_abort(h);
}

int dvc_of_get_stats(dvc_of* h, dvc_of_stats* out)
{
    if (!h || !out) return fail(DVC_E_INVALID, "NULL argument");
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(of_sync_all(h));
    unsigned long long slots[64 * 4], s[4] = {0, 0, 0, 0};
    HIP_OK(hipMemcpy(slots, h->b.stats, sizeof(slots), hipMemcpyDeviceToHost));
    for (int i = 0; i < 64 * 4; ++i) s[i % 4] += slots[i];
    out->frames = h->frames;
    out->motion_px = s[1];
    out->components = s[2];
    out->static_blocks = s[3];
    return DVC_OK;
}

int dvc_of_read_plane(dvc_of* h, int plane, uint8_t* dst)
{
    if (!h || !dst) return fail(DVC_E_INVALID, "NULL argument");
    if (!h->frames) return fail(DVC_E_STATE, "no frame stepped yet");
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(of_sync_all(h));
    const size_t W = h->p.width, H = h->p.height, N = W * H, WW = h->g.WW, t = (size_t)h->last_n - 1;
    if (plane == DVC_OF_PLANE_GRAY) {   // rows of GP on the device
        const size_t GP = h->g.GP;
        HIP_OK(hipMemcpy2D(dst, W, h->b.gray + t * GP * H, GP, W, H, hipMemcpyDeviceToHost));
        return DVC_OK;
    }
    const uint64_t* src = nullptr;
    switch (plane) {
    case DVC_OF_PLANE_RAW: src = h->b.mring + (size_t)((h->a_next - 1) % h->g.RB) * H * WW; break;
    case DVC_OF_PLANE_SMOOTH: src = h->b.sbits + t * H * WW; break;
    case DVC_OF_PLANE_MORPH: src = h->b.obits + t * H * WW; break;
    case DVC_OF_PLANE_RECT: src = h->b.rbits + t * H * WW; break;
    default: return fail(DVC_E_INVALID, "unknown plane %d", plane);
    }
    std::vector<uint64_t> bits(H * WW);
    HIP_OK(hipMemcpy(bits.data(), src, 8 * H * WW, hipMemcpyDeviceToHost));
    for (size_t y = 0; y < H; ++y)
        for (size_t x = 0; x < W; ++x) dst[y * W + x] = ((bits[y * WW + x / 64] >> (x % 64)) & 1) ? 255 : 0;
    return DVC_OK;
}

int dvc_of_read_flow(dvc_of* h, float* dst)
{
    if (!h || !dst) return fail(DVC_E_INVALID, "NULL argument");
    if (!h->frames) return fail(DVC_E_STATE, "no frame stepped yet");
    if (!h->b.dbg_flow) return fail(DVC_E_STATE, "flow readback needs DVC_FLAG_KEEP_PLANES");
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(of_sync_all(h));
    HIP_OK(hipMemcpy(dst, h->b.dbg_flow, 8 * (size_t)h->p.width * h->p.height, hipMemcpyDeviceToHost));
    return DVC_OK;
}

int dvc_of_ktime(dvc_of* h, double* total_ms, uint64_t* launches, int reset)
{
    if (!h) return fail(DVC_E_INVALID, "NULL handle");
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(of_sync_all(h));
    double t = 0.0;
    for (size_t i = 0; i + 1 < h->ev_used; i += 2) {
        float ms = 0.f;
        HIP_OK(hipEventElapsedTime(&ms, h->ev[i], h->ev[i + 1]));
        t += ms;
    }
    if (total_ms) *total_ms = t;
    if (launches) *launches = (h->ev_used / 2) * (uint64_t)h->g.iters;
    if (reset) h->ev_used = 0;
    return DVC_OK;
}

int dvc_of_ktime_kernel(const dvc_of* h)
{
    if (!h) return fail(DVC_E_INVALID, "NULL handle");
    if (h->l0_kernel < 0) return fail(DVC_E_STATE, "no batch stepped yet");
    return h->l0_kernel;
}

int dvc_of_debug_read(dvc_of* h, int what, int level, void* dst, int* w, int* hgt)
{
    if (!h) return fail(DVC_E_INVALID, "NULL handle");
    if (level < 0 || level > h->g.L) return fail(DVC_E_INVALID, "level %d outside 0..%d", level, h->g.L);
    const dvc::Level& L = h->lv[level];
    if (w) *w = L.w;
    if (hgt) *hgt = L.h;
    if (!dst) return DVC_OK;
    if (!h->frames) return fail(DVC_E_STATE, "no frame stepped yet");
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(of_sync_all(h));
    const size_t px = (size_t)L.w * L.h;
    const long long a = h->a_next - 1;
    const void* src = nullptr;
    size_t bytes = 0;
    if (what == 0 || what == 1) {
        src = L.R + (size_t)(((a - what) % h->g.RS + h->g.RS) % h->g.RS) * px * 5;
        bytes = 20 * px;
    } else if (what == 2) {
        if (level == 0 && h->g.iters < 2) return fail(DVC_E_STATE, "level 0 keeps no flow with 1 iteration");
        src = L.flow[0] + (size_t)(h->last_n - 1) * px * 2;
        bytes = 8 * px;
    } else {
        return fail(DVC_E_INVALID, "unknown debug item %d", what);
    }
    HIP_OK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return DVC_OK;
}

void dvc_of_destroy(dvc_of* h)
{
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)of_sync_all(h);
    of_free(h);
    delete h;
}

}  // extern "C"

// compress_with_motion (of:111-193) as a handle: the frames and decoded mask
// frames of one video, n at a time. Device buffers for max_batch frames:
// staged input frames (rows of ip), mask bits, outputs (host-pointer mode).
struct dvc_ofc {
    int W = 0, H = 0, WW = 0, ip = 0, device = 0, max_batch = 1;
    uint32_t flags = 0;
    float quant = 100.f;
    hipStream_t stream = nullptr;    // the caller's (may be NULL = legacy default) or our own
    bool own_stream = false;
    uint8_t *fin = nullptr, *d_mask = nullptr, *d_out = nullptr;
    uint64_t* bits = nullptr;
    dvc::DctMat M{};
};

static void ofc_free(dvc_ofc* h)
{
    for (void* p : {(void*)h->fin, (void*)h->d_mask, (void*)h->d_out, (void*)h->bits})
        if (p) (void)hipFree(p);
    if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
}

extern "C" {

int dvc_ofc_create(int width, int height, float quant, int max_batch, int device, void* hip_stream, uint32_t flags,
                   dvc_ofc** out)
{
    if (!out) return fail(DVC_E_INVALID, "NULL argument");
    if (width < 1 || height < 1 || width > 65520) return fail(DVC_E_INVALID, "frame %dx%d invalid", width, height);
    if (!(quant == quant) || quant == 0.0f) return fail(DVC_E_INVALID, "quant must be nonzero");
    if (max_batch < 0 || max_batch > DVC_MAX_BATCH) return fail(DVC_E_INVALID, "max_batch %d outside 1..%d", max_batch,
                                                                DVC_MAX_BATCH);
    HIP_OK(hipSetDevice(device));
    dvc_ofc* h = new dvc_ofc();
    h->W = width;
    h->H = height;
    h->WW = (width + 63) / 64;
    h->ip = 3 * ((width + 3) & ~3);
    h->device = device;
    h->max_batch = max_batch ? max_batch : 1;
    h->flags = flags;
    h->quant = quant;
    dvc_host::dct_matrix(8, h->M);
    const size_t W = width, H = height, mb = h->max_batch;
    hipError_t e = hipSuccess;
    if (hip_stream) {
        h->stream = (hipStream_t)hip_stream;
    } else {
        e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
        h->own_stream = e == hipSuccess;
    }
    if (e == hipSuccess) e = hipMalloc((void**)&h->bits, 8 * H * h->WW * mb);
    if (e == hipSuccess) e = hipMalloc((void**)&h->fin, (size_t)h->ip * H * mb);   // staged / re-pitched frames
    if (e == hipSuccess && !(flags & DVC_FLAG_DEVICE_PTRS)) {
        e = hipMalloc((void**)&h->d_mask, 3 * W * H * mb);
        if (e == hipSuccess) e = hipMalloc((void**)&h->d_out, 3 * W * H * mb);
    }
    if (e != hipSuccess) {
        ofc_free(h);
        delete h;
        return fail(e == hipErrorOutOfMemory ? DVC_E_NOMEM : DVC_E_HIP, "ofc create: %s", hipGetErrorString(e));
    }
    *out = h;
    return DVC_OK;
}

int dvc_ofc_run(dvc_ofc* h, const uint8_t* bgr, size_t pitch, size_t frame_stride, const uint8_t* mask,
                size_t mask_pitch, size_t mask_stride, int mask_channels, int n, uint8_t* out, size_t out_stride)
{
    if (!h || !bgr || !mask || !out) return fail(DVC_E_INVALID, "NULL argument");
    if (n < 0) return fail(DVC_E_INVALID, "negative frame count");
    if (mask_channels != 1 && mask_channels != 3) return fail(DVC_E_INVALID, "mask_channels %d: 1 or 3", mask_channels);
    const size_t W = h->W, H = h->H, N = W * H, FS = (size_t)h->ip * H;
    if (pitch < 3 * W || mask_pitch < W * mask_channels) return fail(DVC_E_INVALID, "pitch invalid");
    if (n > 1 && (frame_stride < pitch * (H - 1) + 3 * W || mask_stride < mask_pitch * (H - 1) + W * mask_channels ||
                  out_stride < 3 * N))
        return fail(DVC_E_INVALID, "frame / mask / output stride invalid");
    HIP_OK(hipSetDevice(h->device));
    const bool devp = h->flags & DVC_FLAG_DEVICE_PTRS;
    hipStream_t st = h->stream;
    dvc::OfGeom g{};
    g.W = h->W;
    g.H = h->H;
    g.WW = h->WW;
    g.GP = (h->W + 3) & ~3;
    dvc::OfBufs b{};
    for (int f0 = 0; f0 < n; f0 += h->max_batch) {
        const int m = std::min(h->max_batch, n - f0);
        const uint8_t* in = bgr + (size_t)f0 * frame_stride;
        const uint8_t* mk = mask + (size_t)f0 * mask_stride;
        uint8_t* o = out + (size_t)f0 * out_stride;
        // frames the kernel reads: rows of pitch % 4 == 0 reaching whole quads
        const uint8_t* kd = in;
        size_t kp = pitch, kfs = frame_stride;
        if (!devp || pitch % 4 || pitch < (size_t)h->ip || ((uintptr_t)in & 3) || (m > 1 && frame_stride % 4)) {
            const hipMemcpyKind k = devp ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
            for (int t = 0; t < m; ++t)
                HIP_OK(hipMemcpy2DAsync(h->fin + t * FS, h->ip, in + (size_t)t * frame_stride, pitch, 3 * W, H, k, st));
            kd = h->fin;
            kp = h->ip;
            kfs = FS;
        }
        const uint8_t* dm = mk;
        size_t dmp = mask_pitch, dms = mask_stride;
        if (!devp) {   // decoded masks up (rows of W * channels)
            const size_t mrow = W * mask_channels;
            for (int t = 0; t < m; ++t)
                HIP_OK(hipMemcpy2DAsync(h->d_mask + t * mrow * H, mrow, mk + (size_t)t * mask_stride, mask_pitch, mrow,
                                        H, hipMemcpyHostToDevice, st));
            dm = h->d_mask;
            dmp = mrow;
            dms = mrow * H;
        }
        HIP_OK(dvc::of_launch_mask_bits(dm, dmp, dms, mask_channels, h->W, h->H, m, h->bits, st));
        dvc::OfOutArgs a{};
        a.bgr = kd;
        a.pitch = (int)kp;
        a.fstride = kfs;
        a.mbits = h->bits;
        a.mbstride = H * h->WW;
        a.compressed = devp ? o : h->d_out;
        a.ostride = devp ? out_stride : 3 * N;
        a.quant = h->quant;
        a.qinv = 1.0 / (double)h->quant;
        a.M = h->M;
        HIP_OK(dvc::of_launch_out(g, b, a, m, st));
        if (!devp) {
            for (int t = 0; t < m; ++t)
                HIP_OK(hipMemcpyAsync(o + (size_t)t * out_stride, h->d_out + t * 3 * N, 3 * N, hipMemcpyDeviceToHost, st));
            HIP_OK(hipStreamSynchronize(st));
        }
    }
    return DVC_OK;
}

int dvc_ofc_sync(dvc_ofc* h)
{
    if (!h) return fail(DVC_E_INVALID, "NULL handle");
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(hipStreamSynchronize(h->stream));
    return DVC_OK;
}

void dvc_ofc_destroy(dvc_ofc* h)
{
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)hipStreamSynchronize(h->stream);
    ofc_free(h);
    delete h;
}

// One frame, host pointers, synchronous: a one-frame dvc_ofc (any W, H; the
// partial edge blocks are skipped as of:159,177 skip them).
int dvc_of_compress(const uint8_t* bgr, size_t pitch, const uint8_t* mask, int width, int height, float quant,
                    int device, uint8_t* out)
{
    dvc_ofc* h = nullptr;
    int rc = dvc_ofc_create(width, height, quant, 1, device, nullptr, 0, &h);
    if (rc) return rc;
    rc = dvc_ofc_run(h, bgr, pitch, 0, mask, (size_t)width, 0, 1, 1, out, 0);
    dvc_ofc_destroy(h);
    return rc;
}

}  // extern "C"
