// fd_kernels.h — launch interface between the C-ABI host code (fd_api.hip) and
// the gfx950 kernels (fd_kernels.hip). Internal; not part of include/dvc.h.
//
// Every launch covers a BATCH of n consecutive frames of one feed. The only
// true recurrences of the reference loop (fd:85-138) are prev_gray (fd:133) and
// accumulated_mask (fd:107); both are elementwise, so k_front and k_back walk
// the batch's frames in order inside each tile with that state in registers,
// while the contour filter of every frame of the batch (independent given the
// motion masks) runs as one grid with the frame in blockIdx.y.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dvc {

// Row geometry of the run-length (CCL) stage.
struct RowGeom {
    int W, H;
    int WW;   // 64-px words per mask row = ceil(W/64)
    int CAP;  // max foreground runs per row = W/2 + 1 (gaps per row <= CAP+1)
};

struct GaussTaps {
    int n;
    uint16_t t[64];
};

struct alignas(8) DctMat {
    float m[64];   // BxB row-major orthonormal DCT-II basis M[k][n], float32
    float mt[64];  // its transpose: the pairs (M[k][n], M[k+1][n]) adjacent for
                   // 64-bit scalar kernarg loads (block_dct_quant_pk)
};

// Device buffers of the contour-filter stage: frame f of a batch owns the f-th
// slice of each array (sizes per frame below, see frame()).
struct CclBufs {
    uint64_t* mbits;        // H x WW motion mask
    uint64_t* fbits;        // H x WW filled mask (not-E)
    uint16_t *rs, *re;      // H x CAP run starts / ends
    uint32_t* nfg;          // H runs per row
    uint32_t* fpar;         // H x CAP run union-find parents (root after k_area)
    uint32_t* gpar;         // 1 + H x (CAP+1) gap parents, node 0 = outside
    uint8_t* gE;            // H x (CAP+1) gap is outside (1) / hole (0)
    uint32_t* area2;        // H x CAP 2*area per root
    uint64_t* kbits;        // H x WW kept (filtered) mask
    unsigned long long* stats;  // 64 slots x 4 counters (shared by all frames)
    // Sparse masks (a surveillance frame is mostly still): nullable H bytes per
    // frame, kocc[y] = kept row y has a bit set. With kocc, k_paint writes only
    // the kept rows that have bits (kfull: every row, for plane read-back) and
    // the dilate kernels read only those; without it every row is written.
    uint8_t* kocc = nullptr;
    int kfull = 0;
    // Run index packed per band (k_band): the runs of band b's rows are nodes
    // b*16*CAP + (runs of the band's earlier rows) + k, its gaps 1 + b*16*(CAP+1)
    // + (gaps of earlier rows) + k; rowb[2y], rowb[2y+1] = the first run / gap
    // node of row y (2 x H per frame). A band's few runs share cache lines.
    uint32_t* rowb = nullptr;
    static size_t rowb_bytes(const RowGeom& g, size_t frames) { return (size_t)8 * g.H * frames; }

    __host__ __device__ static size_t bits_per_frame(const RowGeom& g) { return (size_t)g.H * g.WW; }
    __host__ __device__ CclBufs frame(size_t f, const RowGeom& g) const
    {
        const size_t nb = (size_t)g.H * g.WW, nr = (size_t)g.H * g.CAP, ng = (size_t)g.H * (g.CAP + 1);
        return CclBufs{mbits + f * nb, fbits + f * nb, rs + f * nr, re + f * nr, nfg + f * g.H, fpar + f * nr,
                       gpar + f * (ng + 1), gE + f * ng, area2 + f * nr, kbits + f * nb, stats,
                       kocc ? kocc + f * g.H : nullptr, kfull, rowb + f * 2 * g.H};
    }
    // Bytes of every array for `frames` frames (host allocation), in the order
    // of ptrs(): a caller that allocates these NARR arrays has every buffer the
    // kernels touch (launch_ccl refuses a CclBufs without rowb).
    static constexpr int NARR = 11;
    static void sizes(const RowGeom& g, size_t frames, size_t out[NARR])
    {
        const size_t nb = (size_t)g.H * g.WW, nr = (size_t)g.H * g.CAP, ng = (size_t)g.H * (g.CAP + 1);
        const size_t s[NARR] = {8 * nb, 8 * nb, 2 * nr, 2 * nr, 4 * (size_t)g.H, 4 * nr, 4 * (ng + 1), ng, 4 * nr, 8 * nb,
                                rowb_bytes(g, 1)};
        for (int i = 0; i < NARR; ++i) out[i] = s[i] * frames;
    }
    // the arrays sizes() describes; indices 1..8 and 10 are contour-filter
    // working set (touched only inside launch_ccl), 0 and 9 its input / output
    void ptrs(void** out[NARR])
    {
        void** p[NARR] = {(void**)&mbits, (void**)&fbits, (void**)&rs,    (void**)&re,    (void**)&nfg, (void**)&fpar,
                          (void**)&gpar,  (void**)&gE,    (void**)&area2, (void**)&kbits, (void**)&rowb};
        for (int i = 0; i < NARR; ++i) out[i] = p[i];
    }
    static bool working_set(int i) { return (i >= 1 && i <= 8) || i == 10; }
};

// The frames k_front / k_out / k_out_gen read: packed BGR rows (fmt 0,
// DVC_FMT_BGR), or a decoder's 4:2:0 surfaces read in place (DVC_FMT_I420 /
// DVC_FMT_NV12, include/dvc.h): luma rows of the frames' pitch, chroma row r
// at + uoff / voff + r * cpitch (NV12: UV pairs at uoff, voff = uoff + 1),
// cvtColor YUV2BGR per pixel as the pixels are loaded (fd:87's
// VideoCapture.read() without a staged BGR copy: 1.5 B/px read instead of 3).
// In-place reads need pitch % 4 == 0 and a 4-byte aligned base and stride.
struct SrcFmt {
    int fmt;
    size_t uoff, voff, cpitch;
};

// The back of the loop (dilate, accumulate, overlay, compress). Blocks are
// B x B (fd:117-118); NBX x NBY of them cover the frame, the last column / row
// partial when W % B or H % B (fd:120-121). Two layouts:
//  * fast (B = 4, 8): block-major bit fields per frame (k_dilate -> k_acc ->
//    k_out, one lane per block), acc padded to NBX*B x NBY*B;
//  * generic (any other B, and the partial edge blocks of the fast layout):
//    row-major H x WW bit planes (k_dilate_rows -> k_acc_rows -> k_out_gen,
//    LDS-staged block DCTs of any shape).
struct BackArgs {
    RowGeom g;
    const uint8_t* bgr;   // frame t at bgr + t * fstride, rows of `pitch` bytes (pitch % 4 == 0)
    int pitch;
    size_t fstride;
    SrcFmt sf;            // BGR, or 4:2:0 surfaces read in place
    uint8_t* acc;         // read before frame 0, written after frame n-1; rows of `ap` bytes
    int ap;
    uint8_t* overlay;     // nullable; frame t at overlay + t * ostride, rows of opitch
    uint8_t* compressed;  // nullable; same layout
    int opitch;
    size_t ostride;
    int obytes;             // outputs not 4-byte aligned: byte stores
    int out_i420;           // outputs are I420 frames (W x H luma + two W/2 x H/2 chroma planes)
    const uint64_t* kbits;  // kept (filtered) masks from k_paint, H x WW per frame
    const uint8_t* kocc;    // nullable: kept row has bits, H per frame (CclBufs::kocc); rows without are not read
    uint8_t* docc;          // fast layout with kocc: block row by of frame t has dilated bits, docc[by * n + t]
    // fast layout
    void* dblk;             // dilated mask, block-major BxB bit fields per frame (k_dilate -> k_acc)
    void* rblk;             // acc > 127 per pixel, block-major BxB bit fields per frame (k_acc -> k_out)
    uint64_t* sbits;        // acc all zero per block, NBY x SW per frame (k_acc -> k_out)
    int SW;                 // 64-block words per block row = ceil(NBX/64)
    size_t sstride;         // NBY * SW
    // generic layout (row-major H x WW words per frame)
    uint64_t* dbits;        // dilated mask
    uint64_t* rbits;        // acc > 127
    uint64_t* zbits;        // acc != 0
    int B, NBX, NBY;        // block size, blocks across / down (ceil)
    int n;                  // frames in the batch
    int ksize, anchor;
    float alpha, beta, gamma, quant;
    double qinv;            // RN53(1 / (double)quant): the quantiser division as a product (div_rn)
    int acc0_fixed;         // addWeighted(acc 0, dilated 0) == 0: zero blocks stay zero
    int acc_fast;           // k_acc's short form holds (acc_fast_ok): dil0 == +0, no clamp can bind
    uint32_t dil1_bits;     // bits of fmaf(255, beta, gamma), the dilated-pixel addend
    DctMat M;               // fast B x B basis (kernargs)
    const float* Mtab;      // generic bases in device memory: M_B (B*B) | M_{W%B} | M_{H%B}
    unsigned long long* stats;
    uint64_t* dbg_dil;      // nullable: dilated mask bits of frame n-1 (H x WW)
    unsigned long long* err;  // first frame (feed index) with an odd static block side > 1 (atomicMin)
    unsigned long long frame0;  // feed index of the batch's frame 0
};

// Gray planes (prev gray, the prime's scratch) have rows of gs = roundup(W, 4)
// bytes; frames read by the kernels have pitch % 4 == 0 and pitch >= 3 * gs.
hipError_t launch_prime(const uint8_t* bgr, int pitch, uint8_t* gray_tmp, uint32_t* tmp32, uint8_t* out,
                        int W, int H, int gs, const GaussTaps& k, hipStream_t s);

// Speculative outputs of the fused front (block_size 4, BGR outputs; BGR frames or 4:2:0 surfaces read in place;
// dword-aligned output rows). A frame is read from HBM once: while k_front has
// its 4x4 blocks in registers it writes every full block as if it were static —
// overlay = the frame (no acc > 127 pixel can lie in a block whose acc is all
// zero, fd:110-111) and compressed = (Y', Y', Y') of the block's quantised DCT
// (fd:117-130) — and k_fix4 later rewrites only the blocks the
// accumulated mask makes non-static (their YCrCb round trip, and the red
// overlay where acc > 127). Every output byte ends equal to k_out's.
struct FrontOut {
    uint8_t* ov;       // nullable; frame t at ov + t * ostride, rows of opitch
    uint8_t* cp;       // nullable; same layout
    int opitch;
    size_t ostride;
    float quant;
    double qinv;
    DctMat M;          // B x B basis
    int B;             // block size: 4, or 8 (BGR frames in, NW = 4 tiles)
    int i420;          // outputs as BGR2YUV_I420 frames (B = 4, NW = 4): Y plane W x H, U, V of W/2 x H/2
};
// frames t = 0..n-1 at bgr + t*fstride; gray_in = the previous blurred gray,
// gray_out := frame n-1's (distinct buffers); motion mask of frame t -> mbits + t*H*WW;
// fo (nullable): the fused speculative outputs above
hipError_t launch_front(const uint8_t* bgr, int pitch, size_t fstride, const SrcFmt& sf, int n, const uint8_t* gray_in,
                        uint8_t* gray_out, int gs, uint64_t* mbits, const RowGeom& g, int ithresh, hipStream_t s,
                        const FrontOut* fo = nullptr);
// cv2.resize(frame, (W, H)) INTER_LINEAR 8UC3 (fd:74,91) of n frames into dst
// (rows of dpitch, frames of dstride). Tables from resize_tables().
struct ResizeTab {
    int sw, sh, dw, dh;
    int area2x;             // exact 2x downscale: OpenCV's INTER_AREA fast path
    int simd_end;           // bytes of a row done by the 128-bit SIMD formula (VResizeLinearVec_32s8u)
    const int* xo;          // per output column: source column, alpha0, alpha1 (device, 3*dw)
    const int* yo;          // per output row: source row, beta0, beta1 (device, 3*dh)
};
void resize_tables(int sw, int sh, int dw, int dh, int* host_x /* 3*dw */, int* host_y /* 3*dh */, int* area2x,
                   int* simd_end);
hipError_t launch_resize(const uint8_t* src, int spitch, size_t sstride, uint8_t* dst, int dpitch, size_t dstride,
                         int n, const ResizeTab& t, hipStream_t s);
int band_rows(const RowGeom& g);
size_t ccl_max_lds(const RowGeom& g);   // dvc_fd_create refuses frames wider than the LDS allows
hipError_t launch_ccl(const CclBufs& c, const RowGeom& g, int n, int64_t min_area2, hipStream_t s);
// k_dilate then k_acc (the accumulated-mask recurrence: batches in order)
hipError_t launch_accumulate(const BackArgs& a, hipStream_t s);
// k_acc's short form computes fmaf(acc, alpha, D) with D = +0 or fmaf(255, beta,
// gamma) and drops the [0, 255] clamp. Exact when fmaf(0, beta, gamma) is +0
// (the dilated-0 addend; D is then a sign-mask AND of the dil-1 bits) and the
// clamp cannot bind: fmaf and round-to-nearest-even are monotone in acc and D,
// so with alpha >= 0 and D >= 0 every result lies between rint(+0) = 0 and
// rint(fmaf(255, alpha, D1)) <= 255 (NaN fails every comparison below).
inline bool acc_fast_ok(float alpha, float beta, float gamma)
{
    const float d0 = __builtin_fmaf(0.0f, beta, gamma), d1 = __builtin_fmaf(255.0f, beta, gamma);
    uint32_t d0b;
    __builtin_memcpy(&d0b, &d0, 4);
    return d0b == 0 && alpha >= 0.0f && alpha <= 1.0f && d1 >= 0.0f && d1 <= 255.0f &&
           __builtin_rintf(__builtin_fmaf(255.0f, alpha, d1)) <= 255.0f;
}
// k_out (overlay + compressed frames; no recurrence) and k_out_gen for the
// generic layout / partial edge blocks (always launched: it also detects the
// odd-size DCT stop and counts generic static blocks). fix: the fused front
// wrote every full block speculatively (FrontOut); k_out only rewrites the
// blocks that are not static.
hipError_t launch_out(const BackArgs& a, hipStream_t s, bool fix = false);
inline bool fast_block(int B) { return B == 4 || B == 8; }

}  // namespace dvc
