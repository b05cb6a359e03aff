// of_kernels.h — launch interface between the OF C-ABI host code (of_api.hip)
// and the gfx950 kernels of the optical-flow path (of_kernels.hip). Internal.
//
// The per-frame worker of motion_compression_opt.py (temporal_smoothing_flow,
// of:65-101, fused with compress_with_motion, of:141-185). Every launch covers
// a BATCH of n consecutive frames of one feed. Farneback flow of frame t
// depends only on gray t-1 and gray t (of:72-81), so the whole pyramid and
// every flow iteration run as grids over (tiles x frames); the only recurrence
// is the 30-frame vote (of:84-86), walked in order per tile by k_vote; the
// morphology, bounding-box union and compression are again per frame.
//
// Frame numbering: the primed frame is a = 0, stepped frames a = 1, 2, ...
// Per-level polynomial expansions R live in a ring of RS = max_batch + 1 slots
// (slot a % RS), so frame a's "previous" expansion is the one computed for a-1
// (in this batch or the previous one) — never recomputed. Raw motion bits live
// in a ring of RB = window + max_batch slots (slot a % RB) for the vote.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fd_kernels.h"

namespace dvc {

constexpr int OF_MAX_LEVELS = 6;
constexpr int OF_MAX_POLY_N = 7;   // FarnebackPolyExp half-width n = poly_n (5 or 7)
constexpr int OF_MAX_BOX_M = 8;    // winsize <= 17
constexpr int OF_MAX_BLUR = 63;    // pyramid smoothing kernel taps
constexpr int OF_MAX_MORPH = 64;   // morph_kernel (the ellipse's side, of:62)

// FarnebackPrepareGaussian (optflowgf.cpp), n = poly_n: float taps, index k + n.
struct PolyCoef {
    int n;
    float g[2 * OF_MAX_POLY_N + 1], xg[2 * OF_MAX_POLY_N + 1], xxg[2 * OF_MAX_POLY_N + 1];
    double ig11, ig03, ig33, ig55;
};

constexpr int FU_ROWS_LDS = 8;           // output rows per k_flow_up_lds workgroup (DVC_OF_UP_ROWS)
constexpr int FU_ROWS = 4;               // output rows per k_flow_up workgroup
constexpr size_t FU_LDS_MAX = 48 * 1024;  // k_flow_up_lds: coarse rows staged in LDS, at most this

// INTER_LINEAR source coordinates of one destination column / row.
struct LinTap {
    int s0, s1;
    float w0, w1;
};

// One pyramid level of calcOpticalFlowFarneback (of:72-81).
struct Level {
    int w, h;          // cvRound(W * scale), cvRound(H * scale)
    int r;             // smoothing radius: taps 2r+1 = max(cvRound(sigma*5)|1, 3)
    float kf[OF_MAX_BLUR + 1];   // float Gaussian taps (getGaussianKernel, CV_32F)
    const LinTap* xt;  // w entries: source columns of the full-res blurred image
    const LinTap* yt;  // h entries
    float* R;          // ring of RS slots x w*h*5 floats
    float* tmpc;       // level > 0: n x H x 2w horizontal blur sums at the needed columns
    float* vtmp;       // level > 0: n x 2h x 2w blurred values at the needed (row, column) pairs
    float* flow[2];    // ping-pong n x w*h*2 floats
    const LinTap* ux;  // upsample of the coarser level's flow (k < L): w / h entries
    const LinTap* uy;
    int up_rows;
    int up_per;   // output rows per k_flow_up_lds workgroup       // most coarse rows a k_flow_up workgroup's rows read (0: stage none in LDS)
};

struct OfGeom {
    int W, H, WW, CAP;
    int GP;            // row pitch of the gray frames: W rounded up to 4 (whole dword quads)
    int L;             // coarsest level index (levels L..0 are processed)
    int RS, RB;        // ring slots of R and of the raw motion bits
    int iters, m;      // Farneback iterations, box half-width (winsize / 2)
    double box_scale;  // 1 / (winsize * winsize)
    float up;          // (float)(1 / pyr_scale)
    float flow_thr;
    int sliding;       // box sums: 0 direct per pixel (k_flow); OpenCV's running order by 1 k_flow_scan,
                       // 2 k_flow_scan2 where it applies (winsize 9, else k_flow_scan)
    PolyCoef pc;
    // getStructuringElement(MORPH_ELLIPSE, (mk, mk)) (of:62), anchor (mk/2, mk/2):
    // element row i (dy = i - mk/2) covers dx = mlo[i] .. mhi[i] (empty if
    // mlo > mhi); dilate / erode read src(x + dx, y + dy)
    int mk;
    int8_t mlo[OF_MAX_MORPH], mhi[OF_MAX_MORPH];
};

struct OfBufs {
    uint8_t* gray;         // n x GP*H, this batch's gray frames (rows of GP)
    uint64_t* mring;       // RB x H*WW raw motion bits (|flow| > thr, of:82-83)
    uint32_t* cnt;         // H x WW*16 u32: vote counts, 4 px (bytes) per u32
    const uint16_t* vthr;  // vthr[L] = votes needed with L masks in the window (of:86), L <= window; L+1 = never
    uint64_t* sbits;       // n x H*WW smoothed (vote) bits
    uint64_t* obits;       // n x H*WW after close + open (of:89-90)
    uint64_t* rbits;       // n x H*WW rectangle mask (of:93-97)
    uint16_t *rs, *re;     // n x H*CAP run starts / ends
    uint32_t* nfg;         // n x H runs per row
    uint32_t* fpar;        // n x H*CAP union-find parents
    uint32_t* bx0;         // n x H*CAP bounding box per root (x0, x1, y0, y1)
    uint32_t* bx1;
    uint32_t* by0;
    uint32_t* by1;
    uint32_t* roots;       // n x H*CAP compacted root ids
    uint32_t* nroots;      // n
    float* dbg_flow;       // nullable: final flow of the batch's last frame (W*H*2)
    unsigned long long* stats;  // 64 slots x 4: frames, motion px, components, static blocks
    // k_flow_scan (sliding box sums): strip hand-off state, one 16-B slot per
    // (frame, strip, row block, row, channel) — {tag, sum lo, sum hi, tag},
    // 64 slots (1 KB, whole 128-B lines) per row block; sized for the largest
    // level by of_scan_slots
    uint32_t* scan_g;
    unsigned int* scan_ctr;        // work-item counters (SCAN_Q = 8 queues) per scan launch of a batch
    unsigned int* scan_abort;      // a hand-off wait timed out
};

struct OfOutArgs {
    const uint8_t* bgr;    // frame t at bgr + t*fstride, rows of `pitch` bytes (pitch % 4 == 0 and
                           // >= 3 * roundup(W, 4): whole dword quads are readable)
    int pitch;
    size_t fstride;
    uint8_t* mask;         // nullable: rectangle mask {0,255}, frame t at mask + t*mstride, rows of W
    size_t mstride;
    const uint64_t* mbits; // nullable: the gating mask as bits (H x WW per frame at t*mbstride) instead
    size_t mbstride;       //   of b.rbits (dvc_ofc: a decoded mask.mp4, of:141-149)
    uint8_t* compressed;   // nullable: frame t at compressed + t*ostride, rows of 3W
    size_t ostride;
    float quant;
    double qinv;           // RN53(1 / (double)quant), see div_rn
    DctMat M;              // 8x8 orthonormal DCT-II basis
    SrcFmt sf;             // bgr: packed BGR (fmt 0) or 4:2:0 surfaces read in place (of_launch_pyramid)
};

// gray + pyramid + polynomial expansion of frames a0 .. a0+n-1 (their BGR at
// bgr + t*fstride) into the R rings; gray kept in b.gray.
// sf: how the frames are read — packed BGR rows of `pitch` (sf.fmt = BGR), or
// 4:2:0 decoder surfaces read in place (luma rows of `pitch`, chroma at
// sf.uoff / sf.voff, rows of sf.cpitch; fd_kernels.h SrcFmt), converted as
// cvtColor YUV2BGR per pixel as they load (what cap.read() returns, of:66)
// s2 / ev_gray / ev_side (all or none): levels 2..L on s2 beside level 1 on s
hipError_t of_launch_pyramid(const OfGeom& g, const Level* lv, const OfBufs& b, const uint8_t* bgr, int pitch,
                             size_t fstride, const SrcFmt& sf, long long a0, int n, hipStream_t s,
                             hipStream_t s2 = nullptr, hipEvent_t ev_gray = nullptr, hipEvent_t ev_side = nullptr);
// Farneback levels k_hi down to k_lo (L..0 in total, coarse to fine) for frames
// a0..a0+n-1 (prev = a-1); level 0's last iteration -> raw motion bits in mring
// `kernel` (nullable): which flow kernel the launches of level k_lo took —
// DVC_KTIME_FLOW (k_flow, direct sums), DVC_KTIME_FLOW_SCAN, DVC_KTIME_FLOW_SCAN2
hipError_t of_launch_flow(const OfGeom& g, const Level* lv, const OfBufs& b, long long a0, int n, int k_hi, int k_lo,
                          hipStream_t s, unsigned int* epoch, hipEvent_t ev_it0 = nullptr, int* kernel = nullptr);
// hand-off slots (16 B each) k_flow_scan needs per frame at a level of w x h
size_t of_scan_slots(const OfGeom& g, int w, int h);
// vote (frames in order) -> close/open -> 8-CC bounding boxes -> rectangle mask
hipError_t of_launch_mask(const OfGeom& g, const OfBufs& b, long long a0, int window, int n, hipStream_t s);
// the LDS one row of the mask stage needs (morph_kernel and the width set it): create refuses more than the device has
size_t of_mask_min_lds(const OfGeom& g);
// compress_with_motion (of:151-183) + the mask bytes
hipError_t of_launch_out(const OfGeom& g, const OfBufs& b, const OfOutArgs& o, int n, hipStream_t s);
// a decoded mask plane (1 or 3 channels, rows of mpitch, frames of mstride) ->
// nonzero-after-BGR2GRAY bits, H x WW words per frame (of:147-149)
hipError_t of_launch_mask_bits(const uint8_t* mask, size_t mpitch, size_t mstride, int channels, int W, int H, int n,
                               uint64_t* bits, hipStream_t s);

}  // namespace dvc
