// fd_kernels.hip — gfx950 (MI355X / CDNA4) kernels of the frame-differencing
// per-frame worker (reference: frame_differencing.py:85-138).
//
// One batch of n consecutive frames of a feed = seven launches (fd_kernels.h
// explains the batching):
//   k_front   BGR->gray (fd:92), 5x5 Q8 Gaussian (fd:93), absdiff+threshold
//             (fd:96-97) -> new gray plane + 1-bit motion mask (64 px / u64)
//   k_band    per band of rows, one workgroup: maximal foreground runs and
//             background gaps of every row straight from the bit mask, then
//             union-find in LDS (runs 8-connected, gaps 4-connected, border gaps
//             joined to the OUTSIDE node) -> band-local roots as global ids
//   k_merge   per band seam: global unions of band roots (atomicMin links)
//   k_resolve gaps reaching node 0 are outside (E); the rest are holes: hole
//             pixels are painted into the filled mask F = not E, and the runs
//             left/right of a hole are united (nested components join the
//             external component that encloses them)
//   k_area    2*contourArea of every external component from F's 2x2 windows,
//             accumulated per root (fd:100-103)
//   k_paint   kept components -> filtered bit mask (drawContours FILLED, fd:104)
//   k_back    7x7 dilate (fd:106), addWeighted (fd:107), red overlay
//             (fd:110-111), static BxB block DCT quantisation + YCrCb round trip
//             (fd:115-130)
//
// Everything is integer/byte work except the addWeighted rint and the block
// DCT (fp32, explicit fmaf chains — compiled with -ffp-contract=off).
// No MFMA: there is no dense contraction on this path; the roofline is HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "dvc_device.h"
#include "fd_kernels.h"
#include "klaunch.h"
#include "dct_const.h"
#include "yuv_px.h"
#include "../../include/dvc.h"
#include "tune.h"

namespace dvc {

thread_local std::vector<KNode>* g_krec = nullptr;   // klaunch.h

// ------------------------------------------------------------ prime (fd:77) -
// gray rows of gs = roundup(W, 4) bytes; the last quad of a row may be partial
// (its bytes past W are don't-care padding, read from the padded frame row)
__global__ void __launch_bounds__(256) k_gray(const uint8_t* __restrict__ bgr, int pitch,
                                              uint8_t* __restrict__ gray, int W, int H, int gs)
{
    int q = blockIdx.x * 256 + threadIdx.x;  // quad index in the row
    int y = blockIdx.y;
    if (4 * q >= W) return;
    const uint32_t* p = reinterpret_cast<const uint32_t*>(bgr + (size_t)y * pitch + 12 * q);
    *reinterpret_cast<uint32_t*>(gray + (size_t)y * gs + 4 * q) = gray4(p[0], p[1], p[2]);
}

__global__ void __launch_bounds__(256) k_hblur_q8(const uint8_t* __restrict__ src, uint32_t* __restrict__ tmp,
                                                  int W, int H, int gs, GaussTaps k)
{
    int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    int r = k.n / 2;
    uint32_t s = 0;
    for (int j = 0; j < k.n; ++j) s += (uint32_t)k.t[j] * src[(size_t)y * gs + reflect101(x + j - r, W)];
    tmp[(size_t)y * W + x] = s;
}

__global__ void __launch_bounds__(256) k_vblur_q8(const uint32_t* __restrict__ tmp, uint8_t* __restrict__ dst,
                                                  int W, int H, int gs, GaussTaps k)
{
    int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    int r = k.n / 2;
    uint64_t s = 0;
    for (int i = 0; i < k.n; ++i) s += (uint64_t)k.t[i] * tmp[(size_t)reflect101(y + i - r, H) * W + x];
    dst[(size_t)y * gs + x] = (uint8_t)((s + 32768u) >> 16);
}

// ------------------------------------------------------------------ front ---
// Tile: 256 px (64 lanes x 4 px) x 4*NW rows; NW waves, 4 output rows each
// (interleaved: wave w owns rows w, w+NW, w+2NW, w+3NW). Gray halo 2 px / 2
// rows, loaded as 66 quads x (4*NW + 4) rows with BORDER_REFLECT_101 at the
// image edges — taller tiles re-read fewer halo rows (20/16 at NW = 4, 68/64 at
// NW = 16) at the same registers per lane.
// The workgroup walks a chunk of the batch's frames in order: the previous
// blurred gray of its 4x4 px per lane stays in registers (fd:133), and frame
// t+1's BGR loads are issued as soon as frame t's gray is in LDS, so they fly
// under t's blur. blockIdx.z = chunk of `chunk` frames: chunk 0 starts from the
// previous batch's gray (gray_in), chunk c > 0 first re-derives frame
// c*chunk-1's blurred gray (a warm-up pass that emits no mask) — more
// workgroups in flight for one extra frame read per chunk.
constexpr int FT_W = 256, FT_Q = FT_W / 4 + 2;


typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

// Arithmetic per quad of 4 px (VALU-bound kernel: every op counts):
//   gray      gray4_dot: 2 v_dot4_u32_u8 per pixel
//   5-tap h   one v_dot4 with taps (1,4,6,4) + the 5th byte per output, on
//             v_alignbyte windows of the gray quads
//   5-tap v   packed u16 lanes (sums <= 16 * 4080 < 2^16), (s + 128) >> 8
//   threshold |cur - prev| > t per u16 lane as bit 15 of d + (0x7fff - t)
// The previous blurred gray (fd:133) stays in registers as two u16 pairs.
// A 4-px quad (x even) of a 4:2:0 surface as loaded (y4 = its luma dword;
// I420: c1 / c2 = the u16 of U / V samples; NV12: c1 = the dword U0 V0 U1 V1)
// -> 12 packed BGR bytes (cvtColor YUV2BGR, yuv_px.h)
template <int FMT>
__device__ __forceinline__ void quad_bgr(uint32_t y4, uint32_t c1, uint32_t c2, uint32_t o[3])
{
    if constexpr (FMT == DVC_FMT_NV12) yuvpx::yuv4_bgr(y4, c1 & 255, (c1 >> 8) & 255, (c1 >> 16) & 255, c1 >> 24, o);
    else yuvpx::yuv4_bgr(y4, c1 & 255, c2 & 255, (c1 >> 8) & 255, (c2 >> 8) & 255, o);
}

// gray of a loaded quad: 12 BGR bytes (v0..v2), or a 4:2:0 quad via quad_bgr
template <int FMT>
__device__ __forceinline__ uint32_t quad_gray(uint32_t v0, uint32_t v1, uint32_t v2)
{
    if constexpr (FMT == DVC_FMT_BGR) {
        return gray4_dot(v0, v1, v2);
    } else {
        uint32_t o[3];
        quad_bgr<FMT>(v0, v1, v2, o);
        return gray4_dot(o[0], o[1], o[2]);
    }
}

// OUT (fused speculative outputs, FrontOut in fd_kernels.h; NW = 4 or 8): the
// rows are dealt by block row instead — wave w loads and owns tile rows
// 4w..4w+3, so each lane holds one 4x4 block of the frame, plus one halo row
// (LDS rows 0, 1, 18, 19 for waves 0..3) — and the block's pixels go out as
// the overlay straight from the registers they were loaded into (4:2:0
// surfaces: converted to BGR once, for the overlay and the gray), its gray
// quads (BGR2GRAY luma = BGR2YCrCb Y) from LDS through the quantised DCT into
// the compressed frame.
// fused front workgroups per CU (the VGPR budget: 4 -> 128, 5 -> 96): BGR 4
// (5 measured neutral, with scratch spills), NV12 surfaces 5 (two loads a row:
// the extra wave per SIMD hides them, +2.4 % NV12, experiments/README.md), I420
// surfaces 4 (three loads a row; at 5 the kernel spills 16 VGPRs to scratch:
// 325 k against 359 k Mpx/s, round 6)
#ifndef DVC_FRONT_WGS_BGR
#define DVC_FRONT_WGS_BGR 4
#endif
#ifndef DVC_FRONT_WGS_PF2   // two frames in flight (the fused BGR default): 119 VGPRs
#define DVC_FRONT_WGS_PF2 4
#endif
#ifndef DVC_FRONT_WGS_YUV
#define DVC_FRONT_WGS_YUV 5
#endif
#ifndef DVC_FRONT_WGS_I420
#define DVC_FRONT_WGS_I420 4
#endif
// 8x8 blocks of the fused front (OB = 8, the reference's __main__ variant):
// four lanes per block (lanes 4q..4q+3 of a wave, r = lane & 3 holds rows 2r,
// 2r+1), the block's intermediate planes in an LDS scratch of 68 floats (8
// rows of 8; the pad puts the 16 blocks of a wave on distinct banks). The same
// operation order as block_dct_quant_pk<8> — every output a first product then
// fmaf in index order, two outputs per v_pk_fma_f32 — so bit-identical to the
// one-pass k_out<8>; the quad's lanes are in one wave, so LDS hand-offs between
// the passes need only wave-level ordering.
constexpr int DCT8_S = 68;
__device__ __forceinline__ void dct8_quad(float* S, int r, const float (&x)[2][8], float q, double qinv,
                                          float (&out)[2][8])
{
    const DctMat& M = kDct8;
    // rows: T[i][k] = sum_n X[i][n] M[k][n], i = 2r, 2r+1
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int k = 0; k < 8; k += 2) {
            const f32x2* mt = reinterpret_cast<const f32x2*>(M.mt + k);   // (M[k][n], M[k+1][n]) at mt[4n]
            f32x2 t = (f32x2)(x[ii][0]) * mt[0];
#pragma unroll
            for (int n = 1; n < 8; ++n) t = __builtin_elementwise_fma((f32x2)(x[ii][n]), mt[n * 4], t);
            *reinterpret_cast<f32x2*>(S + (2 * r + ii) * 8 + k) = t;
        }
    wave_sync_lds();
    // columns + quantise: X[k][l] = rint(sum_i M[k][i] T[i][l] / q) q, l = 2r, 2r+1
    f32x2 tc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) tc[i] = *reinterpret_cast<const f32x2*>(S + i * 8 + 2 * r);
    wave_sync_lds();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        f32x2 t = (f32x2)(M.m[k * 8]) * tc[0];
#pragma unroll
        for (int i = 1; i < 8; ++i) t = __builtin_elementwise_fma((f32x2)(M.m[k * 8 + i]), tc[i], t);
        *reinterpret_cast<f32x2*>(S + k * 8 + 2 * r) =
            f32x2{__builtin_rintf(div_rn(t.x, qinv)) * q, __builtin_rintf(div_rn(t.y, qinv)) * q};
    }
    wave_sync_lds();
    // inverse rows: T2[k][n] = sum_l X[k][l] M[l][n], k = 2r, 2r+1
    float xr[2][8];
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int l = 0; l < 8; ++l) xr[ii][l] = S[(2 * r + ii) * 8 + l];
    wave_sync_lds();
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int n = 0; n < 8; n += 2) {
            const f32x2* mp = reinterpret_cast<const f32x2*>(M.m + n);    // (M[l][n], M[l][n+1]) at mp[4l]
            f32x2 t = (f32x2)(xr[ii][0]) * mp[0];
#pragma unroll
            for (int l = 1; l < 8; ++l) t = __builtin_elementwise_fma((f32x2)(xr[ii][l]), mp[l * 4], t);
            *reinterpret_cast<f32x2*>(S + (2 * r + ii) * 8 + n) = t;
        }
    wave_sync_lds();
    // inverse columns: out[i][n] = sum_k M[k][i] T2[k][n], i = 2r, 2r+1 (k in order)
    f32x2 acc[2][4];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        f32x2 row[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) row[p] = *reinterpret_cast<const f32x2*>(S + k * 8 + 2 * p);
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
            const f32x2 m = (f32x2)(M.m[k * 8 + 2 * r + ii]);
#pragma unroll
            for (int p = 0; p < 4; ++p) acc[ii][p] = k == 0 ? m * row[p] : __builtin_elementwise_fma(m, row[p], acc[ii][p]);
        }
    }
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            out[ii][2 * p] = acc[ii][p].x;
            out[ii][2 * p + 1] = acc[ii][p].y;
        }
    wave_sync_lds();   // the scratch is rewritten by the next frame
}

// One row of a BxB block of an output frame as the encoder's 4:2:0 input
// (cvtColor BGR2YUV_I420, include/dvc.h DVC_FLAG_OUT_I420): B luma bytes, and
// on even rows the B/2 chroma samples of the 2x2 quads (their top-left pixel).
// I420 frame at f: Y plane W x H, then U and V planes of W/2 x H/2.
template <int B>
__device__ __forceinline__ void store_i420_row(uint8_t* f, int W, int H, int y, int x, const uint32_t* w)
{
    using namespace yuvpx;
    uint32_t yv[B], uv[B / 2], vv[B / 2];
#pragma unroll
    for (int j = 0; j < B; ++j) {
        const int b = (int)((w[(3 * j) >> 2] >> (8 * ((3 * j) & 3))) & 255);
        const int g = (int)((w[(3 * j + 1) >> 2] >> (8 * ((3 * j + 1) & 3))) & 255);
        const int r = (int)((w[(3 * j + 2) >> 2] >> (8 * ((3 * j + 2) & 3))) & 255);
        yv[j] = luma(b, g, r);
        if (!(j & 1)) {
            uv[j >> 1] = chroma_u(b, g, r);
            vv[j >> 1] = chroma_v(b, g, r);
        }
    }
    uint32_t* yo = reinterpret_cast<uint32_t*>(f + (size_t)y * W + x);
#pragma unroll
    for (int d = 0; d < B / 4; ++d)
        __builtin_nontemporal_store(pack4(yv[4 * d], yv[4 * d + 1], yv[4 * d + 2], yv[4 * d + 3]), yo + d);
    if (!(y & 1)) {
        const size_t c = (size_t)W * H + (size_t)(y >> 1) * (W >> 1) + (x >> 1), q = (size_t)(W >> 1) * (H >> 1);
        if constexpr (B == 4) {
            __builtin_nontemporal_store((uint16_t)(uv[0] | (uv[1] << 8)), reinterpret_cast<uint16_t*>(f + c));
            __builtin_nontemporal_store((uint16_t)(vv[0] | (vv[1] << 8)), reinterpret_cast<uint16_t*>(f + c + q));
        } else {
#pragma unroll
            for (int d = 0; d < B / 8; ++d) {
                __builtin_nontemporal_store(pack4(uv[4 * d], uv[4 * d + 1], uv[4 * d + 2], uv[4 * d + 3]),
                                            reinterpret_cast<uint32_t*>(f + c) + d);
                __builtin_nontemporal_store(pack4(vv[4 * d], vv[4 * d + 1], vv[4 * d + 2], vv[4 * d + 3]),
                                            reinterpret_cast<uint32_t*>(f + c + q) + d);
            }
        }
    }
}


// BGR2YUV_I420 luma of the 4 packed BGR pixels of a quad row (dwords d0..d2),
// as v_dot4 with the 20-bit coefficients split into bytes: the same integer as
// yuvpx::luma (no saturation needed: 16 <= Y <= 235 for every BGR).
__device__ __forceinline__ uint32_t luma4_i420(uint32_t d0, uint32_t d1, uint32_t d2)
{
    using namespace yuvpx;
    constexpr uint32_t K0 = (CBY & 255) | ((CGY & 255) << 8) | ((CRY & 255) << 16);
    constexpr uint32_t K1 = ((CBY >> 8) & 255) | (((CGY >> 8) & 255) << 8) | (((CRY >> 8) & 255) << 16);
    constexpr uint32_t K2 = (CBY >> 16) | ((CGY >> 16) << 8) | ((CRY >> 16) << 16);
    static_assert((CBY >> 24) == 0 && (CGY >> 24) == 0 && (CRY >> 24) == 0 && CBY > 0 && CGY > 0 && CRY > 0,
                  "luma coefficients: three bytes each");
    static_assert((255 * (CBY + CGY + CRY) + HALF + (16 << SHIFT)) >> SHIFT <= 255, "luma never saturates");
    const uint32_t p[4] = {d0, __builtin_amdgcn_alignbyte(d1, d0, 3), __builtin_amdgcn_alignbyte(d2, d1, 2), d2 >> 8};
    uint32_t y[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t t2 = __builtin_amdgcn_udot4(p[j] & 0x00ffffffu, K2, 0u, false);
        const uint32_t t1 = __builtin_amdgcn_udot4(p[j] & 0x00ffffffu, K1, t2 << 8, false);
        y[j] = __builtin_amdgcn_udot4(p[j] & 0x00ffffffu, K0, (t1 << 8) + (uint32_t)(HALF + (16 << SHIFT)), false) >> SHIFT;
    }
    return yuvpx::pack4(y[0], y[1], y[2], y[3]);
}
// chroma of pixels 0 and 2 of the quad row (the top-left pixels of its two
// 2x2 quads): U0 | U2 << 8 in the low half, V0 | V2 << 8 in the high half
__device__ __forceinline__ uint32_t chroma2_i420(uint32_t d0, uint32_t d1, uint32_t d2)
{
    using namespace yuvpx;
    const int b0 = d0 & 255, g0 = (d0 >> 8) & 255, r0 = (d0 >> 16) & 255;
    const int b2 = (d1 >> 16) & 255, g2 = d1 >> 24, r2 = d2 & 255;   // bytes 6, 7, 8
    return chroma_u(b0, g0, r0) | (chroma_u(b2, g2, r2) << 8) | (chroma_v(b0, g0, r0) << 16) |
           (chroma_v(b2, g2, r2) << 24);
}
// a gray pixel (R = G = B = u) has U = V = 128: both chroma rows of coefficients sum to 1
static_assert(yuvpx::CRU + yuvpx::CGU + yuvpx::CBU == 1 && yuvpx::CBU + yuvpx::CGV + yuvpx::CBV == 1,
              "gray chroma is 128");

#ifndef DVC_FRONT_WGS_YUV_OI   // 4:2:0 input, I420 outputs
#define DVC_FRONT_WGS_YUV_OI 4
#endif
#ifndef DVC_FRONT_WGS_B8   // fused 8x8 blocks: 3 workgroups a CU (4 spill 20 VGPRs)
#define DVC_FRONT_WGS_B8 3
#endif
template <int NW, int PF, int FMT, bool OUT, int OB = 4, bool OI = false>
__global__ void __launch_bounds__(64 * NW, OUT ? (OB == 8 ? DVC_FRONT_WGS_B8 : PF == 1 ? (FMT == DVC_FMT_BGR ? DVC_FRONT_WGS_BGR : OI ? DVC_FRONT_WGS_YUV_OI : FMT == DVC_FMT_I420 ? DVC_FRONT_WGS_I420 : DVC_FRONT_WGS_YUV) : DVC_FRONT_WGS_PF2) : 1) k_front(const uint8_t* __restrict__ bgr, int pitch, size_t fstride, SrcFmt sf,
                                                   int n, int chunk, const uint8_t* __restrict__ gray_in,
                                                   uint8_t* __restrict__ gray_out, int gs, uint64_t* __restrict__ mbits,
                                                   int W, int H, int WW, int ithresh, int xcd_bands, FrontOut fo)
{
    static_assert(!OUT || NW == 4 || NW == 8, "fused outputs: 16- or 32-row tiles");
    static_assert(!OUT || OB == 4 || (OB == 8 && NW == 4), "fused 8x8 blocks: 16-row tiles (64 blocks, 4 lanes each)");
    static_assert(!OI || (OUT && OB == 4 && NW == 4), "fused I420 outputs: 4x4 blocks, 16-row tiles");
    constexpr int FT_H = 4 * NW, FT_R = FT_H + 4, NT = 64 * NW;
    constexpr bool B8 = OUT && OB == 8;
    __shared__ uint32_t sg[FT_R][FT_Q];        // gray quads
    __shared__ uint2 sh[FT_R][FT_W / 4];       // horizontal Q8 sums, 4 x u16 per quad
    __shared__ __attribute__((aligned(16))) float s8[B8 ? 64 * DCT8_S : 1];   // OB = 8: the blocks' DCT planes
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // LDS row of this wave's j-th loaded row, and tile row of its i-th output row
    // (OUT: the 4 halo rows 0, 1, FT_H + 2, FT_H + 3 go to waves 0..3; a wave
    // past them has no 5th row: FT_R, never stored)
    auto lrow = [&](int j) {
        return OUT ? (j < 4 ? 2 + 4 * wave + j : (wave < 2 ? wave : (wave < 4 ? FT_H + wave : FT_R))) : wave + NW * j;
    };
    auto orow = [&](int i) { return OUT ? 4 * wave + i : wave + NW * i; };
    // XCD bands: blocks b, b+8, .. share an XCD (and its L2); the bijective remap
    // below deals each such group a contiguous run of (chunk, tile row, tile)
    // ids, so a tile's halo rows and halo quads are mostly its own XCD's lines
    // (the default raster gives an XCD a tile column: every left/right halo
    // quad then costs two 128-B lines fetched by another XCD)
    int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    if (xcd_bands) {
        const int nwg = gridDim.x * gridDim.y * gridDim.z;
        const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        const int q = nwg >> 3, r = nwg & 7, xcd = L & 7;
        const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (L >> 3);
        const int T = gridDim.x * gridDim.y;
        bz = id / T;
        by = (id - bz * T) / gridDim.x;
        bx = id - bz * T - by * gridDim.x;
    }
    const int x0 = bx * FT_W, y0 = by * FT_H;
    const int x = x0 + 4 * lane;
    const size_t mstride = (size_t)H * WW;
    const int t_first = bz * chunk, t_end = min(n, t_first + chunk);
    const int t_begin = bz == 0 ? 0 : t_first - 1;   // warm-up frame for c > 0
    const u16x2 bias = (u16x2)(unsigned short)(0x7fff - ithresh);   // ithresh in -1..255

    // Every load below is unconditional from a clamped, always-valid address
    // (the value is discarded where it is not needed): a conditional load makes
    // hipcc branch around it and drain vmcnt to 0 before the next one.
    // previous blurred gray of this lane's 4 output rows, as u16 pairs. The
    // quad holding px W-1 may be partial (W % 4): it is loaded in place (frame
    // rows are padded to 3 * gs bytes); quads past it reload the last quad.
    const int xc = x < W ? x : gs - 4;
    u16x2 pl[4], ph[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int y = min(y0 + orow(i), H - 1);
        const uint32_t v = *reinterpret_cast<const uint32_t*>(gray_in + (size_t)y * gs + xc);
        pl[i] = as_u16x2(__builtin_amdgcn_perm(0u, v, 0x0c010c00u));
        ph[i] = as_u16x2(__builtin_amdgcn_perm(0u, v, 0x0c030c02u));
    }
    // BGR of the FT_R halo rows: wave w loads rows w, w+NW, ..; lane l its quad
    // l (12 contiguous bytes); rows past FT_R (NW > 4) reload a valid row and
    // are dropped. The 2 x FT_R halo quads left / right of the tile are loaded
    // and converted once, by threads 0 .. 2*FT_R-1 (thread 2r + side).
    // Addresses are a uniform frame base + 32-bit per-lane offsets. A 4:2:0
    // surface (FMT != BGR): the quad's luma dword and its chroma (I420: a u16
    // of U and one of V, dv bytes apart; NV12: one UVUV dword) instead.
    constexpr bool YUV = FMT != DVC_FMT_BGR;
    constexpr int NR = (FT_R + NW - 1) / NW;
    uint32_t off[NR], coff[NR];
    auto row_off = [&](int y, int xq, uint32_t& o, uint32_t& co) {
        if constexpr (YUV) {
            o = (uint32_t)(y * pitch + xq);
            co = (uint32_t)(sf.uoff + (size_t)(y >> 1) * sf.cpitch + (FMT == DVC_FMT_NV12 ? xq : xq >> 1));
        } else {
            o = (uint32_t)(y * pitch + 3 * xq);
            co = 0;
        }
    };
#pragma unroll
    for (int j = 0; j < NR; ++j) row_off(reflect1(y0 - 2 + min(lrow(j), FT_R - 1), H), xc, off[j], coff[j]);
    const uint32_t dv = (uint32_t)(sf.voff - sf.uoff);
    const bool halo_wave = __builtin_amdgcn_readfirstlane(wave) < (2 * FT_R + 63) / 64;   // scalar branch
    const bool halo = halo_wave && tid < 2 * FT_R;
    const int hr = min(tid >> 1, FT_R - 1), hs = tid & 1;
    const int hx = x0 + (hs ? FT_W : -4);
    uint32_t hoff, hcoff;
    row_off(reflect1(y0 - 2 + min(hr, FT_R - 1), H), hx >= 0 && hx < W ? hx : xc, hoff, hcoff);
    // one frame's quads in registers; PF sets in flight (PF - 1 frames of
    // prefetch beyond the one being converted)
    struct Quads { uint32_t v0[NR], v1[NR], v2[NR], h0, h1, h2; };
    auto load_quad = [&](const uint8_t* f, uint32_t o, uint32_t co, uint32_t& a, uint32_t& b, uint32_t& c) {
        if constexpr (FMT == DVC_FMT_BGR) {
            const uint3 q = *reinterpret_cast<const uint3*>(f + o);
            a = q.x; b = q.y; c = q.z;
        } else if constexpr (FMT == DVC_FMT_NV12) {
            a = *reinterpret_cast<const uint32_t*>(f + o);
            b = *reinterpret_cast<const uint32_t*>(f + co);
            c = 0;
        } else {
            a = *reinterpret_cast<const uint32_t*>(f + o);
            b = *reinterpret_cast<const uint16_t*>(f + co);
            c = *reinterpret_cast<const uint16_t*>(f + co + dv);
        }
    };
    // the offsets pass through voff in place once per frame (no copies): every
    // load and store below is a uniform base + a 32-bit VGPR offset
    auto load = [&](Quads& qs, const uint8_t* f) {
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            off[j] = voff(off[j]);
            if constexpr (YUV) coff[j] = voff(coff[j]);
            load_quad(f, off[j], coff[j], qs.v0[j], qs.v1[j], qs.v2[j]);
        }
        hoff = voff(hoff);
        if constexpr (YUV) hcoff = voff(hcoff);
        load_quad(f, hoff, hcoff, qs.h0, qs.h1, qs.h2);
    };
    Quads qa, qb;
    load(qa, bgr + (size_t)t_begin * fstride);
    if constexpr (PF == 2) load(qb, bgr + (size_t)min(t_begin + 1, t_end - 1) * fstride);

    // BORDER_REFLECT_101 columns: the halo quad left of x = 0 and px W, W+1
    // (when they lie in this tile's LDS columns) are copies of px 4..1 and
    // W-2, W-3, fixed up in LDS after the straight loads land. LDS byte b of
    // quad column c holds px x0 - 4 + 4c + b.
    const bool fix_l = x0 == 0;
    const int iW = W - x0 + 4;                    // LDS byte index of px W
    const bool fix_r = iW < 4 * FT_Q;
    constexpr int FB = 64 * ((FT_R + 63) / 64);   // first thread of the right fix-up (after the left one's)
    constexpr uint32_t K5 = 1u | (4u << 8) | (6u << 16) | (4u << 24);
    // OUT: this lane's block lies inside the frame (partial edge blocks are
    // k_out_gen's) and the frame is one of the chunk's (not its warm-up)
    // (OB = 8: the lane's 4x4 quarter lies in a full 8x8 block)
    const bool full_blk = OUT && (OB == 8 ? (x & ~7) + 8 <= W && ((y0 + 4 * wave) & ~7) + 8 <= H
                                          : x + 4 <= W && y0 + 4 * wave + 4 <= H);
    // OB = 8: this thread's quarter of block q8 (32 x 2 blocks a tile): rows 2 r8,
    // 2 r8 + 1; the block's compressed rows go out from these lanes
    const int q8 = threadIdx.x >> 2, r8 = threadIdx.x & 3, bx8 = q8 & 31, by8 = q8 >> 5;
    const bool full8 = B8 && x0 + 8 * bx8 + 8 <= W && y0 + 8 * by8 + 8 <= H;
    uint32_t o8[2];
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
        o8[ii] = B8 ? (uint32_t)((size_t)(y0 + 8 * by8 + 2 * r8 + ii) * fo.opitch + 3 * (size_t)(x0 + 8 * bx8)) : 0u;
    // OUT rows and motion-bit words: per-lane 32-bit offsets from the frame's
    // wave-uniform base (through voff once per frame, like the loads)
    uint32_t oro[4], mwo[4], cro[2];   // OI: oro = luma rows, cro = the U rows of row pairs 0-1, 2-3
    const uint32_t cq = OI ? (uint32_t)((W >> 1) * (H >> 1)) : 0u;   // U plane -> V plane
#pragma unroll
    for (int k = 0; k < 2; ++k)
        cro[k] = OI ? (uint32_t)((size_t)W * H + (size_t)((y0 + 4 * wave) / 2 + k) * (W >> 1) + (x >> 1)) : 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        oro[i] = OI  ? (uint32_t)((size_t)(y0 + 4 * wave + i) * W + x)
                 : OUT ? (uint32_t)((size_t)(y0 + 4 * wave + i) * fo.opitch + 3 * (size_t)x) : 0u;
        mwo[i] = (uint32_t)(min(y0 + orow(i), H - 1) * WW + min((x0 >> 6) + (lane >> 4), WW - 1)) * 8u + ((lane >> 1) & 4u);
    }
    auto frame = [&](Quads& qs, int t) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if constexpr (OUT) oro[i] = voff(oro[i]);
            mwo[i] = voff(mwo[i]);
        }
        if constexpr (OI) {
            cro[0] = voff(cro[0]);
            cro[1] = voff(cro[1]);
        }
        if constexpr (B8) {
            o8[0] = voff(o8[0]);
            o8[1] = voff(o8[1]);
        }
        // OUT: the block's 4 rows as BGR (4:2:0 surfaces converted once, for
        // both the gray and the overlay); other rows straight to gray
        uint32_t cb[4][3];
        if constexpr (OUT) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if constexpr (YUV) {
                    quad_bgr<FMT>(qs.v0[j], qs.v1[j], qs.v2[j], cb[j]);
                } else {
                    cb[j][0] = qs.v0[j];
                    cb[j][1] = qs.v1[j];
                    cb[j][2] = qs.v2[j];
                }
                sg[lrow(j)][lane + 1] = gray4_dot(cb[j][0], cb[j][1], cb[j][2]);
                if constexpr (OI) {   // the frame as BGR2YUV_I420, row by row (rows 4 wave + j: even rows carry the chroma)
                    if (fo.ov && full_blk && t >= t_first) {
                        uint8_t* o = fo.ov + (size_t)t * fo.ostride;
                        __builtin_nontemporal_store(luma4_i420(cb[j][0], cb[j][1], cb[j][2]),
                                                    reinterpret_cast<uint32_t*>(o + oro[j]));
                        if (!(j & 1)) {
                            const uint32_t uv = chroma2_i420(cb[j][0], cb[j][1], cb[j][2]);
                            __builtin_nontemporal_store((uint16_t)uv, reinterpret_cast<uint16_t*>(o + cro[j >> 1]));
                            __builtin_nontemporal_store((uint16_t)(uv >> 16),
                                                        reinterpret_cast<uint16_t*>(o + (cro[j >> 1] + cq)));
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int j = OUT ? 4 : 0; j < NR; ++j)
            if (NR * NW == FT_R || lrow(j) < FT_R)
                sg[lrow(j)][lane + 1] = quad_gray<FMT>(qs.v0[j], qs.v1[j], qs.v2[j]);
        if constexpr (OUT) {
            // overlay := the frame (a static block has no acc > 127 pixel); the
            // registers are reloaded with frame t + PF right after the barrier
            if (!OI && fo.ov && full_blk && t >= t_first) {   // (OI: written row by row above)
                uint8_t* o = fo.ov + (size_t)t * fo.ostride;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    uint32_t* r = reinterpret_cast<uint32_t*>(o + oro[j]);
                    __builtin_nontemporal_store(cb[j][0], r);
                    __builtin_nontemporal_store(cb[j][1], r + 1);
                    __builtin_nontemporal_store(cb[j][2], r + 2);
                }
            }
        }
        if (halo_wave) {
            const uint32_t gh = quad_gray<FMT>(qs.h0, qs.h1, qs.h2);
            if (halo) sg[hr][hs ? FT_Q - 1 : 0] = gh;
        }
        if (fix_l || fix_r) {            // uniform per workgroup
            __syncthreads();
            if (tid < FT_R) {
                if (fix_l) {             // px -4..-1 = px 4, 3, 2, 1
                    const uint32_t a = sg[tid][1], b = sg[tid][2];
                    sg[tid][0] = (b & 255) | (((a >> 24) & 255) << 8) | (((a >> 16) & 255) << 16) | (((a >> 8) & 255) << 24);
                }
            } else if (tid >= FB && tid < FB + FT_R) {
                if (fix_r) {             // px W, W+1 = px W-2, W-3 (later bytes are never read)
                    uint8_t* row = reinterpret_cast<uint8_t*>(&sg[tid - FB][0]);
                    const uint8_t a = row[iW - 2], b = row[iW - 3];
                    row[iW] = a;
                    if (iW + 1 < 4 * FT_Q) row[iW + 1] = b;
                }
            }
        }
        __syncthreads();
        if constexpr (B8) {
            // OB = 8: the compressed blocks, before the next frame's loads are
            // issued (their registers are free here; sg holds this frame until
            // the next barrier). Every lane runs its block's passes (the
            // wave-level LDS ordering needs the whole quad); only full blocks
            // are stored
            if (fo.cp && t >= t_first) {
                float xg[2][8], yo[2][8];
#pragma unroll
                for (int ii = 0; ii < 2; ++ii)
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj) {   // rows 2 r8, 2 r8 + 1 of block q8: two quads each
                        const uint32_t gw = sg[2 + 8 * by8 + 2 * r8 + ii][1 + 2 * bx8 + jj];
#pragma unroll
                        for (int j = 0; j < 4; ++j) xg[ii][4 * jj + j] = (float)((int)((gw >> (8 * j)) & 255u) - 128);
                    }
                dct8_quad(s8 + q8 * DCT8_S, r8, xg, fo.quant, fo.qinv, yo);
                if (full8) {
                    uint8_t* o = fo.cp + (size_t)t * fo.ostride;
#pragma unroll
                    for (int ii = 0; ii < 2; ++ii) {
                        uint32_t cw[6];
#pragma unroll
                        for (int h4 = 0; h4 < 2; ++h4) {
                            uint32_t u[4];
#pragma unroll
                            for (int j = 0; j < 4; ++j)   // clip to [0, 255], truncating uint8 cast
                                u[j] = (uint32_t)__builtin_amdgcn_fmed3f(yo[ii][4 * h4 + j] + 128.0f, 0.0f, 255.0f);
                            gray_bgr4(u[0], u[1], u[2], u[3], &cw[3 * h4]);
                        }
                        uint32_t* r = reinterpret_cast<uint32_t*>(o + o8[ii]);
#pragma unroll
                        for (int d = 0; d < 6; ++d) __builtin_nontemporal_store(cw[d], r + d);
                    }
                }
            }
        }
        // frame t + PF into the set just converted (the last frames reload
        // themselves: an unconditional load)
        load(qs, bgr + (size_t)min(t + PF, t_end - 1) * fstride);
        // OUT: the block's gray quads (this frame's sg is rewritten only after
        // the barrier below)
        uint32_t gq[4];
        if constexpr (OUT && !B8) {
#pragma unroll
            for (int i = 0; i < 4; ++i) gq[i] = sg[2 + 4 * wave + i][lane + 1];
        }

#pragma unroll
        for (int i = 0; i < (FT_R * 64 + NT - 1) / NT; ++i) {
            const int it = tid + NT * i;
            if (it < FT_R * 64) {
                const int r = it >> 6, q = it & 63;
                const uint32_t a = sg[r][q], b = sg[r][q + 1], c = sg[r][q + 2];
                // window bytes a2 a3 b0 b1 b2 b3 c0 c1: output j = dot(W[j..j+3], K5) + W[j+4]
                const uint32_t D0 = __builtin_amdgcn_alignbyte(b, a, 2), D1 = __builtin_amdgcn_alignbyte(b, a, 3);
                const uint32_t D3 = __builtin_amdgcn_alignbyte(c, b, 1), D4 = __builtin_amdgcn_alignbyte(c, b, 2);
                const uint32_t q0 = __builtin_amdgcn_udot4(D0, K5, D1 >> 24, false);
                const uint32_t q1 = __builtin_amdgcn_udot4(D1, K5, b >> 24, false);
                const uint32_t q2 = __builtin_amdgcn_udot4(b, K5, D3 >> 24, false);
                const uint32_t q3 = __builtin_amdgcn_udot4(D3, K5, D4 >> 24, false);
                sh[r][q] = make_uint2(__builtin_amdgcn_perm(q1, q0, 0x05040100u), __builtin_amdgcn_perm(q3, q2, 0x05040100u));
            }
        }
        __syncthreads();

        uint64_t* mb = mbits + (size_t)t * mstride;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int rr = orow(i), y = y0 + rr;
            const uint2 a0 = sh[rr][lane], a1 = sh[rr + 1][lane], a2 = sh[rr + 2][lane], a3 = sh[rr + 3][lane],
                        a4 = sh[rr + 4][lane];
            // 16-bit lanes: sum <= 16 * 4080 = 65280, packed adds cannot carry across halves
            // 4 * (a1 + a3) + (6 * a2 + (a0 + a4)) as two v_pk_mad_u16 (the
            // compiler turns * 4 back into a shift and an add)
            auto vsum = [](uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3, uint32_t b4) {
                const uint32_t m = as_u32(as_u16x2(b2) * (u16x2)6 + (as_u16x2(b0) + as_u16x2(b4)));
                const uint32_t p = as_u32(as_u16x2(b1) + as_u16x2(b3));
                uint32_t r;
                asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(r) : "v"(p), "s"(0x00040004u), "v"(m));
                return as_u16x2(r);
            };
            const u16x2 sx = vsum(a0.x, a1.x, a2.x, a3.x, a4.x);
            const u16x2 sy = vsum(a0.y, a1.y, a2.y, a3.y, a4.y);
            const u16x2 gl = (sx + (u16x2)128) >> 8, gh = (sy + (u16x2)128) >> 8;
            const u16x2 dl = __builtin_elementwise_max(gl, pl[i]) - __builtin_elementwise_min(gl, pl[i]);
            const u16x2 dh = __builtin_elementwise_max(gh, ph[i]) - __builtin_elementwise_min(gh, ph[i]);
            const uint32_t xl = as_u32(dl + bias) & 0x80008000u, xh = as_u32(dh + bias) & 0x80008000u;
            const uint32_t xm = (xl >> 15) | (xh >> 13);          // px 0..3 at bits 0, 16, 2, 18
            uint32_t nib = (xm | (xm >> 15)) & 15u;
            pl[i] = gl;
            ph[i] = gh;
            if (y >= H || x >= W || t < t_first) nib = 0;
            if (x + 4 > W) nib &= (1u << max(W - x, 0)) - 1u;   // partial quad: px >= W are not pixels
            // 8 lanes x 4 px = one 32-bit half of a mask word: OR-reduce within
            // each group of 8 lanes with DPP (quad_perm xor 1, xor 2, row_half_mirror)
            uint32_t w = nib << (4 * (lane & 7));
            w |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0xB1, 0xF, 0xF, false);
            w |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x4E, 0xF, 0xF, false);
            w |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x141, 0xF, 0xF, false);
            const int wi = (x0 >> 6) + (lane >> 4);
            if ((lane & 7) == 0 && y < H && wi < WW && t >= t_first)
                *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(mb) + mwo[i]) = w;
        }
        // OUT: compressed := the block as static (fd:117-130): Y' = trunc(clip(
        // IDCT(rint(DCT(Y - 128) / q) q) + 128)), Cr = Cb = 128 -> (Y', Y', Y')
        if constexpr (OUT && !B8) {
            if (fo.cp && full_blk && t >= t_first) {
                float X[16];
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) X[4 * i + j] = (float)((int)((gq[i] >> (8 * j)) & 255u) - 128);
                block_dct_quant_pk<4>(X, kDct4, fo.quant, fo.qinv);
                uint8_t* o = fo.cp + (size_t)t * fo.ostride;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    uint32_t u[4], cw[3];
#pragma unroll
                    for (int j = 0; j < 4; ++j)   // clip to [0, 255], truncating uint8 cast
                        u[j] = (uint32_t)__builtin_amdgcn_fmed3f(X[4 * i + j] + 128.0f, 0.0f, 255.0f);
                    if constexpr (OI) {   // Y of (u, u, u); U = V = 128
                        uint32_t yv[4];
#pragma unroll
                        for (int j = 0; j < 4; ++j) yv[j] = yuvpx::luma((int)u[j], (int)u[j], (int)u[j]);
                        __builtin_nontemporal_store(yuvpx::pack4(yv[0], yv[1], yv[2], yv[3]),
                                                    reinterpret_cast<uint32_t*>(o + oro[i]));
                        if (!(i & 1)) {
                            __builtin_nontemporal_store((uint16_t)0x8080u, reinterpret_cast<uint16_t*>(o + cro[i >> 1]));
                            __builtin_nontemporal_store((uint16_t)0x8080u,
                                                        reinterpret_cast<uint16_t*>(o + (cro[i >> 1] + cq)));
                        }
                    } else {
                        gray_bgr4(u[0], u[1], u[2], u[3], cw);
                        uint32_t* r = reinterpret_cast<uint32_t*>(o + oro[i]);
                        __builtin_nontemporal_store(cw[0], r);
                        __builtin_nontemporal_store(cw[1], r + 1);
                        __builtin_nontemporal_store(cw[2], r + 2);
                    }
                }
            }
        }
    };
    if constexpr (PF == 2) {
        for (int t = t_begin; t < t_end; t += 2) {
            frame(qa, t);
            if (t + 1 < t_end) frame(qb, t + 1);   // uniform
        }
    } else {
        for (int t = t_begin; t < t_end; ++t) frame(qa, t);
    }
    // frame n-1's blurred gray becomes the previous gray of the next batch
    if (t_end == n) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int y = y0 + orow(i);
            if (y < H && x < W)
                *reinterpret_cast<uint32_t*>(gray_out + (size_t)y * gs + x) =
                    __builtin_amdgcn_perm(as_u32(ph[i]), as_u32(pl[i]), 0x06040200u);
        }
    }
}

// ------------------------------------------------------------------- band ---
// One workgroup (256 threads) per band of BAND_ROWS = 16 rows, a group of BG =
// 16 lanes per row: build the row's run index (start/end bit words + prefix
// counts, in LDS) straight from the bit mask and write its runs to global,
// then union-find over the band's runs (8-connected) and gaps (4-connected;
// gaps on the image border joined to the OUTSIDE node), flatten, and publish
// every run/gap's band-local root as a global id.
// The band's nodes are numbered compactly from its actual run counts n_r:
// 0 = OUTSIDE, run (r,k) = 1 + roff[r] + k, gap (r,k) = 1 + RT + goff[r] + k
// (roff / goff prefix sums of n_r / n_r + 1, RT = sum n_r) — order-preserving
// against the global ids, so "root = smallest id" carries over. When the band
// has more nodes than the LDS budget (`budget`, e.g. pure-noise masks), the same
// unions run on the global parent arrays instead (monotone atomicMin links).
// Small workgroups (4 waves, ~14 KB LDS at 1080p) keep the band stage schedulable
// beside the streaming kernels of the other two streams. Dynamic LDS: band_lds().
#ifndef DVC_BAND_BG
#define DVC_BAND_BG 16
#endif
constexpr int BG = DVC_BAND_BG, BAND_ROWS = 16, BAND_NT = BG * BAND_ROWS;

__global__ void __launch_bounds__(BAND_NT) k_band(CclBufs cb, RowGeom g, int budget)
{
    constexpr int BH = BAND_ROWS;
    const CclBufs fb = cb.frame(blockIdx.y, g);
    const uint64_t* __restrict__ mbits = fb.mbits;
    uint16_t* __restrict__ rs = fb.rs;
    uint16_t* __restrict__ re = fb.re;
    uint32_t* __restrict__ nfg = fb.nfg;
    uint32_t* fpar = fb.fpar;
    uint32_t* gpar = fb.gpar;
    uint32_t* __restrict__ area2 = fb.area2;
    unsigned long long* __restrict__ stats = fb.stats;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    const int WW = g.WW, W = g.W;
    uint64_t* l_st = lds;
    uint64_t* l_en = l_st + BH * WW;
    uint16_t* l_ps = reinterpret_cast<uint16_t*>(l_en + BH * WW);
    uint16_t* l_pe = l_ps + BH * (WW + 1);
    uint32_t* lp = reinterpret_cast<uint32_t*>(l_pe + BH * (WW + 1) + 2);   // 4-byte aligned
    __shared__ int s_n[BH], s_roff[BH + 1], s_goff[BH + 1];
    const int slot = threadIdx.x / BG, sl = threadIdx.x & (BG - 1);
    const int y0 = blockIdx.x * BH, y = y0 + slot;
    const bool act = y < g.H;
    const uint32_t CAP = (uint32_t)g.CAP;
    // the band's node ranges (CclBufs::rowb): runs RB0.., gaps GB0..
    const uint32_t RB0 = (uint32_t)blockIdx.x * BH * CAP, GB0 = 1u + (uint32_t)blockIdx.x * BH * (CAP + 1);
    uint64_t* st = l_st + slot * WW;
    uint64_t* en = l_en + slot * WW;
    uint16_t* ps = l_ps + slot * (WW + 1);
    uint16_t* pe = l_pe + slot * (WW + 1);

    // ---- phase 1: run index of row y in LDS
    int n = 0;
    unsigned long long motion = 0;
    if (act) n = build_row_idx_g<BG>(mbits + (size_t)y * WW, WW, W, st, en, ps, pe, &motion);
    if (sl == 0) s_n[slot] = act ? n : 0;
    for (int d = 32; d >= 1; d >>= 1) motion += __shfl_xor(motion, d, 64);   // the wave's 4 rows
    if ((threadIdx.x & 63) == 0 && motion) atomicAdd(stats + STAT_SLOT(y) * 4 + 1, motion);
    __syncthreads();
    if (threadIdx.x == 0) {
        int ro = 0, go = 0;
        for (int r = 0; r < BH; ++r) {
            s_roff[r] = ro;
            s_goff[r] = go;
            ro += s_n[r];
            go += s_n[r] + 1;
        }
        s_roff[BH] = ro;
        s_goff[BH] = go;
    }
    __syncthreads();
    const int RT = s_roff[BH];
    const uint32_t base = RB0 + (uint32_t)s_roff[slot], gbase = GB0 + (uint32_t)s_goff[slot];
    if (act && sl == 0) {
        fb.rowb[2 * y] = base;
        fb.rowb[2 * y + 1] = gbase;
    }
    if (RT == 0) {   // uniform: a band without runs — each row is one border gap, outside
        if (act && sl == 0) {
            gpar[gbase] = 0u;
            nfg[y] = 0u;
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) gpar[0] = 0;
        return;
    }
    // the row's runs to global (later kernels), packed after the band's earlier rows
    if (act)
        for (int i = sl; i < WW; i += BG) {
            uint64_t s = st[i], e = en[i];
            int ks = ps[i], ke = pe[i];
            while (s) { rs[base + ks++] = (uint16_t)(i * 64 + __builtin_ctzll(s)); s &= s - 1; }
            while (e) { re[base + ke++] = (uint16_t)(i * 64 + __builtin_ctzll(e)); e &= e - 1; }
        }
    const bool local = 1 + RT + s_goff[BH] <= budget;   // uniform
    const bool left_bg = act && !(st[0] & 1ull);
    const bool right_bg = act && !((en[(W - 1) >> 6] >> ((W - 1) & 63)) & 1ull);
    auto border_gap = [&](int k) {
        const bool nonempty = (k == 0) ? left_bg : (k == n ? right_bg : true);
        return nonempty && (y == 0 || y == g.H - 1 || k == 0 || k == n);
    };

    if (local) {
        const uint32_t FG = 1 + s_roff[slot], GP = 1 + RT + s_goff[slot];
        if (act) {
            for (int k = sl; k < n; k += BG) lp[FG + k] = FG + k;
            for (int k = sl; k <= n; k += BG) lp[GP + k] = border_gap(k) ? 0u : GP + k;
        }
        if (threadIdx.x == 0) lp[0] = 0;
        __syncthreads();
        // ---- phase 2: unions between the band's consecutive rows, in LDS
        if (act && slot + 1 < BH && y + 1 < g.H) {
            const uint32_t f1 = 1 + s_roff[slot + 1], q1 = 1 + RT + s_goff[slot + 1];
            const RowIdx r0{st, en, ps, pe}, r1{st + WW, en + WW, ps + WW + 1, pe + WW + 1};
            row_pair_unions<BG>(W, WW, r0, n, r1,
                                [&](int i, int j) { lunion(lp, FG + i, f1 + j); },
                                [&](int i, int j) { lunion(lp, GP + i, q1 + j); });
        }
        __syncthreads();
        // ---- phase 3: flatten; publish band-local roots as global ids (the
        // local numbering is the band's packed global numbering minus RB0 / GB0)
        if (act) {
            for (int k = sl; k < n; k += BG) {
                fpar[base + k] = RB0 + (lfind(lp, FG + k) - 1);
                area2[base + k] = 0;
            }
            for (int k = sl; k <= n; k += BG) {
                const uint32_t r = lfind(lp, GP + k);
                gpar[gbase + k] = r != 0 ? GB0 + (r - 1 - RT) : 0u;
            }
        }
    } else {
        // over budget: identity parents in global memory, unions with atomicMin links
        if (act) {
            for (int k = sl; k < n; k += BG) {
                fpar[base + k] = base + k;
                area2[base + k] = 0;
            }
            for (int k = sl; k <= n; k += BG) gpar[gbase + k] = border_gap(k) ? 0u : gbase + k;
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) gpar[0] = 0;
        __threadfence_block();
        __syncthreads();
        if (act && slot + 1 < BH && y + 1 < g.H) {
            const uint32_t b1 = RB0 + (uint32_t)s_roff[slot + 1], g1 = GB0 + (uint32_t)s_goff[slot + 1];
            const RowIdx r0{st, en, ps, pe}, r1{st + WW, en + WW, ps + WW + 1, pe + WW + 1};
            row_pair_unions<BG>(W, WW, r0, n, r1,
                                [&](int i, int j) { uf_union(fpar, base + i, b1 + j); },
                                [&](int i, int j) { uf_union(gpar, gbase + i, g1 + j); });
        }
    }
    if (act && sl == 0) nfg[y] = (uint32_t)n;
    if (blockIdx.x == 0 && threadIdx.x == 0) gpar[0] = 0;  // the OUTSIDE node is its own root
}

// Contour-filter kernels after k_band give each row (seam) a group of lanes of
// its own and synchronise only within the wave (each group its own LDS slice,
// wave_sync_lds in dvc_device.h).

// ------------------------------------------------------------------ merge ---
// One group of MG lanes per band seam (rows b*BH-1 and b*BH): run indexes of
// both rows in LDS, then global unions of the band roots with monotone
// atomicMin links. 64/MG seams per wave, each its own dependency chain.
#ifndef DVC_MERGE_MG
#define DVC_MERGE_MG 64
#endif
constexpr int MG = DVC_MERGE_MG;   // only ~H/16 seams per frame: a whole wave each keeps enough waves in flight

__host__ __device__ constexpr size_t merge_lds_words(int WW) { return (size_t)4 * WW + (size_t)(WW + 1); }

__global__ void __launch_bounds__(256) k_merge(CclBufs cb, RowGeom g, int BH)
{
    const CclBufs fb = cb.frame(blockIdx.y, g);
    uint32_t* fpar = fb.fpar;
    uint32_t* gpar = fb.gpar;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    const int WW = g.WW, slot = threadIdx.x / MG, sl = threadIdx.x & (MG - 1);
    const int y = (blockIdx.x * (256 / MG) + slot + 1) * BH - 1;
    const bool act = y + 1 < g.H;
    uint64_t* st = lds + (size_t)slot * merge_lds_words(WW);
    uint64_t* en = st + 2 * WW;
    uint16_t* ps = reinterpret_cast<uint16_t*>(en + 2 * WW);
    uint16_t* pe = ps + 2 * (WW + 1);
    int n0 = 0;
    if (act) {
        n0 = build_row_idx_g<MG>(fb.mbits + (size_t)y * WW, WW, g.W, st, en, ps, pe, nullptr);
        build_row_idx_g<MG>(fb.mbits + (size_t)(y + 1) * WW, WW, g.W, st + WW, en + WW, ps + WW + 1, pe + WW + 1,
                            nullptr);
    }
    wave_sync_lds();
    if (!act) return;
    const uint32_t b0 = fb.rowb[2 * y], b1 = fb.rowb[2 * y + 2], g0 = fb.rowb[2 * y + 1], g1 = fb.rowb[2 * y + 3];
    for (int i = sl; i < n0; i += MG) {
        const int a = select_k(st, ps, WW, i), b = select_k(en, pe, WW, i);
        const int j0 = rank_le(en + WW, pe + WW + 1, WW, a - 2), j1 = rank_le(st + WW, ps + WW + 1, WW, b + 1);
        for (int j = j0; j < j1; ++j) uf_union(fpar, b0 + i, b1 + j);
    }
    for (int i = sl; i <= n0; i += MG) {
        const int a = i == 0 ? 0 : select_k(en, pe, WW, i - 1) + 1;
        const int b = i == n0 ? g.W - 1 : select_k(st, ps, WW, i) - 1;
        if (a > b) continue;
        const int j0 = rank_le(st + WW, ps + WW + 1, WW, a), j1 = rank_le(en + WW, pe + WW + 1, WW, b - 1);
        for (int j = j0; j <= j1; ++j) uf_union(gpar, g0 + i, g1 + j);
    }
}

// The per-row kernels below (paint, resolve, area) give each row a group of
// CG lanes — CG = 16: 4 rows per wave, 16 per workgroup; CG = 8 (batches of
// >= 64 frames, launch_ccl): 8 rows per wave, 32 per workgroup — so one wave
// carries several independent global-memory dependency chains (the union-find
// walks); a row's runs are strided over its CG lanes. LDS: one mask row per group.
template <int CG> constexpr int cg_rows() { return 4 * (64 / CG); }

template <int CG>
__device__ __forceinline__ int group_incl_scan(int v)
{
    const int sl = threadIdx.x & (CG - 1);
#pragma unroll
    for (int d = 1; d < CG; d <<= 1) {
        const int t = __shfl_up(v, d, CG);
        if (sl >= d) v += t;
    }
    return v;
}

// ------------------------------------------------------------------ paint ---
// The kept (filtered) mask, fd:101-104 — every run of a kept component plus
// the holes between its runs (drawContours FILLED).
template <int CG>
__global__ void __launch_bounds__(256) k_paint(CclBufs cb, RowGeom g, int64_t min_area2)
{
    const CclBufs fb = cb.frame(blockIdx.y, g);
    const uint16_t* __restrict__ rs = fb.rs;
    const uint16_t* __restrict__ re = fb.re;
    const uint32_t* __restrict__ nfg = fb.nfg;
    const uint32_t* __restrict__ fpar = fb.fpar;
    const uint8_t* __restrict__ gE = fb.gE;
    const uint32_t* __restrict__ area2 = fb.area2;
    uint64_t* __restrict__ kbits = fb.kbits;
    extern __shared__ __attribute__((aligned(16))) unsigned long long lds_k[];
    const int slot = threadIdx.x / CG, sl = threadIdx.x & (CG - 1);
    const int y = blockIdx.x * cg_rows<CG>() + slot;
    const bool act = y < g.H;
    unsigned long long* s_k = lds_k + (size_t)slot * g.WW;
    if (act)
        for (int w = sl; w < g.WW; w += CG) s_k[w] = 0ull;
    wave_sync_lds();
    if (act) {
        const int n = (int)nfg[y];
        const uint32_t base = fb.rowb[2 * y];
        const uint8_t* ge = gE + (fb.rowb[2 * y + 1] - 1);   // gap node g at gE[g - 1]
        for (int k = sl; k < n; k += CG) {
            const uint32_t root = fpar[base + k];
            if (!((int64_t)area2[root] > min_area2)) continue;  // contourArea > min_area
            const int e = re[base + k];
            paint_bits(s_k, 0, g.WW, rs[base + k], e);
            if (k + 1 < n && !ge[k + 1]) paint_bits(s_k, 0, g.WW, e + 1, (int)rs[base + k + 1] - 1);
        }
    }
    wave_sync_lds();
    // rows without kept bits are only flagged (fb.kocc): most rows of a
    // surveillance frame, whose zero words would cost a write here and a read
    // in the dilation
    unsigned long long any = 0;
    if (act)
        for (int w = sl; w < g.WW; w += CG) any |= s_k[w];
    for (int d = 1; d < CG; d <<= 1) any |= __shfl_xor(any, d, CG);
    if (act && (any || !fb.kocc || fb.kfull))
        for (int w = sl; w < g.WW; w += CG) kbits[(size_t)y * g.WW + w] = s_k[w];
    if (act && sl == 0 && fb.kocc) fb.kocc[y] = any ? 1 : 0;
}

// ---------------------------------------------------------------- resolve ---
// Gaps whose root is OUTSIDE are E; the rest are holes: painted into the
// filled row F = not E, and the runs either side of a hole united (the
// component inside a hole of another joins the external one enclosing it).
template <int CG>
__global__ void __launch_bounds__(256) k_resolve(CclBufs cb, RowGeom g)
{
    const CclBufs fb = cb.frame(blockIdx.y, g);
    const uint16_t* __restrict__ rs = fb.rs;
    const uint16_t* __restrict__ re = fb.re;
    const uint32_t* __restrict__ nfg = fb.nfg;
    uint32_t* fpar = fb.fpar;
    uint32_t* gpar = fb.gpar;
    uint8_t* __restrict__ gE = fb.gE;
    const uint64_t* __restrict__ mbits = fb.mbits;
    uint64_t* __restrict__ fbits = fb.fbits;
    extern __shared__ __attribute__((aligned(16))) unsigned long long lds_r[];
    const int slot = threadIdx.x / CG, sl = threadIdx.x & (CG - 1);
    const int y = blockIdx.x * cg_rows<CG>() + slot;
    const bool act = y < g.H;
    unsigned long long* s_f = lds_r + (size_t)slot * g.WW;
    // a row without runs is one gap touching both image borders: outside (E),
    // its filled row is zero — k_area knows that from nfg and never reads it
    const int n = act ? (int)nfg[y] : 0;
    if (n)
        for (int w = sl; w < g.WW; w += CG) s_f[w] = mbits[(size_t)y * g.WW + w];
    wave_sync_lds();
    // (no runs: the row's one gap is the border gap k_band already tied to
    // OUTSIDE, and no kernel reads its gE)
    if (n) {
        const uint32_t base = fb.rowb[2 * y], gbase = fb.rowb[2 * y + 1];
        for (int k = sl; k <= n; k += CG) {
            const int a = k == 0 ? 0 : (int)re[base + k - 1] + 1;
            const int b = k == n ? g.W - 1 : (int)rs[base + k] - 1;
            uint8_t e = 1;
            if (a <= b) {
                const uint32_t r = uf_find(gpar, gbase + k);
                atomicMin(gpar + gbase + k, r);
                e = r == 0;
                if (!e) {  // a hole: interior gap, both neighbours are runs of this row
                    uf_union(fpar, base + k - 1, base + k);
                    paint_bits(s_f, 0, g.WW, a, b);
                }
            }
            gE[gbase - 1 + k] = e;
        }
    }
    wave_sync_lds();
    if (n)
        for (int w = sl; w < g.WW; w += CG) fbits[(size_t)y * g.WW + w] = s_f[w];
}

// ------------------------------------------------------------------- area ---
// Row y with F row y+1 staged in LDS. 2*area per filled run:
//   2*popc(F'[s..e]) - F'(s) - F'(e) + [F'(s-1)&F'(s)] + [F'(e)&F'(e+1)]
// (F' = row y+1), split additively over the runs and holes of the filled run.
template <int CG>
__global__ void __launch_bounds__(256) k_area(CclBufs cb, RowGeom g)
{
    const CclBufs fb = cb.frame(blockIdx.y, g);
    const uint16_t* __restrict__ rs = fb.rs;
    const uint16_t* __restrict__ re = fb.re;
    const uint32_t* __restrict__ nfg = fb.nfg;
    uint32_t* fpar = fb.fpar;
    const uint8_t* __restrict__ gE = fb.gE;
    const uint64_t* __restrict__ fbits = fb.fbits;
    uint32_t* __restrict__ area2 = fb.area2;
    unsigned long long* __restrict__ stats = fb.stats;
    extern __shared__ __attribute__((aligned(16))) unsigned long long lds_b[];
    const int lane = threadIdx.x & 63;
    const int slot = threadIdx.x / CG, sl = threadIdx.x & (CG - 1), g0 = lane & ~(CG - 1);
    const int y = blockIdx.x * cg_rows<CG>() + slot;
    const bool act = y < g.H;
    unsigned long long* s_b = lds_b + (size_t)slot * g.WW;
    const bool last = y == g.H - 1;
    const int n = act ? (int)nfg[y] : 0;
    // F row y+1 (k_resolve): zero when row y+1 has no runs, not needed when row y has none
    const bool fnext = n && !last && nfg[y + 1];
    if (n)
        for (int w = sl; w < g.WW; w += CG) s_b[w] = fnext ? fbits[(size_t)(y + 1) * g.WW + w] : 0ull;
    wave_sync_lds();
    int comps = 0;
    if (act) {
        const uint32_t base = fb.rowb[2 * y];
        const uint8_t* ge = gE + (fb.rowb[2 * y + 1] - 1);
        const uint64_t* b = reinterpret_cast<const uint64_t*>(s_b);
        const unsigned long long gmask = ((1ull << CG) - 1ull) << g0;
        for (int k0 = 0; k0 < n; k0 += CG) {   // uniform trip count within the group: it reduces below
            const int k = k0 + sl;
            const bool valid = k < n;
            const uint32_t id = base + (valid ? k : 0);
            uint32_t r = 0xffffffffu;
            int c = 0;
            if (valid) {
                r = uf_find(fpar, id);
                atomicMin(fpar + id, r);
                comps += r == id;
            }
            if (valid && !last) {
                int s = rs[id], e = re[id];
                c = 2 * popc_range(b, s, e);
                if (k == 0 || ge[k]) {
                    int bs = bit_at(b, s);
                    c -= bs;
                    if (s >= 1 && bs && bit_at(b, s - 1)) c += 1;
                }
                if (k == n - 1 || ge[k + 1]) {
                    int be = bit_at(b, e);
                    c -= be;
                    if (e <= g.W - 2 && be && bit_at(b, e + 1)) c += 1;
                }
                if (k + 1 < n && !ge[k + 1]) c += 2 * popc_range(b, e + 1, (int)rs[id + 1] - 1);
            }
            // one atomic per run of lanes with the same root (a large component's
            // runs of a row would otherwise all hit one address)
            const uint32_t rp = __shfl_up(r, 1, CG);
            const bool head = sl == 0 || rp != r;
            const unsigned long long heads = __ballot(head) & gmask;
            const unsigned long long after = heads & (lane == 63 ? 0ull : (~0ull << (lane + 1)));
            const int seg_end = after ? __builtin_ctzll(after) - 1 : g0 + CG - 1;
            const int incl = group_incl_scan<CG>(c);
            const int seg = __shfl(incl, seg_end, 64) - incl + c;
            if (head && valid && seg) atomicAdd(area2 + r, (uint32_t)seg);
        }
    }
    for (int d = 32; d >= 1; d >>= 1) comps += __shfl_xor(comps, d, 64);
    if (lane == 0 && comps) atomicAdd(stats + STAT_SLOT(blockIdx.x) * 4 + 2, (unsigned long long)comps);
}

// ------------------------------------------------------------------- back ---
// The back of the loop is split at its only recurrence:
//   k_dilate (tiles x frames, no recurrence) k x k dilation of the kept mask
//          (fd:106) -> block-major bits: one BxB bit field per block
//   k_acc  (frames in order, one lane per BxB block, no LDS / barriers) the
//          accumulated-mask update (fd:107) with acc in registers; per frame it
//          emits only bits: acc > 127 per pixel as the block's bit field (the
//          overlay's red mask, fd:110) and "acc all zero" per block (fd:117)
//   k_out  (tiles x frames, no recurrence) red overlay (fd:110-111) and the
//          static-block DCT quantisation with the YCrCb round trip
//          (fd:115-130) from the BGR frame and those bits
// Block-major bit field of a BxB block: bit B*i + j = row i, column j (u16 for
// B = 4, u64 for B = 8); frame t's fields are dense at t * (H/B) * (W/B).
template <int B> struct BlkT;
template <> struct BlkT<4> { typedef uint16_t T; };
template <> struct BlkT<8> { typedef uint64_t T; };

// One lane per (64-px word column, block row) of frame blockIdx.y: the B + k - 1
// kept-mask rows it needs (out-of-image rows are skipped = ignored, as OpenCV's
// dilate border), dilated horizontally by shifts across the neighbour words
// (out bit x = OR of src bits x - anchor .. x + k - 1 - anchor), ORed into the
// B output rows, then transposed into the 64/B block fields of the word.
template <int B>
__global__ void __launch_bounds__(256) k_dilate(BackArgs a)
{
    typedef typename BlkT<B>::T BT;
    const int W = a.g.W, H = a.g.H, WW = a.g.WW, NBX = a.NBX, NBY = a.NBY;
    const int idx = blockIdx.x * 256 + threadIdx.x, t = blockIdx.y;
    if (idx >= WW * NBY) return;
    const int wi = idx % WW, by = idx / WW, y0 = by * B;
    const int k = a.ksize, an = a.anchor;
    const uint64_t* kb = a.kbits + (size_t)t * H * WW;
    // sparse masks (a.kocc): the rows of the window without kept bits are never
    // read; a block row whose whole window is empty writes no fields, only
    // docc = 0, and k_acc then reads none either
    const uint8_t* ko = a.kocc ? a.kocc + (size_t)t * H : nullptr;
    // Loads are unconditional from clamped addresses and unrolled, so several
    // are in flight at once (a load behind a per-row test waits out the one
    // before it). Window rows kept (in the image and, sparse, with kept bits):
    // bit r of kmask for windows of <= 64 rows, ko re-read past that.
    const int R = B + k - 1;
    auto in_img = [&](int r) { const int y = y0 - an + r; return y >= 0 && y < H; };
    auto row_of = [&](int r) { return min(max(y0 - an + r, 0), H - 1); };
    uint64_t kmask = 0;
    if (ko) {
        int any = 0;
#pragma unroll 8
        for (int r = 0; r < R; ++r) {
            const int kp = (int)in_img(r) & (int)(ko[row_of(r)] != 0);
            any |= kp;
            kmask |= (uint64_t)kp << (r & 63);
        }
        if (wi == 0) a.docc[(size_t)by * a.n + t] = (uint8_t)any;
        if (!any && !(a.dbg_dil && t == a.n - 1)) return;
    } else {
        for (int r = 0; r < min(R, 64); ++r) kmask |= (uint64_t)in_img(r) << r;
    }
    // pixels past W (the last word) are not pixels: their dilated bits stay 0
    const uint64_t vmask = (wi == WW - 1 && (W & 63)) ? (1ull << (W & 63)) - 1ull : ~0ull;
    const int wl = max(wi - 1, 0), wr = min(wi + 1, WW - 1);
    uint64_t out[B];
#pragma unroll
    for (int i = 0; i < B; ++i) out[i] = 0;
    // rows four at a time: the 12 loads first (rows not kept read row 0 and
    // are discarded), then the shifts
    auto ld64 = [&](uint32_t w) { return *reinterpret_cast<const uint64_t*>(reinterpret_cast<const uint8_t*>(kb) + w * 8u); };
    auto rows = [&](auto big) {   // big: windows past 64 rows test ko per row
        for (int r0 = 0; r0 < R; r0 += 4) {
            uint64_t c[4], pv[4], nv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int r = r0 + u;
                bool keep;
                if constexpr (decltype(big)::value) keep = r < R && in_img(r) && (!ko || ko[row_of(r)]);
                else keep = r < R && ((kmask >> r) & 1) != 0;
                // kb (frame t = blockIdx.y) is wave-uniform: 32-bit lane offsets
                const uint32_t ro = (uint32_t)(keep ? row_of(r) * WW : 0);
                const uint64_t c0 = ld64(ro + wi), p0 = ld64(ro + wl), n0 = ld64(ro + wr);
                // the masks pass through an empty asm so that the compiler
                // cannot turn "keep ? load : 0" back into a branch around the load
                uint32_t mc = keep ? ~0u : 0u, mp = keep && wi > 0 ? ~0u : 0u, mn = keep && wi + 1 < WW ? ~0u : 0u;
                asm("" : "+v"(mc), "+v"(mp), "+v"(mn));
                c[u] = c0 & (((uint64_t)mc << 32) | mc);
                pv[u] = p0 & (((uint64_t)mp << 32) | mp);
                nv[u] = n0 & (((uint64_t)mn << 32) | mn);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int r = r0 + u;
                uint64_t o = c[u];
                for (int off = 1; off <= k - 1 - an; ++off) o |= (c[u] >> off) | (nv[u] << (64 - off));
                for (int off = 1; off <= an; ++off) o |= (c[u] << off) | (pv[u] >> (64 - off));
                o &= vmask;
#pragma unroll
                for (int i = 0; i < B; ++i)
                    if (r - i >= 0 && r - i < k) out[i] |= o;
            }
        }
    };
    if (R <= 64) rows(std::false_type{});
    else rows(std::true_type{});
#pragma unroll
    for (int i = 0; i < B; ++i)   // rows past H (a partial last block row) are not pixels
        if (y0 + i >= H) out[i] = 0;
    if (a.dbg_dil && t == a.n - 1) {
#pragma unroll
        for (int i = 0; i < B; ++i)
            if (y0 + i < H) a.dbg_dil[(size_t)(y0 + i) * WW + wi] = out[i];
    }
    uint8_t* db = reinterpret_cast<uint8_t*>(a.dblk) + (size_t)t * NBY * NBX * sizeof(BT);   // wave-uniform
    constexpr int PER = 64 / B;
    const int nb = min(PER, NBX - wi * PER);
    const uint32_t dbo = (uint32_t)(by * NBX + wi * PER) * (uint32_t)sizeof(BT);
#pragma unroll
    for (int b = 0; b < PER; ++b) {
        uint64_t f = 0;
#pragma unroll
        for (int i = 0; i < B; ++i) f |= ((out[i] >> (B * b)) & ((1ull << B) - 1)) << (B * i);
        if (b < nb) *reinterpret_cast<BT*>(db + (dbo + (uint32_t)(b * sizeof(BT)))) = (BT)f;
    }
}

// Bit 7 of each byte of w[0..3] (4 pixels a word) as 16 bits, pixel j of word k
// at bit 4k + j. Packed 16-bit multiplies gather bits without carries (every
// product's set bits land on distinct positions) and byte permutes keep the
// bytes holding them: 11 VALU for 16 pixels instead of ~45 shifts and masks.
__device__ __forceinline__ uint32_t hibits16(const uint32_t (&w)[4])
{
    auto pm = [](uint32_t x, unsigned short k) { return as_u32(as_u16x2(x) * (u16x2)k); };
    uint32_t y[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) y[k] = pm(w[k] & 0x80808080u, 0x81);   // half: bits 7, 15 -> 14, 15
    // bytes 1, 3 of two words: the first word's pixels at 6, 7, 14, 15, the second's at 22, 23, 30, 31
    const uint32_t z01 = __builtin_amdgcn_perm(y[1], y[0], 0x07050301u);
    const uint32_t z23 = __builtin_amdgcn_perm(y[3], y[2], 0x07050301u);
    // half: bits 6, 7, 14, 15 -> 12..15; bytes 1, 3 again: word k's nibble at 8k + 4
    const uint32_t v = __builtin_amdgcn_perm(pm(z23, 0x41), pm(z01, 0x41), 0x07050301u);
    // half: nibbles at 4, 12 -> 8..15 (bytes 1, 3)
    return __builtin_amdgcn_perm(0u, pm(v, 0x11), 0x04040301u);
}

// One lane per BxB block (64 blocks across per wave, one block row), frames in
// order with the block's acc bytes in registers; the block fields of 8 frames
// are loaded one chunk ahead. FAST (acc_fast_ok): the dilated addend is a
// sign-mask AND, the multiply-adds run as packed pairs and the clamp is gone.
template <int B, bool FAST>
__global__ void __launch_bounds__(64) k_acc(BackArgs a)
{
    typedef typename BlkT<B>::T BT;
    constexpr BT ROWM = (BT)((1u << B) - 1);
    const int lane = threadIdx.x;
    const int NBX = a.NBX, NBY = a.NBY, AP = a.ap;   // acc padded to NBX*B x NBY*B: partial blocks' pad stays 0
    const int bxi = blockIdx.x * 64 + lane, by = blockIdx.y;
    const bool active = bxi < NBX;
    const int bxc = min(bxi, NBX - 1);
    const size_t blk = (size_t)by * NBX + bxc, NB = (size_t)NBY * NBX;
    const int x0 = bxc * B, y0 = by * B;
    uint32_t acv[B][B / 4];
#pragma unroll
    for (int i = 0; i < B; ++i) {
        const uint32_t* ac = reinterpret_cast<const uint32_t*>(a.acc + (size_t)(y0 + i) * AP + x0);
#pragma unroll
        for (int d = 0; d < B / 4; ++d) acv[i][d] = ac[d];
    }
    const BT* db = reinterpret_cast<const BT*>(a.dblk);
    BT* rb = reinterpret_cast<BT*>(a.rblk);
    constexpr int U = 8;
    BT dA[U], dB[U];
    // docc (uniform over the workgroup's block row): frames whose block row has
    // no dilated bit take a zero field. Read once up front as a frame bit mask
    // in LDS, so that the field loads below are unconditional and never wait:
    // a load behind a per-frame docc test drained vmcnt to 0 before each one
    // (two memory round trips a frame, the kernel's whole time).
    __shared__ unsigned long long dmask[DVC_MAX_BATCH / 64];
    const uint8_t* dc = a.docc ? a.docc + (size_t)by * a.n : nullptr;
    if (dc) {
        uint8_t v[DVC_MAX_BATCH / 64];
#pragma unroll
        for (int c = 0; c < DVC_MAX_BATCH / 64; ++c) v[c] = dc[min(c * 64 + lane, a.n - 1)];
#pragma unroll
        for (int c = 0; c < DVC_MAX_BATCH / 64; ++c) {
            const unsigned long long m = __ballot(c * 64 + lane < a.n && v[c] != 0);
            if (lane == 0) dmask[c] = m;
        }
        __syncthreads();
    }
    auto load_chunk = [&](int t0, BT (&dst)[U]) {   // t0 % 8 == 0: one mask word
        const unsigned long long m = dc ? dmask[min(t0, DVC_MAX_BATCH - 1) >> 6] >> (t0 & 63) : ~0ull;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int tt = min(t0 + u, a.n - 1);   // clamped: the last frames reload
            const bool on = (m >> u) & 1u;
            const BT v = db[on ? (size_t)tt * NB + blk : blk];   // off: frame 0's field, discarded
            dst[u] = on ? v : (BT)0;
        }
    };
    unsigned long long nstatic = 0;
    const float dil0 = __builtin_fmaf(0.f, a.beta, a.gamma), dil1 = __builtin_fmaf(255.f, a.beta, a.gamma);
    auto frame = [&](int t, BT d) {
        uint32_t aor = 0;
#pragma unroll
        for (int i = 0; i < B; ++i)
#pragma unroll
            for (int q = 0; q < B / 4; ++q) aor |= acv[i][q];
        // addWeighted (fd:107); an all-zero block with no dilated pixel stays all
        // zero when addWeighted(0, 0) = 0 (a.acc0_fixed), skipping the float math
        bool zero = true;
        if (FAST && !(d == 0 && aor == 0)) {   // acc_fast_ok implies acc0_fixed
            const f32x2 al = (f32x2)a.alpha;
            uint32_t nor = 0;
#pragma unroll
            for (int i = 0; i < B; ++i) {
                const uint32_t dw = (uint32_t)((d >> (B * i)) & ROWM);
#pragma unroll
                for (int q = 0; q < B / 4; ++q) {
                    const uint32_t av = acv[i][q];
                    float dv[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j)   // D = dil bit ? dil1 : +0
                        dv[j] = __builtin_bit_cast(float, (uint32_t)((int32_t)(dw << (31 - 4 * q - j)) >> 31) & a.dil1_bits);
                    const f32x2 t01 = __builtin_elementwise_fma(
                        (f32x2){(float)(av & 255), (float)((av >> 8) & 255)}, al, (f32x2){dv[0], dv[1]});
                    const f32x2 t23 = __builtin_elementwise_fma(
                        (f32x2){(float)((av >> 16) & 255), (float)(av >> 24)}, al, (f32x2){dv[2], dv[3]});
                    uint32_t nv = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_rintf(t01.x), 0u, 0u);
                    nv = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_rintf(t01.y), 1u, nv);
                    nv = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_rintf(t23.x), 2u, nv);
                    nv = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_rintf(t23.y), 3u, nv);
                    acv[i][q] = nv;
                    nor |= nv;
                }
            }
            zero = nor == 0;
        } else if (!FAST && !(a.acc0_fixed && d == 0 && aor == 0)) {
#pragma unroll
            for (int i = 0; i < B; ++i) {
                const uint32_t dw = (uint32_t)((d >> (B * i)) & ROWM);
#pragma unroll
                for (int q = 0; q < B / 4; ++q) {
                    uint32_t av = acv[i][q], nv = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        // fmaf(dil, beta, gamma) for dil in {0, 255}: one of two
                        // uniform values; sat_u8(rint(t)): clamp (fmax/fmin send NaN
                        // to 0 like the reference's saturate_cast) then an exact
                        // integer -> byte conversion packed in place
                        const float tv = __builtin_fmaf((float)((av >> (8 * j)) & 255), a.alpha,
                                                        ((dw >> (4 * q + j)) & 1u) ? dil1 : dil0);
                        const float c = __builtin_fminf(__builtin_fmaxf(__builtin_rintf(tv), 0.f), 255.f);
                        nv = __builtin_amdgcn_cvt_pk_u8_f32(c, (uint32_t)j, nv);
                    }
                    acv[i][q] = nv;
                    zero = zero && nv == 0;
                }
            }
        }
        // bits out: acc > 127 per pixel (bit 7 of each byte), all-zero per block
        // (word k = B/4 * i + q holds bits 4k .. 4k + 3 of the field)
        BT r = 0;
#pragma unroll
        for (int g = 0; g < B * B / 16; ++g) {
            const uint32_t w[4] = {acv[(4 * g) / (B / 4)][(4 * g) % (B / 4)],
                                   acv[(4 * g + 1) / (B / 4)][(4 * g + 1) % (B / 4)],
                                   acv[(4 * g + 2) / (B / 4)][(4 * g + 2) % (B / 4)],
                                   acv[(4 * g + 3) / (B / 4)][(4 * g + 3) % (B / 4)]};
            r |= (BT)((BT)hibits16(w) << (16 * g));
        }
        // a static block (acc all zero) has no acc > 127 bit: its field is not
        // written, k_out / k_out_gen take it as zero from sbits
        if (active && !zero) rb[(size_t)t * NB + blk] = r;
        const unsigned long long sb = __ballot(active && zero);
        if (lane == 0) a.sbits[(size_t)t * a.sstride + (size_t)by * a.SW + blockIdx.x] = sb;
        nstatic += (unsigned long long)__popcll(sb);
    };

    load_chunk(0, dA);
    for (int t0 = 0; t0 < a.n; t0 += 2 * U) {
        load_chunk(t0 + U, dB);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (t0 + u < a.n) frame(t0 + u, dA[u]);
        load_chunk(t0 + 2 * U, dA);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (t0 + U + u < a.n) frame(t0 + U + u, dB[u]);
    }

    // the accumulated mask after frame n-1 (fd:107)
    if (active) {
#pragma unroll
        for (int i = 0; i < B; ++i) {
            uint32_t* ac = reinterpret_cast<uint32_t*>(a.acc + (size_t)(y0 + i) * AP + x0);
#pragma unroll
            for (int d = 0; d < B / 4; ++d) ac[d] = acv[i][d];
        }
    }
    if (lane == 0 && nstatic) atomicAdd(a.stats + STAT_SLOT(blockIdx.x * 7 + blockIdx.y) * 4 + 3, nstatic);
}

// ND dwords to a row of an output frame: dword stores, or byte stores when the
// output layout is not 4-byte aligned (W % 4 != 0 and dense output rows)
template <int ND>
__device__ __forceinline__ void store_row(uint8_t* dst, const uint32_t* w, int bytes)
{
    if (!bytes) {
        uint32_t* o = reinterpret_cast<uint32_t*>(dst);
        // nontemporal: the output frames are never re-read by the pipeline and
        // would otherwise evict lines the other stages re-read from L2 and the
        // Infinity Cache (+4 % end to end, interleaved A/B at 1080p x 383)
#pragma unroll
        for (int d = 0; d < ND; ++d) __builtin_nontemporal_store(w[d], o + d);
    } else {
#pragma unroll
        for (int d = 0; d < 4 * ND; ++d) dst[d] = (uint8_t)(w[d >> 2] >> (8 * (d & 3)));
    }
}

#ifndef DVC_OUT_NTLOAD
#define DVC_OUT_NTLOAD 0
#endif

// k_out tile: 64 blocks across (64*B px) x 4 block rows, one wave per block
// row, one lane per full BxB block, of frame t of the batch. FMT != BGR: the
// block's pixels from a 4:2:0 surface (B luma bytes per row, the chroma row of
// each row pair loaded once), converted to packed BGR in registers.
// FIX: the fused front already wrote every full block as static (FrontOut);
// only the blocks that are not static load their pixels and are rewritten —
// the compressed frame's YCrCb round trip, and the overlay where acc > 127.
template <int B, int FMT, bool FIX>
__device__ __forceinline__ void out_tile(const BackArgs& a, int t, int tx, int ty, int lane, int wave)
{
    const int W = a.g.W, H = a.g.H;
    const int bx = tx * 64 * B + lane * B, by = (ty * 4 + wave) * B;
    if (bx + B > W || by + B > H) return;   // partial edge blocks: k_out_gen
    const bool is_static =
        (a.sbits[(size_t)t * a.sstride + (size_t)(by / B) * a.SW + (bx / B >> 6)] >> ((bx / B) & 63)) & 1ull;
    if (FIX && is_static) return;
    const uint8_t* f = a.bgr + (size_t)t * a.fstride;
    uint32_t px[B][3 * B / 4];
    if constexpr (FMT == DVC_FMT_BGR) {
#pragma unroll
        for (int i = 0; i < B; ++i) {
            const uint32_t* src = reinterpret_cast<const uint32_t*>(f + (size_t)(by + i) * a.pitch + 3 * bx);
#if DVC_OUT_NTLOAD
            // the frame's last use (k_front read it a batch earlier): nontemporal
            // loads leave L2 / MALL to the lines other stages re-read
#pragma unroll
            for (int d = 0; d < 3 * B / 4; ++d) px[i][d] = __builtin_nontemporal_load(src + d);
#else
#pragma unroll
            for (int d = 0; d < 3 * B / 4; ++d) px[i][d] = src[d];
#endif
        }
    } else {
#pragma unroll
        for (int i = 0; i < B; i += 2) {
            const uint8_t* cr = f + a.sf.uoff + (size_t)((by + i) >> 1) * a.sf.cpitch + (FMT == DVC_FMT_NV12 ? bx : bx / 2);
            uint32_t c1[B / 4], c2[B / 4];
#pragma unroll
            for (int d = 0; d < B / 4; ++d) {
                if constexpr (FMT == DVC_FMT_NV12) {
                    c1[d] = reinterpret_cast<const uint32_t*>(cr)[d];
                    c2[d] = 0;
                } else {
                    c1[d] = reinterpret_cast<const uint16_t*>(cr)[d];
                    c2[d] = reinterpret_cast<const uint16_t*>(cr + (a.sf.voff - a.sf.uoff))[d];
                }
            }
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const uint32_t* yr = reinterpret_cast<const uint32_t*>(f + (size_t)(by + i + k) * a.pitch + bx);
#pragma unroll
                for (int d = 0; d < B / 4; ++d) quad_bgr<FMT>(yr[d], c1[d], c2[d], &px[i + k][3 * d]);
            }
        }
    }
    // overlay (fd:110-111): (0,0,255) where acc > 127
    if (a.overlay) {
        typedef typename BlkT<B>::T BT;
        const int NBX = a.NBX;
        const BT rf = is_static ? (BT)0
                                : reinterpret_cast<const BT*>(a.rblk)[(size_t)t * a.NBY * NBX + (size_t)(by / B) * NBX + bx / B];
        uint32_t red[B];
        const bool rany = rf != 0;
#pragma unroll
        for (int i = 0; i < B; ++i) red[i] = (uint32_t)(rf >> (B * i)) & ((1u << B) - 1);
        uint8_t* ovf = a.overlay + (size_t)t * a.ostride;
#pragma unroll
        for (int i = 0; i < B; ++i) {
            if (FIX && !rany) break;   // no red pixel: the speculative copy is exact
            uint32_t ow[3 * B / 4];
            if (!rany) {
#pragma unroll
                for (int d = 0; d < 3 * B / 4; ++d) ow[d] = px[i][d];
            } else {
                uint8_t ob[3 * B];
#pragma unroll
                for (int j = 0; j < B; ++j) {
                    const bool r = (red[i] >> j) & 1u;
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        const int bi = 3 * j + c;
                        const uint32_t v = (px[i][bi >> 2] >> (8 * (bi & 3))) & 255;
                        ob[bi] = r ? (c == 2 ? 255 : 0) : (uint8_t)v;
                    }
                }
#pragma unroll
                for (int d = 0; d < 3 * B / 4; ++d)
                    ow[d] = ob[4 * d] | (ob[4 * d + 1] << 8) | (ob[4 * d + 2] << 16) | ((uint32_t)ob[4 * d + 3] << 24);
            }
            if (a.out_i420) store_i420_row<B>(ovf, W, H, by + i, bx, ow);
            else store_row<3 * B / 4>(ovf + (size_t)(by + i) * a.opitch + 3 * bx, ow, a.obytes);
        }
    }
    // compressed (fd:115-130): BGR -> YCrCb; static block: Y' = trunc(clip(IDCT(
    // rint(DCT(Y - 128) / q) q) + 128)), Cr = Cb = 128 -> (Y', Y', Y'); otherwise
    // the YCrCb -> BGR round trip of the pixels
    if (a.compressed) {
        uint8_t* cpf = a.compressed + (size_t)t * a.ostride;
        uint32_t cw[B][3 * B / 4];
        if (is_static) {
            float X[B * B];
#pragma unroll
            for (int i = 0; i < B; ++i)
#pragma unroll
                for (int qd = 0; qd < B / 4; ++qd) {
                    // 1868 + 9617 + 4899 = 2^14: Y of u8 input is in 0..255, no saturation
                    uint32_t y[4];
                    luma4(px[i][3 * qd], px[i][3 * qd + 1], px[i][3 * qd + 2], y);
#pragma unroll
                    for (int j = 0; j < 4; ++j) X[i * B + 4 * qd + j] = (float)((int)y[j] - 128);
                }
            if constexpr (B == 4) block_dct_quant_pk<B>(X, kDct4, a.quant, a.qinv);   // (launch_out checks a.M)
            else block_dct_quant<B>(X, kDct8, a.quant, a.qinv);   // B = 8 (the packed form spills); launch_out checks a.M
#pragma unroll
            for (int i = 0; i < B; ++i)
#pragma unroll
                for (int qd = 0; qd < B / 4; ++qd) {
                    uint32_t u[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j)   // clip to [0, 255], truncating uint8 cast
                        u[j] = (uint32_t)__builtin_amdgcn_fmed3f(X[i * B + 4 * qd + j] + 128.0f, 0.0f, 255.0f);
                    gray_bgr4(u[0], u[1], u[2], u[3], &cw[i][3 * qd]);
                }
        } else {
#pragma unroll
            for (int i = 0; i < B; ++i) {
                uint8_t ob[3 * B];
#pragma unroll
                for (int j = 0; j < B; ++j) {
                    const int b = (px[i][(3 * j) >> 2] >> (8 * ((3 * j) & 3))) & 255;
                    const int gg = (px[i][(3 * j + 1) >> 2] >> (8 * ((3 * j + 1) & 3))) & 255;
                    const int r = (px[i][(3 * j + 2) >> 2] >> (8 * ((3 * j + 2) & 3))) & 255;
                    const int yv = descale14(b * 1868 + gg * 9617 + r * 4899);
                    const int cr = (int)satu8(descale14((r - yv) * 11682 + (128 << 14))) - 128;
                    const int cb = (int)satu8(descale14((b - yv) * 9241 + (128 << 14))) - 128;
                    ob[3 * j] = (uint8_t)satu8(yv + descale14(cb * 29049));
                    ob[3 * j + 1] = (uint8_t)satu8(yv + descale14(cb * -5636 + cr * -11698));
                    ob[3 * j + 2] = (uint8_t)satu8(yv + descale14(cr * 22987));
                }
#pragma unroll
                for (int d = 0; d < 3 * B / 4; ++d)
                    cw[i][d] = ob[4 * d] | (ob[4 * d + 1] << 8) | (ob[4 * d + 2] << 16) | ((uint32_t)ob[4 * d + 3] << 24);
            }
        }
#pragma unroll
        for (int i = 0; i < B; ++i) {
            if (a.out_i420) store_i420_row<B>(cpf, W, H, by + i, bx, cw[i]);
            else store_row<3 * B / 4>(cpf + (size_t)(by + i) * a.opitch + 3 * bx, cw[i], a.obytes);
        }
    }
}

// Grid-stride over the batch's (frame, tile) pairs with a bounded grid: a few
// long-lived workgroups per CU keep HBM saturated while leaving wave slots to
// the latency-bound contour-filter kernels running beside it on other streams.
template <int B, int FMT, bool FIX>
__global__ void __launch_bounds__(256) k_out(BackArgs a, int ntx, int nty)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int per = ntx * nty, total = per * a.n;
    for (int u = blockIdx.x; u < total; u += gridDim.x) {   // no barrier in the loop
        const int t = u / per, r = u - t * per, ty = r / ntx;
        out_tile<B, FMT, FIX>(a, t, r - ty * ntx, ty, lane, wave);
    }
}

// The fused front's fix-up (FrontOut, fd_kernels.h), block_size 4, BGR frames
// in and out: a wave per unit of (frame, RG block rows), grid-stride. One load
// of the rows' static-block words (lane = (row, word), RG x SW <= 64) finds the
// 64-block words that hold a full block which is not static; those words are
// then rewritten two at a time — both words' pixels and acc > 127 fields are
// loaded before either is computed, so a pair costs one round trip — a lane
// per block: the compressed frame's YCrCb round trip (fd:115-130) and, where
// the block has a red pixel, its overlay rows (fd:110-111). A row of a
// surveillance frame rarely holds more than a few such words.
struct Fix4 {
    uint32_t px[4][3];
    uint16_t rf;
};

template <int FMT>
__device__ __forceinline__ void fix4_load(const BackArgs& a, int t, int row, int bx, bool act, Fix4& b)
{
    const int bxc = act ? bx : 0, rowc = act ? row : 0;   // inactive lanes load a valid block, unused
    // wave-uniform frame bases + 32-bit per-lane offsets (SGPR-base addressing)
    if constexpr (FMT == DVC_FMT_BGR) {
        const uint8_t* f = a.bgr + (size_t)t * a.fstride;
        const uint32_t o = (uint32_t)(rowc * 4 * a.pitch + 12 * bxc);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint3 v = *reinterpret_cast<const uint3*>(f + (o + (uint32_t)(i * a.pitch)));
            b.px[i][0] = v.x;
            b.px[i][1] = v.y;
            b.px[i][2] = v.z;
        }
    } else {   // a 4:2:0 surface read in place: the quad's luma dword and its chroma, as k_front
        const uint8_t* f = a.bgr + (size_t)t * a.fstride;
        const int xq = 4 * bxc;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int y = 4 * rowc + i;
            const uint32_t y4 = *reinterpret_cast<const uint32_t*>(f + (uint32_t)(y * a.pitch + xq));
            const uint32_t cr = (uint32_t)(a.sf.uoff + (size_t)(y >> 1) * a.sf.cpitch + (FMT == DVC_FMT_NV12 ? xq : xq / 2));
            uint32_t c1, c2 = 0;
            if constexpr (FMT == DVC_FMT_NV12) {
                c1 = *reinterpret_cast<const uint32_t*>(f + cr);
            } else {
                c1 = *reinterpret_cast<const uint16_t*>(f + cr);
                c2 = *reinterpret_cast<const uint16_t*>(f + (cr + (uint32_t)(a.sf.voff - a.sf.uoff)));
            }
            quad_bgr<FMT>(y4, c1, c2, b.px[i]);
        }
    }
    b.rf = a.overlay ? *reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(a.rblk) +
                                                           (size_t)t * a.NBY * a.NBX * 2 + (uint32_t)(rowc * a.NBX + bxc) * 2u)
                     : (uint16_t)0;
}

// OI: I420 outputs (DVC_FLAG_OUT_I420) as a template parameter, so the BGR
// fix-up carries no inlined I420 row store (63 -> 52 VGPRs, 32 -> 2 SGPR
// spills for k_fix4<BGR>)
template <bool OI>
__device__ __forceinline__ void fix4_store(const BackArgs& a, int t, int row, int bx, const Fix4& b)
{
    const size_t fo = (size_t)t * a.ostride;                            // wave-uniform
    const uint32_t o = (uint32_t)(row * 4 * a.opitch + 12 * bx);         // per lane
    if (a.overlay && b.rf) {   // (0, 0, 255) where acc > 127; other blocks keep the speculative copy
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            // byte j of M = 0xFF where pixel j's acc > 127 (the four bits spread
            // to bytes by one carry-free multiply), then the row's 12 bytes as
            // per-channel masks: B G R B | G R B G | R B G R
            const uint32_t r4 = (b.rf >> (4 * i)) & 15u;
            const uint32_t M = ((r4 * 0x00204081u) & 0x01010101u) * 0xFFu;
            const uint32_t m[3] = {__builtin_amdgcn_perm(M, M, 0x01000000u), __builtin_amdgcn_perm(M, M, 0x02020101u),
                                   __builtin_amdgcn_perm(M, M, 0x03030302u)};
            constexpr uint32_t red[3] = {0x00FF0000u, 0x0000FF00u, 0xFF0000FFu};   // (0, 0, 255) per pixel
            uint32_t ow[3];
#pragma unroll
            for (int d = 0; d < 3; ++d) ow[d] = ((red[d] ^ b.px[i][d]) & m[d]) ^ b.px[i][d];
            if constexpr (OI) store_i420_row<4>(a.overlay + fo, a.g.W, a.g.H, 4 * row + i, 4 * bx, ow);
            else store_row<3>(a.overlay + fo + (o + (uint32_t)(i * a.opitch)), ow, 0);
        }
    }
    if (a.compressed) {   // not static: the YCrCb -> BGR round trip of every pixel
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint8_t ob[12];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int bb = (b.px[i][(3 * j) >> 2] >> (8 * ((3 * j) & 3))) & 255;
                const int gg = (b.px[i][(3 * j + 1) >> 2] >> (8 * ((3 * j + 1) & 3))) & 255;
                const int rr = (b.px[i][(3 * j + 2) >> 2] >> (8 * ((3 * j + 2) & 3))) & 255;
                const int yv = descale14(bb * 1868 + gg * 9617 + rr * 4899);
                const int cr = (int)satu8(descale14((rr - yv) * 11682 + (128 << 14))) - 128;
                const int cb = (int)satu8(descale14((bb - yv) * 9241 + (128 << 14))) - 128;
                ob[3 * j] = (uint8_t)satu8(yv + descale14(cb * 29049));
                ob[3 * j + 1] = (uint8_t)satu8(yv + descale14(cb * -5636 + cr * -11698));
                ob[3 * j + 2] = (uint8_t)satu8(yv + descale14(cr * 22987));
            }
            uint32_t cw[3];
#pragma unroll
            for (int d = 0; d < 3; ++d)
                cw[d] = ob[4 * d] | (ob[4 * d + 1] << 8) | (ob[4 * d + 2] << 16) | ((uint32_t)ob[4 * d + 3] << 24);
            if constexpr (OI) store_i420_row<4>(a.compressed + fo, a.g.W, a.g.H, 4 * row + i, 4 * bx, cw);
            else store_row<3>(a.compressed + fo + (o + (uint32_t)(i * a.opitch)), cw, 0);
        }
    }
}

// position of the r-th (0-based) set bit of m (r < popc(m))
__device__ __forceinline__ int select_bit(uint64_t m, int r)
{
    int base = 0;
    const int lo = __popc((uint32_t)m);
    if (r >= lo) { r -= lo; m >>= 32; base = 32; }
    uint32_t v = (uint32_t)m;
    const int c16 = __popc(v & 0xffffu);
    if (r >= c16) { r -= c16; v >>= 16; base += 16; }
    const int c8 = __popc(v & 0xffu);
    if (r >= c8) { r -= c8; v >>= 8; base += 8; }
    for (; r > 0; --r) v &= v - 1;
    return base + __builtin_ctz(v);
}

template <int FMT, bool OI>
__global__ void __launch_bounds__(256) k_fix4(BackArgs a, int RG)
{
    const int lane = threadIdx.x & 63;
    // the wave id through readfirstlane: units (frame t, row0) provably
    // wave-uniform, so frame bases stay in SGPRs (SGPR-base addressing)
    const int gw = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)), nw = gridDim.x * 4;
    const int SW = a.SW;
    const int ug = (a.NBY + RG - 1) / RG, total = ug * a.n;
    const int fullx = a.g.W / 4, fully = a.g.H / 4;   // full blocks (partial edge blocks: k_out_gen)
    const int lr = lane / SW, lw = lane - lr * SW;     // the lane's (row in the unit, word) in the scan
    const int nb = min(64, fullx - lw * 64);
    const uint64_t valid = nb >= 64 ? ~0ull : (nb > 0 ? (1ull << nb) - 1ull : 0ull);
    for (int u = gw; u < total; u += nw) {   // uniform per wave, no barrier in the loop
        const int t = u / ug, row0 = (u - t * ug) * RG;
        const bool ok = lr < RG && row0 + lr < fully;
        const uint64_t sw = ok ? a.sbits[(size_t)t * a.sstride + (size_t)(row0 + lr) * SW + lw] : ~0ull;
        const uint64_t ns = ok ? (~sw & valid) : 0ull;   // non-static full blocks of the lane's word
        // the unit's non-static blocks, compacted onto the lanes: block j of the
        // unit (in (row, word, bit) order) goes to lane j % 64 of pass j / 64
        const int cnt = __popcll(ns);
        const int incl = wave_incl_scan(cnt);
        const int nblk = __shfl(incl, 63, 64);
        for (int j0 = 0; j0 < nblk; j0 += 64) {
            const int j = j0 + lane;
            const bool act = j < nblk;
            // source lane: the first s with incl[s] > j (binary search over the lanes)
            int s = 0;
#pragma unroll
            for (int step = 32; step >= 1; step >>= 1) {
                const int probe = s + step - 1;
                if (__shfl(incl, probe, 64) <= j) s += step;
            }
            s = min(s, 63);
            const int excl = __shfl(incl, s, 64) - __shfl(cnt, s, 64);
            const uint64_t m = __shfl(ns, s, 64);
            const int bit = act ? select_bit(m, j - excl) : 0;
            const int row = row0 + s / SW, bx = (s % SW) * 64 + bit;
            Fix4 b;
            fix4_load<FMT>(a, t, row, bx, act, b);
            if (act) fix4_store<OI>(a, t, row, bx, b);
        }
    }
}

// ------------------------------------------------------------- resize ------
// cv2.resize(frame, (W, H)) of 8UC3 with INTER_LINEAR (fd:74, fd:91), one lane
// per output pixel (3 bytes): exact 2x down = OpenCV's INTER_AREA fast path,
// (a + b + c + d + 2) >> 2; otherwise the fixed-point linear path with the
// host-built tables (resize_tables): horizontal products exact in int32, the
// vertical combination with OpenCV's 128-bit SIMD rounding for the first
// simd_end bytes of a row and the scalar FixedPtCast after them.
__global__ void __launch_bounds__(256) k_resize(const uint8_t* __restrict__ src, int spitch, size_t sstride,
                                                uint8_t* __restrict__ dst, int dpitch, size_t dstride, ResizeTab rt)
{
    const int dx = blockIdx.x * 256 + threadIdx.x, dy = blockIdx.y, t = blockIdx.z;
    if (dx >= rt.dw) return;
    const uint8_t* f = src + (size_t)t * sstride;
    uint8_t* o = dst + (size_t)t * dstride + (size_t)dy * dpitch + 3 * dx;
    if (rt.area2x) {
        const uint8_t* r0 = f + (size_t)(2 * dy) * spitch + 6 * dx;
        const uint8_t* r1 = r0 + spitch;
#pragma unroll
        for (int c = 0; c < 3; ++c) o[c] = (uint8_t)((r0[c] + r0[c + 3] + r1[c] + r1[c + 3] + 2) >> 2);
        return;
    }
    const int sx = rt.xo[3 * dx], a0 = rt.xo[3 * dx + 1], a1 = rt.xo[3 * dx + 2];
    const int sy = rt.yo[3 * dy], b0 = rt.yo[3 * dy + 1], b1 = rt.yo[3 * dy + 2];
    const int sx1 = sx + 1 < rt.sw ? sx + 1 : sx, sy1 = sy + 1 < rt.sh ? sy + 1 : sy;
    const uint8_t* r0 = f + (size_t)sy * spitch;
    const uint8_t* r1 = f + (size_t)sy1 * spitch;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const int S0 = r0[3 * sx + c] * a0 + r0[3 * sx1 + c] * a1;
        const int S1 = r1[3 * sx + c] * a0 + r1[3 * sx1 + c] * a1;
        int v;
        if (3 * dx + c < rt.simd_end)
            v = ((((S0 >> 4) * b0) >> 16) + (((S1 >> 4) * b1) >> 16) + 2) >> 2;
        else
            v = (int)(((long long)S0 * b0 + (long long)S1 * b1 + (1 << 21)) >> 22);
        o[c] = (uint8_t)satu8(v);
    }
}

// ------------------------------------------------------ generic back end ----
// Any block size (and the partial edge blocks of B = 4, 8): row-major bit
// planes instead of block fields.
//   k_dilate_rows  one lane per (64-px word, row): k x k dilation (fd:106)
//   k_acc_rows     one lane per pixel, frames in order: addWeighted (fd:107)
//                  -> acc > 127 (rbits) and acc != 0 (zbits) per frame
//   k_out_gen      a workgroup per rectangle of blocks: overlay (fd:110-111),
//                  static test (fd:120), block DCT / quantise / IDCT of any
//                  block shape through LDS (fd:121-127), YCrCb round trip
__global__ void __launch_bounds__(256) k_dilate_rows(BackArgs a)
{
    const int W = a.g.W, H = a.g.H, WW = a.g.WW;
    const int idx = blockIdx.x * 256 + threadIdx.x, t = blockIdx.y;
    if (idx >= WW * H) return;
    const int wi = idx % WW, y = idx / WW;
    const int k = a.ksize, an = a.anchor;
    const uint64_t* kb = a.kbits + (size_t)t * H * WW;
    const uint64_t vmask = (wi == WW - 1 && (W & 63)) ? (1ull << (W & 63)) - 1ull : ~0ull;
    uint64_t out = 0;
    for (int r = 0; r < k; ++r) {
        const int yy = y - an + r;
        if (yy < 0 || yy >= H || (a.kocc && !a.kocc[(size_t)t * H + yy])) continue;
        const uint64_t* row = kb + (size_t)yy * WW;
        const uint64_t c = row[wi], pv = wi > 0 ? row[wi - 1] : 0ull, nv = wi + 1 < WW ? row[wi + 1] : 0ull;
        uint64_t o = c;
        for (int off = 1; off <= k - 1 - an; ++off) o |= (c >> off) | (nv << (64 - off));
        for (int off = 1; off <= an; ++off) o |= (c << off) | (pv >> (64 - off));
        out |= o;
    }
    out &= vmask;
    a.dbits[(size_t)t * H * WW + (size_t)y * WW + wi] = out;
    if (a.dbg_dil && t == a.n - 1) a.dbg_dil[(size_t)y * WW + wi] = out;
}

__global__ void __launch_bounds__(64) k_acc_rows(BackArgs a)
{
    const int lane = threadIdx.x, wi = blockIdx.x, y = blockIdx.y;
    const int W = a.g.W, H = a.g.H, WW = a.g.WW;
    const int x = wi * 64 + lane;
    const bool active = x < W;
    uint8_t* ap = a.acc + (size_t)y * a.ap + (active ? x : 0);
    uint32_t acc = active ? *ap : 0u;
    const size_t plane = (size_t)H * WW, off = (size_t)y * WW + wi;
    const float dil0 = __builtin_fmaf(0.f, a.beta, a.gamma), dil1 = __builtin_fmaf(255.f, a.beta, a.gamma);
    constexpr int U = 8;
    uint64_t dA[U], dB[U];
    auto load_chunk = [&](int t0, uint64_t (&dst)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) dst[u] = a.dbits[(size_t)min(t0 + u, a.n - 1) * plane + off];
    };
    auto frame = [&](int t, uint64_t d) {
        const float tv = __builtin_fmaf((float)acc, a.alpha, ((d >> lane) & 1ull) ? dil1 : dil0);
        acc = (uint32_t)__builtin_fminf(__builtin_fmaxf(__builtin_rintf(tv), 0.f), 255.f);
        const uint64_t r = __ballot(active && acc > 127u), z = __ballot(active && acc != 0u);
        if (lane == 0) {
            a.rbits[(size_t)t * plane + off] = r;
            a.zbits[(size_t)t * plane + off] = z;
        }
    };
    load_chunk(0, dA);
    for (int t0 = 0; t0 < a.n; t0 += 2 * U) {
        load_chunk(t0 + U, dB);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (t0 + u < a.n) frame(t0 + u, dA[u]);
        load_chunk(t0 + 2 * U, dA);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (t0 + U + u < a.n) frame(t0 + U + u, dB[u]);
    }
    if (active) *ap = (uint8_t)acc;
}

// A rectangle of blocks of one frame: the region [rx0, rx1) x [ry0, ry1) cut
// into jobs of jbx x jby blocks (njx jobs across), one workgroup each.
struct GenRegion {
    int rx0, rx1, ry0, ry1;
    int jbx, jby, njx;
};

__device__ __forceinline__ int luma_px(int b, int g, int r) { return descale14(b * 1868 + g * 9617 + r * 4899); }

__global__ void __launch_bounds__(256) k_out_gen(BackArgs a, GenRegion R, int fast)
{
    extern __shared__ __attribute__((aligned(16))) float lds_g[];
    const int t = blockIdx.y, tid = threadIdx.x;
    const int B = a.B, W = a.g.W, H = a.g.H, WW = a.g.WW;
    const int jx = blockIdx.x % R.njx, jy = blockIdx.x / R.njx;
    const int bx0 = R.rx0 + jx * R.jbx, bx1 = min(R.rx1, bx0 + R.jbx);
    const int by0 = R.ry0 + jy * R.jby, by1 = min(R.ry1, by0 + R.jby);
    if (bx0 >= bx1 || by0 >= by1) return;
    const int px0 = bx0 * B, py0 = by0 * B;
    const int JW = min(W, bx1 * B) - px0, JH = min(H, by1 * B) - py0;
    const int nbx = bx1 - bx0, nblk = nbx * (by1 - by0), npx = JW * JH;
    const int cap = R.jbx * R.jby * B * B;
    float* X = lds_g;
    float* T = X + cap;
    int* flag = reinterpret_cast<int*>(T + cap);   // per block: 0 moving, 1 static, 2 static with an odd side
    const int bwp = W % B, bhp = H % B;
    const float* MB = a.Mtab;
    const float* MWp = a.Mtab + B * B;
    const float* MHp = MWp + bwp * bwp;
    const size_t plane = (size_t)H * WW;
    const uint8_t* f = a.bgr + (size_t)t * a.fstride;

    // static test per block (fd:120)
    int nst = 0;
    for (int b = tid; b < nblk; b += 256) {
        const int gbx = bx0 + b % nbx, gby = by0 + b / nbx;
        const int bw = min(B, W - gbx * B), bh = min(B, H - gby * B);
        bool st;
        if (fast) {
            st = (a.sbits[(size_t)t * a.sstride + (size_t)gby * a.SW + (gbx >> 6)] >> (gbx & 63)) & 1ull;
        } else {
            st = true;
            const uint64_t* zb = a.zbits + (size_t)t * plane;
            for (int i = 0; i < bh && st; ++i) {
                const int ya = gby * B + i, s0 = gbx * B, e0 = s0 + bw - 1;
                for (int w = s0 >> 6; w <= (e0 >> 6); ++w) {
                    uint64_t m = ~0ull;
                    if (w == (s0 >> 6)) m &= ~0ull << (s0 & 63);
                    if (w == (e0 >> 6)) m &= ~0ull >> (63 - (e0 & 63));
                    if (zb[(size_t)ya * WW + w] & m) { st = false; break; }
                }
            }
        }
        int fl = st ? 1 : 0;
        if (st && ((bw > 1 && (bw & 1)) || (bh > 1 && (bh & 1)))) {   // cv2.dct raises (fd:122)
            fl = 2;
            atomicMin(a.err, a.frame0 + (unsigned long long)t);
        }
        nst += st;
        flag[b] = fl;
    }
    if (!fast) {
        for (int d = 32; d >= 1; d >>= 1) nst += __shfl_xor(nst, d, 64);
        if ((tid & 63) == 0 && nst) atomicAdd(a.stats + STAT_SLOT(blockIdx.x + 5 * t) * 4 + 3, (unsigned long long)nst);
    }
    __syncthreads();

    // overlay, Y - 128 of static blocks into LDS, round trip of the rest
    for (int e = tid; e < npx; e += 256) {
        const int i = e / JW, j = e - i * JW, y = py0 + i, x = px0 + j;
        const int b = (i / B) * nbx + j / B;
        int cb, cg, cr;
        if (a.sf.fmt == DVC_FMT_BGR) {
            const uint8_t* px = f + (size_t)y * a.pitch + 3 * x;
            cb = px[0];
            cg = px[1];
            cr = px[2];
        } else {   // a 4:2:0 surface read in place
            const size_t c = (size_t)(y >> 1) * a.sf.cpitch + (a.sf.fmt == DVC_FMT_NV12 ? (x & ~1) : (x >> 1));
            yuvpx::yuv_px_bgr(f[(size_t)y * a.pitch + x], f[a.sf.uoff + c], f[a.sf.voff + c], cb, cg, cr);
        }
        if (a.overlay) {
            bool red;
            if (fast) {   // static blocks' fields are not written (k_acc): zero
                const size_t fi = (size_t)t * a.NBY * a.NBX + (size_t)(y / B) * a.NBX + x / B;
                const int bit = (y % B) * B + x % B;
                red = flag[b] == 0 &&
                      (B == 4 ? (reinterpret_cast<const uint16_t*>(a.rblk)[fi] >> bit) & 1
                              : (reinterpret_cast<const uint64_t*>(a.rblk)[fi] >> bit) & 1ull);
            } else {
                red = (a.rbits[(size_t)t * plane + (size_t)y * WW + (x >> 6)] >> (x & 63)) & 1ull;
            }
            uint8_t* o = a.overlay + (size_t)t * a.ostride + (size_t)y * a.opitch + 3 * x;
            o[0] = red ? 0 : (uint8_t)cb;
            o[1] = red ? 0 : (uint8_t)cg;
            o[2] = red ? 255 : (uint8_t)cr;
        }
        const int yv = luma_px(cb, cg, cr);
        if (flag[b] == 1) {
            X[e] = (float)(yv - 128);
        } else if (a.compressed) {
            const int crv = (int)satu8(descale14((cr - yv) * 11682 + (128 << 14))) - 128;
            const int cbv = (int)satu8(descale14((cb - yv) * 9241 + (128 << 14))) - 128;
            uint8_t* o = a.compressed + (size_t)t * a.ostride + (size_t)y * a.opitch + 3 * x;
            o[0] = (uint8_t)satu8(yv + descale14(cbv * 29049));
            o[1] = (uint8_t)satu8(yv + descale14(cbv * -5636 + crv * -11698));
            o[2] = (uint8_t)satu8(yv + descale14(crv * 22987));
        }
    }
    __syncthreads();
    // the separable DCT passes of every static block (the oracle's fmaf chains,
    // oc_dct2d_rect / oc_idct2d_rect), one output element per lane
    auto geom = [&](int e, int& i, int& j, int& b, int& bw, int& bh, const float*& Mw, const float*& Mh) {
        i = e / JW;
        j = e - i * JW;
        b = (i / B) * nbx + j / B;
        bw = min(B, W - (px0 + j - j % B));
        bh = min(B, H - (py0 + i - i % B));
        Mw = bw == B ? MB : MWp;
        Mh = bh == B ? MB : MHp;
    };
    for (int e = tid; e < npx; e += 256) {          // rows: T[i][k] = sum_n X[i][n] Mw[k][n]
        int i, j, b, bw, bh;
        const float *Mw, *Mh;
        geom(e, i, j, b, bw, bh, Mw, Mh);
        if (flag[b] != 1) continue;
        const int k = j % B, xs = i * JW + j - k;
        float v = X[xs] * Mw[k * bw];
        for (int n = 1; n < bw; ++n) v = __builtin_fmaf(X[xs + n], Mw[k * bw + n], v);
        T[e] = v;
    }
    __syncthreads();
    for (int e = tid; e < npx; e += 256) {          // cols + quantise: rint(sum_i Mh[k][i] T[i][l] / q) q
        int i, j, b, bw, bh;
        const float *Mw, *Mh;
        geom(e, i, j, b, bw, bh, Mw, Mh);
        if (flag[b] != 1) continue;
        const int k = i % B, ys = (i - k) * JW + j;
        float v = Mh[k * bh] * T[ys];
        for (int r = 1; r < bh; ++r) v = __builtin_fmaf(Mh[k * bh + r], T[ys + r * JW], v);
        X[e] = __builtin_rintf(div_rn(v, a.qinv)) * a.quant;
    }
    __syncthreads();
    for (int e = tid; e < npx; e += 256) {          // inverse rows: T[k][n] = sum_l Y[k][l] Mw[l][n]
        int i, j, b, bw, bh;
        const float *Mw, *Mh;
        geom(e, i, j, b, bw, bh, Mw, Mh);
        if (flag[b] != 1) continue;
        const int nn = j % B, xs = i * JW + j - nn;
        float v = X[xs] * Mw[nn];
        for (int l = 1; l < bw; ++l) v = __builtin_fmaf(X[xs + l], Mw[l * bw + nn], v);
        T[e] = v;
    }
    __syncthreads();
    for (int e = tid; e < npx; e += 256) {          // inverse cols, +128, clip, truncate; (Y', Y', Y')
        int i, j, b, bw, bh;
        const float *Mw, *Mh;
        geom(e, i, j, b, bw, bh, Mw, Mh);
        if (flag[b] != 1 || !a.compressed) continue;
        const int ii = i % B, ys = (i - ii) * JW + j;
        float v = Mh[ii] * T[ys];
        for (int r = 1; r < bh; ++r) v = __builtin_fmaf(Mh[r * bh + ii], T[ys + r * JW], v);
        const uint8_t g = (uint8_t)(uint32_t)__builtin_amdgcn_fmed3f(v + 128.0f, 0.0f, 255.0f);
        uint8_t* o = a.compressed + (size_t)t * a.ostride + (size_t)(py0 + i) * a.opitch + 3 * (px0 + j);
        o[0] = g;
        o[1] = g;
        o[2] = g;
    }
}

// --------------------------------------------------------------- launchers --
hipError_t launch_prime(const uint8_t* bgr, int pitch, uint8_t* gray_tmp, uint32_t* tmp32, uint8_t* out,
                        int W, int H, int gs, const GaussTaps& k, hipStream_t s)
{
    dim3 gq((gs / 4 + 255) / 256, H), gp((W + 255) / 256, H);
    klaunch(k_gray, gq, dim3(256), 0, s, bgr, pitch, gray_tmp, W, H, gs);
    klaunch(k_hblur_q8, gp, dim3(256), 0, s, gray_tmp, tmp32, W, H, gs, k);
    klaunch(k_vblur_q8, gp, dim3(256), 0, s, tmp32, out, W, H, gs, k);
    return hipGetLastError();
}

template <int NW>
static void launch_front_nw(const uint8_t* bgr, int pitch, size_t fstride, const SrcFmt& sf, int n,
                            const uint8_t* gray_in, uint8_t* gray_out, int gs, uint64_t* mbits, const RowGeom& g,
                            int ithresh, hipStream_t s, const FrontOut* fo)
{
    constexpr int FT_H = 4 * NW;
    const int tx = (g.W + FT_W - 1) / FT_W, ty = (g.H + FT_H - 1) / FT_H;
    // chunks of the batch: ~5120 waves in flight (1280 workgroups of 4 waves),
    // at least 8 frames per chunk — each extra chunk re-reads a warm-up frame
    // and adds waves competing with the contour filter (1080p x 191 at NW = 4:
    // 2 chunks, measured best of 1..9); DVC_FRONT_WAVES / DVC_FRONT_MIN override
    static const int target = [] { const char* e = dvc::tune_env("DVC_FRONT_WAVES"); return e ? std::max(1, atoi(e)) : 5120; }();
    int chunks = (target / NW + tx * ty / 2) / (tx * ty);
    static const int minf = [] { const char* e = dvc::tune_env("DVC_FRONT_MIN"); return e ? std::max(1, atoi(e)) : 8; }();
    if (fo) {
        // fused outputs (4 workgroups per CU, 5 for 4:2:0 surfaces): chunks of ~48 frames
        // (1080p x 383: 8 chunks, 4352 workgroups; measured alone 373 k / 514 k /
        // 534 k Mpx/s at 1 / 4 / 8 chunks — a warm-up frame per chunk is 2 % more
        // reads, more workgroups in flight hide the per-frame barriers);
        // DVC_FUSED_CHUNKS overrides
        // at least ~2048 workgroups (8 a CU) when the batch is short: 1080p x 32
        // frames as one chunk is 544 workgroups, half the device (4 chunks of 8
        // frames: 299.7 -> 314.4 k Mpx/s at --batch 32, experiments/README.md)
        static const int fc = [] { const char* e = dvc::tune_env("DVC_FUSED_CHUNKS"); return e ? atoi(e) : 0; }();
        chunks = fc > 0 ? fc : std::max({1, n / 48, (2048 + tx * ty - 1) / (tx * ty)});
    }
    chunks = std::max(1, std::min(chunks, n / minf));
    const int chunk = (n + chunks - 1) / chunks;
    chunks = (n + chunk - 1) / chunk;
    // XCD bands (k_front: each XCD walks a contiguous run of (chunk, tile row,
    // tile) ids): the fused front's default (+1.2 to +1.4 %, BGR and NV12),
    // not the plain one's; DVC_FRONT_XCD overrides
    static const int xcd_env = [] { const char* e = dvc::tune_env("DVC_FRONT_XCD"); return e ? atoi(e) : -1; }();
    const int xcd = xcd_env >= 0 ? xcd_env : (fo ? 1 : 0);
    // frames in flight per workgroup: the fused BGR front 2 (+1 % against 1 at
    // 4 workgroups a CU, 119 VGPRs), the others 1; DVC_FRONT_PF overrides
    static const int pf_env = [] { const char* e = dvc::tune_env("DVC_FRONT_PF"); return e ? atoi(e) : 0; }();
    const int pf = pf_env > 0 ? pf_env : (fo ? 2 : 1);
    const dim3 grid(tx, ty, chunks), block(64 * NW);
    const FrontOut none{};
    if constexpr (NW == 4 || NW == 8) {
        if (fo) {
            // DVC_FRONT_LDS=<bytes> (experiment): unused dynamic LDS per workgroup, to
            // cap the fused front's workgroups per CU and leave room to the others
            static const size_t pad = [] { const char* e = dvc::tune_env("DVC_FRONT_LDS"); return e ? (size_t)atol(e) : 0; }();
            if constexpr (NW == 4) {
                if (fo->B == 8) {   // 8x8 blocks (BGR frames; launch_front checked the rest)
                    klaunch((k_front<4, 1, DVC_FMT_BGR, true, 8>), grid, block, pad, s, bgr, pitch, fstride, sf,
                                       n, chunk, gray_in, gray_out, gs, mbits, g.W, g.H, g.WW, ithresh, xcd, *fo);
                    return;
                }
            }
            if constexpr (NW == 4) {
                if (fo->i420) {   // I420 outputs (launch_front: B = 4, NW = 4)
                    if (sf.fmt == DVC_FMT_NV12)
                        klaunch((k_front<4, 1, DVC_FMT_NV12, true, 4, true>), grid, block, pad, s, bgr, pitch,
                                           fstride, sf, n, chunk, gray_in, gray_out, gs, mbits, g.W, g.H, g.WW, ithresh,
                                           xcd, *fo);
                    else if (sf.fmt == DVC_FMT_I420)
                        klaunch((k_front<4, 1, DVC_FMT_I420, true, 4, true>), grid, block, pad, s, bgr, pitch,
                                           fstride, sf, n, chunk, gray_in, gray_out, gs, mbits, g.W, g.H, g.WW, ithresh,
                                           xcd, *fo);
                    else if (pf == 2)
                        klaunch((k_front<4, 2, DVC_FMT_BGR, true, 4, true>), grid, block, pad, s, bgr, pitch,
                                           fstride, sf, n, chunk, gray_in, gray_out, gs, mbits, g.W, g.H, g.WW, ithresh,
                                           xcd, *fo);
                    else
                        klaunch((k_front<4, 1, DVC_FMT_BGR, true, 4, true>), grid, block, pad, s, bgr, pitch,
                                           fstride, sf, n, chunk, gray_in, gray_out, gs, mbits, g.W, g.H, g.WW, ithresh,
                                           xcd, *fo);
                    return;
                }
            }
            if (sf.fmt == DVC_FMT_NV12)
                klaunch((k_front<NW, 1, DVC_FMT_NV12, true>), grid, block, pad, s, bgr, pitch, fstride, sf, n,
                                   chunk, gray_in, gray_out, gs, mbits, g.W, g.H, g.WW, ithresh, xcd, *fo);
            else if (sf.fmt == DVC_FMT_I420)
                klaunch((k_front<NW, 1, DVC_FMT_I420, true>), grid, block, pad, s, bgr, pitch, fstride, sf, n,
                                   chunk, gray_in, gray_out, gs, mbits, g.W, g.H, g.WW, ithresh, xcd, *fo);
            else if (pf == 2 && NW == 4)
                klaunch((k_front<4, 2, DVC_FMT_BGR, true>), grid, block, pad, s, bgr, pitch, fstride, sf, n,
                                   chunk, gray_in, gray_out, gs, mbits, g.W, g.H, g.WW, ithresh, xcd, *fo);
            else
                klaunch((k_front<NW, 1, DVC_FMT_BGR, true>), grid, block, pad, s, bgr, pitch, fstride, sf, n,
                                   chunk, gray_in, gray_out, gs, mbits, g.W, g.H, g.WW, ithresh, xcd, *fo);
            return;
        }
    }
    if (sf.fmt == DVC_FMT_I420)
        klaunch((k_front<NW, 1, DVC_FMT_I420, false>), grid, block, 0, s, bgr, pitch, fstride, sf, n, chunk,
                           gray_in, gray_out, gs, mbits, g.W, g.H, g.WW, ithresh, xcd, none);
    else if (sf.fmt == DVC_FMT_NV12)
        klaunch((k_front<NW, 1, DVC_FMT_NV12, false>), grid, block, 0, s, bgr, pitch, fstride, sf, n, chunk,
                           gray_in, gray_out, gs, mbits, g.W, g.H, g.WW, ithresh, xcd, none);
    else if (pf == 2)
        klaunch((k_front<NW, 2, DVC_FMT_BGR, false>), grid, block, 0, s, bgr, pitch, fstride, sf, n, chunk,
                           gray_in, gray_out, gs, mbits, g.W, g.H, g.WW, ithresh, xcd, none);
    else
        klaunch((k_front<NW, 1, DVC_FMT_BGR, false>), grid, block, 0, s, bgr, pitch, fstride, sf, n, chunk,
                           gray_in, gray_out, gs, mbits, g.W, g.H, g.WW, ithresh, xcd, none);
}

hipError_t launch_front(const uint8_t* bgr, int pitch, size_t fstride, const SrcFmt& sf, int n, const uint8_t* gray_in,
                        uint8_t* gray_out, int gs, uint64_t* mbits, const RowGeom& g, int ithresh, hipStream_t s,
                        const FrontOut* fo)
{
    if (fo && !(fo->B == 4 ? dct4_is_const(fo->M) : fo->B == 8 && dct8_is_const(fo->M)))
        return hipErrorInvalidValue;   // the fused DCT's constant basis
    if (fo && fo->B == 8 && sf.fmt != DVC_FMT_BGR) return hipErrorInvalidValue;   // 8x8: BGR frames only
    if (fo && fo->i420 && (fo->B != 4 || g.W % 4 || g.H % 4)) return hipErrorInvalidValue;   // I420: 4x4, whole blocks
    // waves per workgroup = tile height / 4 (DVC_FRONT_NW: 4, 8 or 16; the fused outputs need 4)
    static const int nw = [] { const char* e = dvc::tune_env("DVC_FRONT_NW"); return e ? atoi(e) : 4; }();
    if (nw == 16 && !fo) launch_front_nw<16>(bgr, pitch, fstride, sf, n, gray_in, gray_out, gs, mbits, g, ithresh, s, nullptr);
    else if (nw == 8 && !(fo && (fo->B == 8 || fo->i420))) launch_front_nw<8>(bgr, pitch, fstride, sf, n, gray_in, gray_out, gs, mbits, g, ithresh, s, fo);
    else launch_front_nw<4>(bgr, pitch, fstride, sf, n, gray_in, gray_out, gs, mbits, g, ithresh, s, fo);
    return hipGetLastError();
}

// resizeGeneric_'s coefficient tables (OpenCV 4.11 resize.cpp, INTER_LINEAR,
// fixed point for 8U): fx = (float)((d + 0.5) * scale - 0.5), s = floor(fx),
// fx -= s, clamped at the borders; coefficients cvRound((1 - fx) * 2048) and
// cvRound(fx * 2048). Same restatement as oracle/dvc_oracle.c oc_linear_tab.
static void linear_tab(int ssize, int dsize, int* tab)
{
    const double inv = (double)dsize / ssize, scale = 1. / inv;
    for (int d = 0; d < dsize; ++d) {
        float f = (float)((d + 0.5) * scale - 0.5);
        int sx = (int)std::floor(f);
        f -= (float)sx;
        if (sx < 0) { f = 0.f; sx = 0; }
        if (sx >= ssize - 1) { f = 0.f; sx = ssize - 1; }
        tab[3 * d] = sx;
        tab[3 * d + 1] = std::max(-32768, std::min(32767, (int)std::nearbyint((1.f - f) * 2048.f)));
        tab[3 * d + 2] = std::max(-32768, std::min(32767, (int)std::nearbyint(f * 2048.f)));
    }
}

void resize_tables(int sw, int sh, int dw, int dh, int* host_x, int* host_y, int* area2x, int* simd_end)
{
    const double scx = 1. / ((double)dw / sw), scy = 1. / ((double)dh / sh);
    *area2x = std::fabs(scx - 2.0) < 2.220446049250313e-16 && std::fabs(scy - 2.0) < 2.220446049250313e-16;
    linear_tab(sw, dw, host_x);
    linear_tab(sh, dh, host_y);
    // VResizeLinearVec_32s8u (128-bit): 16-byte steps while x <= w - 16, then
    // 8-byte steps while x < w - 8; the scalar loop does the rest
    const int w = 3 * dw;
    int x = 0;
    while (x <= w - 16) x += 16;
    while (x < w - 8) x += 8;
    *simd_end = x;
}

hipError_t launch_resize(const uint8_t* src, int spitch, size_t sstride, uint8_t* dst, int dpitch, size_t dstride,
                         int n, const ResizeTab& t, hipStream_t s)
{
    klaunch(k_resize, dim3((t.dw + 255) / 256, t.dh, n), dim3(256), 0, s, src, spitch, sstride, dst, dpitch,
                       dstride, t);
    return hipGetLastError();
}

// LDS of one k_band workgroup: run index (2 x BH x WW u64 + 2 x BH x (WW+1)
// u16) and the band's local parents (`budget` u32).
size_t band_lds(const RowGeom& g, int bh, int budget)
{
    return (size_t)16 * bh * g.WW + (size_t)4 * bh * (g.WW + 1) + 8 + (size_t)4 * budget;
}

int band_rows(const RowGeom&) { return BAND_ROWS; }

// the largest dynamic LDS any contour-filter launch asks for at this geometry
// (k_band's run index grows with the row width: 1080p ~14 KB, W ~32k px 160 KB)
size_t ccl_max_lds(const RowGeom& g)
{
    return std::max({band_lds(g, BAND_ROWS, 1024), (size_t)8 * merge_lds_words(g.WW) * (256 / MG),
                     (size_t)8 * g.WW * cg_rows<8>()});
}

// Node budget of a band: 1024 (4 KB of parents beside the run index, ~14 KB
// per workgroup at 1080p) — bands with more runs and gaps (noise) take the
// global-array path. Interleaved A/B at 1080p against round 1's 32 KB of LDS
// per workgroup: clean 310.0 k vs 310.5 k Mpx/s, noisy 277.0 k vs 270.3 k
// (more band workgroups resident beside k_front's LDS tiles).
// DVC_BAND_LDS_KB sizes it by total LDS instead (sweeps).
static int band_budget(const RowGeom& g)
{
    static const int kb = [] { const char* e = dvc::tune_env("DVC_BAND_LDS_KB"); return e ? std::max(8, atoi(e)) : 0; }();
    const long long rest = kb * 1024LL - (long long)band_lds(g, BAND_ROWS, 0);
    return (int)std::max<long long>(1024, rest / 4);
}

hipError_t launch_ccl(const CclBufs& c, const RowGeom& g, int n, int64_t min_area2, hipStream_t s)
{
    if (!c.rowb) return hipErrorInvalidValue;   // every kernel below finds its nodes through rowb
    // DVC_CCL_SUB=F (experiment): the five kernels over sub-batches of F frames
    static const int sub = [] {
        const char* e = dvc::tune_env("DVC_CCL_SUB");
        return e ? atoi(e) : 0;
    }();
    if (sub > 0 && n > sub) {
        for (int f0 = 0; f0 < n; f0 += sub) {
            const hipError_t e = launch_ccl(c.frame(f0, g), g, std::min(sub, n - f0), min_area2, s);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    const int BH = band_rows(g), nb = (g.H + BH - 1) / BH, budget = band_budget(g);
    klaunch(k_band, dim3(nb, n), dim3(BAND_NT), band_lds(g, BH, budget), s, c, g, budget);
    if (nb > 1)
        klaunch(k_merge, dim3((nb - 1 + 256 / MG - 1) / (256 / MG), n), dim3(256),
                           8 * merge_lds_words(g.WW) * (256 / MG), s, c, g, BH);
    // row groups of 8 lanes (8 rows a wave) for launches of >= ~100 k rows (96
    // frames at 1080p), 16 below (1080p x 383: +0.8 to +2.0 %, noisy +2.6 %,
    // x 128 +0.7 %, x 96 +0.7 %, 4K x 95 +0.1 to +0.4 %; 1080p x 64 -1 %, x 32
    // -4 %: the halved workgroup count no longer fills the device); DVC_CCL_CG overrides
    static const int cg_env = [] { const char* e = dvc::tune_env("DVC_CCL_CG"); return e ? atoi(e) : 0; }();
    const int cg = cg_env == 8 || cg_env == 16 ? cg_env : ((long long)n * g.H >= 96LL * 1080 ? 8 : 16);
    if (cg == 8) {
        const int grows = (g.H + cg_rows<8>() - 1) / cg_rows<8>();
        const size_t glds = (size_t)8 * g.WW * cg_rows<8>();
        klaunch(k_resolve<8>, dim3(grows, n), dim3(256), glds, s, c, g);
        klaunch(k_area<8>, dim3(grows, n), dim3(256), glds, s, c, g);
        klaunch(k_paint<8>, dim3(grows, n), dim3(256), glds, s, c, g, min_area2);
    } else {
        const int grows = (g.H + cg_rows<16>() - 1) / cg_rows<16>();
        const size_t glds = (size_t)8 * g.WW * cg_rows<16>();
        klaunch(k_resolve<16>, dim3(grows, n), dim3(256), glds, s, c, g);
        klaunch(k_area<16>, dim3(grows, n), dim3(256), glds, s, c, g);
        klaunch(k_paint<16>, dim3(grows, n), dim3(256), glds, s, c, g, min_area2);
    }
    return hipGetLastError();
}

template <int B>
static hipError_t launch_acc(const BackArgs& a, hipStream_t s)
{
    klaunch(k_dilate<B>, dim3((a.g.WW * a.NBY + 255) / 256, a.n), dim3(256), 0, s, a);
    if (a.acc_fast)
        klaunch((k_acc<B, true>), dim3(a.SW, a.NBY), dim3(64), 0, s, a);
    else
        klaunch((k_acc<B, false>), dim3(a.SW, a.NBY), dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_accumulate(const BackArgs& a, hipStream_t s)
{
    if (a.B == 4) return launch_acc<4>(a, s);
    if (a.B == 8) return launch_acc<8>(a, s);
    klaunch(k_dilate_rows, dim3((a.g.WW * a.g.H + 255) / 256, a.n), dim3(256), 0, s, a);
    klaunch(k_acc_rows, dim3(a.g.WW, a.g.H), dim3(64), 0, s, a);
    return hipGetLastError();
}

// k_out_gen over a region, jobs of about 1024 px (at least one block)
static void launch_gen(const BackArgs& a, int rx0, int rx1, int ry0, int ry1, int jbx, int jby, int fast, hipStream_t s)
{
    if (rx0 >= rx1 || ry0 >= ry1) return;
    GenRegion R{rx0, rx1, ry0, ry1, std::max(1, std::min(jbx, rx1 - rx0)), std::max(1, std::min(jby, ry1 - ry0)), 0};
    R.njx = (rx1 - rx0 + R.jbx - 1) / R.jbx;
    const int njy = (ry1 - ry0 + R.jby - 1) / R.jby;
    const size_t lds = (size_t)8 * R.jbx * R.jby * a.B * a.B + (size_t)4 * R.jbx * R.jby;
    klaunch(k_out_gen, dim3(R.njx * njy, a.n), dim3(256), lds, s, a, R, fast);
}

hipError_t launch_out(const BackArgs& a, hipStream_t s, bool fix)
{
    const int B = a.B;
    if ((B == 4 && !dct4_is_const(a.M)) || (B == 8 && !dct8_is_const(a.M)))
        return hipErrorInvalidValue;   // k_out<4> / k_out<8>'s constant bases
    const int per = std::max(1, 1024 / (B * B));             // blocks of a ~1024-px job
    if (!fast_block(B)) {
        int jb = 1;
        while ((jb + 1) * (jb + 1) <= per) ++jb;
        launch_gen(a, 0, a.NBX, 0, a.NBY, jb, jb, 0, s);
        return hipGetLastError();
    }
    // partial edge blocks (right column, bottom row) of the fast layout
    const bool pw = a.g.W % B, ph = a.g.H % B;
    if (pw) launch_gen(a, a.NBX - 1, a.NBX, 0, a.NBY, 1, per, 1, s);
    if (ph) launch_gen(a, 0, a.NBX - (pw ? 1 : 0), a.NBY - 1, a.NBY, per, 1, 1, s);
    if (!a.overlay && !a.compressed) return hipGetLastError();
    // 128 workgroups per CU (32768 on MI355X): measured best of 8k..64k beside
    // the CCL chain at 1080p x 191 (+1 % over 64/CU); DVC_OUT_WGS overrides
    static const int wgs = [] {
        if (const char* e = dvc::tune_env("DVC_OUT_WGS")) return std::max(1, atoi(e));
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
        return 128 * cus;
    }();
    const int ntx = (a.g.W + 64 * B - 1) / (64 * B), nty = (a.g.H + 4 * B - 1) / (4 * B);
    const int grid = std::max(1, std::min(wgs, ntx * nty * a.n));
    const int f = a.sf.fmt;
    if (fix && B == 8) {   // the fused 8x8 front's fix-up: k_out's per-block pass, non-static blocks only
        if (a.out_i420 || a.obytes || f != DVC_FMT_BGR) return hipErrorInvalidValue;
        klaunch((k_out<8, DVC_FMT_BGR, true>), dim3(grid), dim3(256), 0, s, a, ntx, nty);
        return hipGetLastError();
    }
    if (fix) {   // the fused front's speculative outputs (FrontOut: B = 4, BGR out in dword rows)
        if (B != 4 || a.obytes) return hipErrorInvalidValue;   // (I420 outputs: whole 4x4 blocks, create checked)
        static const int fwgs = [] {   // DVC_FIX_WGS: k_fix4 workgroups (default 6 per CU: all resident at 79 VGPRs)
            if (const char* e = dvc::tune_env("DVC_FIX_WGS")) return std::max(1, atoi(e));
            int dev = 0, cus = 256;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
                cus = 256;
            return 6 * cus;
        }();
        if (a.SW > 64) return hipErrorInvalidValue;   // rows of <= 64 words (W <= 16384 px): the scan's lanes
        // block rows a unit (a wave): as many as the scan's 64 lanes take (8 at
        // 1080p), fewer for short batches so that the launch still has ~1024
        // waves (1080p x 1 frame: 270 one-row units instead of 34 eight-row
        // ones — 27 -> ~5 us a call for the graph path's per-frame calls)
        const int RG = std::max(1, std::min(64 / a.SW, a.NBY * a.n / 1024));
        const int units = (a.NBY + RG - 1) / RG * a.n;
        const dim3 fg(std::max(1, std::min(fwgs, (units + 3) / 4)));
        const bool oi = a.out_i420;
        if (a.sf.fmt == DVC_FMT_NV12 && oi) klaunch((k_fix4<DVC_FMT_NV12, true>), fg, dim3(256), 0, s, a, RG);
        else if (a.sf.fmt == DVC_FMT_NV12) klaunch((k_fix4<DVC_FMT_NV12, false>), fg, dim3(256), 0, s, a, RG);
        else if (a.sf.fmt == DVC_FMT_I420 && oi) klaunch((k_fix4<DVC_FMT_I420, true>), fg, dim3(256), 0, s, a, RG);
        else if (a.sf.fmt == DVC_FMT_I420) klaunch((k_fix4<DVC_FMT_I420, false>), fg, dim3(256), 0, s, a, RG);
        else if (oi) klaunch((k_fix4<DVC_FMT_BGR, true>), fg, dim3(256), 0, s, a, RG);
        else klaunch((k_fix4<DVC_FMT_BGR, false>), fg, dim3(256), 0, s, a, RG);
    }
    else if (B == 4 && f == DVC_FMT_I420) klaunch((k_out<4, DVC_FMT_I420, false>), dim3(grid), dim3(256), 0, s, a, ntx, nty);
    else if (B == 4 && f == DVC_FMT_NV12) klaunch((k_out<4, DVC_FMT_NV12, false>), dim3(grid), dim3(256), 0, s, a, ntx, nty);
    else if (B == 4) klaunch((k_out<4, DVC_FMT_BGR, false>), dim3(grid), dim3(256), 0, s, a, ntx, nty);
    else if (f == DVC_FMT_I420) klaunch((k_out<8, DVC_FMT_I420, false>), dim3(grid), dim3(256), 0, s, a, ntx, nty);
    else if (f == DVC_FMT_NV12) klaunch((k_out<8, DVC_FMT_NV12, false>), dim3(grid), dim3(256), 0, s, a, ntx, nty);
    else klaunch((k_out<8, DVC_FMT_BGR, false>), dim3(grid), dim3(256), 0, s, a, ntx, nty);
    return hipGetLastError();
}

}  // namespace dvc
