// yuv_px.h — per-pixel BT.601 conversions shared by the video-I/O kernels
// (yuv_kernels.hip) and the FD kernels reading decoder surfaces in place
// (k_front, k_out, k_out_gen) and writing encoder-ready I420 (k_out):
// OpenCV 4.11 cvtColor's fixed point
// (color_yuv.simd.hpp; restated in oracle/yuv_oracle.c). Internal.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dvc {
namespace yuvpx {

constexpr int CY = 1220542, CUB = 2116026, CUG = -409993, CVG = -852492, CVR = 1673527;
constexpr int CRY = 269484, CGY = 528482, CBY = 102760, CRU = -155188, CGU = -305135, CBU = 460324, CGV = -385875,
              CBV = -74448;
constexpr int SHIFT = 20, HALF = 1 << (SHIFT - 1);

__device__ __forceinline__ uint32_t sat8(int v) { return (uint32_t)min(max(v, 0), 255); }

// BGR2YUV_I420: luma of a pixel, chroma of the top-left pixel of a 2x2 quad
__device__ __forceinline__ uint32_t luma(int b, int g, int r)
{
    return sat8((CRY * r + CGY * g + CBY * b + HALF + (16 << SHIFT)) >> SHIFT);
}
__device__ __forceinline__ uint32_t chroma_u(int b, int g, int r)
{
    return sat8((CRU * r + CGU * g + CBU * b + HALF + (128 << SHIFT)) >> SHIFT);
}
__device__ __forceinline__ uint32_t chroma_v(int b, int g, int r)
{
    return sat8((CBU * r + CGV * g + CBV * b + HALF + (128 << SHIFT)) >> SHIFT);
}

// four bytes (each < 256) into a dword with v_perm: written as shifts and ORs,
// hipcc (ROCm 7.2) folds pairs of sat8(x >> 20) into v_ashr_pk_u8_i32, which
// keeps the upper half of its destination register, and the ORs then pick
// that garbage up (measured: every 4th converted pixel wrong)
__device__ __forceinline__ uint32_t pack4(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3)
{
    const uint32_t lo = __builtin_amdgcn_perm(b1, b0, 0x0c0c0400u);
    const uint32_t hi = __builtin_amdgcn_perm(b3, b2, 0x0c0c0400u);
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

// YUV2BGR_I420 / _NV12 of one pixel: Y and its 2x2 quad's (u, v)
__device__ __forceinline__ void yuv_px_bgr(int y, int u, int v, int& b, int& g, int& r)
{
    const int cu = u - 128, cv = v - 128, yy = max(y - 16, 0) * CY;
    b = (int)sat8((yy + HALF + CUB * cu) >> SHIFT);
    g = (int)sat8((yy + HALF + CVG * cv + CUG * cu) >> SHIFT);
    r = (int)sat8((yy + HALF + CVR * cv) >> SHIFT);
}

// 4 px of one row (x even) sharing chroma samples (u0, v0) for px 0-1 and
// (u1, v1) for px 2-3 -> 12 packed BGR bytes as 3 dwords
__device__ __forceinline__ void yuv4_bgr(uint32_t y4, int u0, int v0, int u1, int v1, uint32_t o[3])
{
    uint32_t p[12];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        int b, g, r;
        yuv_px_bgr((int)((y4 >> (8 * j)) & 255), j < 2 ? u0 : u1, j < 2 ? v0 : v1, b, g, r);
        p[3 * j] = (uint32_t)b;
        p[3 * j + 1] = (uint32_t)g;
        p[3 * j + 2] = (uint32_t)r;
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) o[d] = pack4(p[4 * d], p[4 * d + 1], p[4 * d + 2], p[4 * d + 3]);
}

}  // namespace yuvpx
}  // namespace dvc
