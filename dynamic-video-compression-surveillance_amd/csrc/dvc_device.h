// dvc_device.h — device helpers shared by the FD and OF kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fd_kernels.h"

namespace dvc {

// Cumulative counters live in 64 slots x 4 so concurrent workgroups do not all
// hit one address; the host sums the slots.
#define STAT_SLOT(i) ((unsigned)(i) & 63u)

// ---------------------------------------------------------------- helpers ---
// BORDER_REFLECT_101 for -n < x < 2n-1 (one reflection; no loop, so it does
// not split a run of independent loads into waited basic blocks).
__device__ __forceinline__ int reflect1(int x, int n) { return x < 0 ? -x : (x >= n ? 2 * n - 2 - x : x); }

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ int reflect101(int x, int n)
{
    if (n == 1) return 0;
    while (x < 0 || x >= n) x = x < 0 ? -x : 2 * n - 2 - x;
    return x;
}

// OpenCV BGR2GRAY 8U: (1868 B + 9617 G + 4899 R + 2^13) >> 14
__device__ __forceinline__ uint32_t gray_px(uint32_t b, uint32_t g, uint32_t r)
{
    return (b * 1868u + g * 9617u + r * 4899u + 8192u) >> 14;
}

// 4 packed BGR pixels (12 bytes = 3 dwords, little endian) -> 4 packed gray bytes
__device__ __forceinline__ uint32_t gray4(uint32_t d0, uint32_t d1, uint32_t d2)
{
    uint32_t y0 = gray_px(d0 & 255, (d0 >> 8) & 255, (d0 >> 16) & 255);
    uint32_t y1 = gray_px(d0 >> 24, d1 & 255, (d1 >> 8) & 255);
    uint32_t y2 = gray_px((d1 >> 16) & 255, d1 >> 24, d2 & 255);
    uint32_t y3 = gray_px((d2 >> 8) & 255, (d2 >> 16) & 255, d2 >> 24);
    return y0 | (y1 << 8) | (y2 << 16) | (y3 << 24);
}

__device__ __forceinline__ uint32_t ald(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Union-find with monotone (atomicMin) links: the root of a set is its smallest
// id, every write lowers a parent to an ancestor, so concurrent finds (with path
// halving) and unions from every workgroup stay correct without locks.
inline __device__ uint32_t uf_find(uint32_t* par, uint32_t x)
{
    for (;;) {
        uint32_t p = ald(par + x);
        if (p == x) return x;
        uint32_t gp = ald(par + p);
        if (gp == p) return p;
        atomicMin(par + x, gp);
        x = gp;
    }
}

inline __device__ void uf_union(uint32_t* par, uint32_t a, uint32_t b)
{
    for (;;) {
        a = uf_find(par, a);
        b = uf_find(par, b);
        if (a == b) return;
        if (a < b) { uint32_t t = a; a = b; b = t; }
        uint32_t old = atomicMin(par + a, b);
        if (old == a) return;
        a = old;
    }
}

__device__ __forceinline__ int wave_incl_scan(int v)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

// first index in [0,n) with a[i] >= v (n if none), a ascending
template <typename T>
__device__ __forceinline__ int lower_bound(const T* a, int n, int v)
{
    int lo = 0, hi = n;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if ((int)a[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ int popc_range(const uint64_t* b, int s, int e)
{
    if (s > e) return 0;
    int ws = s >> 6, we = e >> 6;
    uint64_t ms = ~0ull << (s & 63), me = ~0ull >> (63 - (e & 63));
    if (ws == we) return __popcll(b[ws] & ms & me);
    int c = __popcll(b[ws] & ms) + __popcll(b[we] & me);
    for (int w = ws + 1; w < we; ++w) c += __popcll(b[w]);
    return c;
}

__device__ __forceinline__ int bit_at(const uint64_t* b, int x) { return (int)((b[x >> 6] >> (x & 63)) & 1ull); }

// set bits [s,e] (inclusive, clipped to word window [w0, w0+nw)) in an LDS row
__device__ __forceinline__ void paint_bits(unsigned long long* row, int w0, int nw, int s, int e)
{
    int lo = w0 * 64, hi = (w0 + nw) * 64 - 1;
    if (s < lo) s = lo;
    if (e > hi) e = hi;
    if (s > e) return;
    int ws = s >> 6, we = e >> 6;
    for (int w = ws; w <= we; ++w) {
        uint64_t m = ~0ull;
        if (w == ws) m &= ~0ull << (s & 63);
        if (w == we) m &= ~0ull >> (63 - (e & 63));
        atomicOr(row + (w - w0), (unsigned long long)m);
    }
}

__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

inline __device__ uint32_t lfind(uint32_t* lp, uint32_t x)
{
    for (;;) {
        uint32_t p = lds_ld(lp + x);
        if (p == x) return x;
        uint32_t gp = lds_ld(lp + p);
        if (gp == p) return p;
        atomicMin(lp + x, gp);
        x = gp;
    }
}

inline __device__ void lunion(uint32_t* lp, uint32_t a, uint32_t b)
{
    for (;;) {
        a = lfind(lp, a);
        b = lfind(lp, b);
        if (a == b) return;
        if (a < b) { uint32_t t = a; a = b; b = t; }
        uint32_t old = atomicMin(lp + a, b);
        if (old == a) return;
        a = old;
    }
}

// Overlapping runs / gaps of rows y and y+1 -> union (callback gets local or global ids).
template <typename FG, typename BG>
__device__ __forceinline__ void row_pair_unions(const RowGeom& g, const uint16_t* rs0, const uint16_t* re0, int n0,
                                                const uint16_t* rs1, const uint16_t* re1, int n1, FG fg, BG bg)
{
    const int lane = threadIdx.x & 63;
    // foreground, 8-connectivity: [a,b] ~ [c,d] iff c <= b+1 && d >= a-1
    for (int i = lane; i < n0; i += 64) {
        const int a = rs0[i], b = re0[i];
        for (int j = lower_bound(re1, n1, a - 1); j < n1 && (int)rs1[j] <= b + 1; ++j) fg(i, j);
    }
    // background, 4-connectivity between non-empty gaps
    for (int i = lane; i <= n0; i += 64) {
        const int ga = i == 0 ? 0 : (int)re0[i - 1] + 1;
        const int gb = i == n0 ? g.W - 1 : (int)rs0[i] - 1;
        if (ga > gb) continue;
        for (int j = lower_bound(rs1, n1, ga + 1); j <= n1; ++j) {  // first gap whose end >= ga
            const int ca = j == 0 ? 0 : (int)re1[j - 1] + 1;
            if (ca > gb) break;
            const int cb = j == n1 ? g.W - 1 : (int)rs1[j] - 1;
            if (ca <= cb) bg(i, j);
        }
    }
}

template <int B>
__device__ __forceinline__ void block_dct_quant(float (&X)[B * B], const DctMat& M, float q)
{
    float T[B * B];
    // rows: T[i][k] = sum_n X[i][n] M[k][n]
#pragma unroll
    for (int i = 0; i < B; ++i)
#pragma unroll
        for (int k = 0; k < B; ++k) {
            float t = X[i * B] * M.m[k * B];
#pragma unroll
            for (int n = 1; n < B; ++n) t = __builtin_fmaf(X[i * B + n], M.m[k * B + n], t);
            T[i * B + k] = t;
        }
    // cols + quantise: X[k][l] = rint(sum_i M[k][i] T[i][l] / q) * q
#pragma unroll
    for (int k = 0; k < B; ++k)
#pragma unroll
        for (int l = 0; l < B; ++l) {
            float t = M.m[k * B] * T[l];
#pragma unroll
            for (int i = 1; i < B; ++i) t = __builtin_fmaf(M.m[k * B + i], T[i * B + l], t);
            X[k * B + l] = __builtin_rintf(__fdiv_rn(t, q)) * q;
        }
    // inverse rows: T[k][n] = sum_l X[k][l] M[l][n]
#pragma unroll
    for (int k = 0; k < B; ++k)
#pragma unroll
        for (int n = 0; n < B; ++n) {
            float t = X[k * B] * M.m[n];
#pragma unroll
            for (int l = 1; l < B; ++l) t = __builtin_fmaf(X[k * B + l], M.m[l * B + n], t);
            T[k * B + n] = t;
        }
    // inverse cols: X[i][n] = sum_k M[k][i] T[k][n]
#pragma unroll
    for (int i = 0; i < B; ++i)
#pragma unroll
        for (int n = 0; n < B; ++n) {
            float t = M.m[i] * T[n];
#pragma unroll
            for (int k = 1; k < B; ++k) t = __builtin_fmaf(M.m[k * B + i], T[k * B + n], t);
            X[i * B + n] = t;
        }
}

__device__ __forceinline__ int descale14(int v) { return (v + 8192) >> 14; }
__device__ __forceinline__ uint32_t satu8(int v) { return (uint32_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

}  // namespace dvc
