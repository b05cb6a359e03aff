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

// The same 4 gray bytes with the v_dot4_u32_u8 unit: each coefficient split as
// 256*hi + lo, so Y*2^14 + 2^13 = (dot4(px, hi) << 8) + dot4(px, lo) + 2^13 per
// pixel (byte 3 of each operand is multiplied by 0); v_alignbyte puts pixel i's
// (b, g, r) at bytes 0..2, v_perm packs the four results. Bit-identical to gray4.
__device__ __forceinline__ uint32_t gray4_dot(uint32_t d0, uint32_t d1, uint32_t d2)
{
    constexpr uint32_t LO = 76u | (145u << 8) | (35u << 16);   // 1868, 9617, 4899 mod 256
    constexpr uint32_t HI = 7u | (37u << 8) | (19u << 16);     // ... div 256
    const uint32_t p1 = __builtin_amdgcn_alignbyte(d1, d0, 3), p2 = __builtin_amdgcn_alignbyte(d2, d1, 2);
    const uint32_t p3 = d2 >> 8;
    auto y = [](uint32_t p) {
        return ((__builtin_amdgcn_udot4(p, HI, 0u, false) << 8) + __builtin_amdgcn_udot4(p, LO, 8192u, false)) >> 14;
    };
    const uint32_t lo = __builtin_amdgcn_perm(y(p1), y(d0), 0x0c0c0400u);
    const uint32_t hi = __builtin_amdgcn_perm(y(p3), y(p2), 0x0c0c0400u);
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

// Order LDS accesses of the lanes of ONE wave (no workgroup barrier): for
// exchanges confined to a wave's own LDS slice.
__device__ __forceinline__ void wave_sync_lds()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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

// Run index of one mask row (in LDS): start / end bit words of its maximal
// foreground runs and their exclusive prefix counts (pre[w] = set bits in
// words < w, pre[WW] = runs in the row). Run k = [select(st, k), select(en, k)].
struct RowIdx {
    const uint64_t* st;
    const uint64_t* en;
    const uint16_t* ps;
    const uint16_t* pe;
};

// number of set bits at positions <= x
__device__ __forceinline__ int rank_le(const uint64_t* b, const uint16_t* pre, int WW, int x)
{
    if (x < 0) return 0;
    const int w = x >> 6;
    if (w >= WW) return pre[WW];
    return pre[w] + __popcll(b[w] & (~0ull >> (63 - (x & 63))));
}

// position of the k-th (0-based) set bit, k < pre[WW]
__device__ __forceinline__ int select_k(const uint64_t* b, const uint16_t* pre, int WW, int k)
{
    int lo = 0, hi = WW - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((int)pre[mid] <= k) lo = mid; else hi = mid - 1;
    }
    uint64_t v = b[lo];
    for (int r = k - (int)pre[lo]; r > 0; --r) v &= v - 1;
    return lo * 64 + __builtin_ctzll(v);
}

// A group of CGW lanes (aligned within the wave; 64 = the whole wave): run
// index of mask row `row` (WW words) into LDS; returns the run count;
// *motion (nullable) = this lane's share of the row's set pixels.
template <int CGW>
__device__ __forceinline__ int build_row_idx_g(const uint64_t* row, int WW, int W, uint64_t* st, uint64_t* en,
                                               uint16_t* ps, uint16_t* pe, unsigned long long* motion)
{
    const int sl = threadIdx.x & (CGW - 1);
    int ns = 0, ne = 0;
    unsigned long long m = 0;
    for (int b0 = 0; b0 < WW; b0 += CGW) {
        const int i = b0 + sl;
        const int ic = min(i, WW - 1);
        const uint64_t w0 = row[ic], pw0 = row[max(ic - 1, 0)], nw0 = row[min(ic + 1, WW - 1)];
        const uint64_t w = i < WW ? w0 : 0, pw = i > 0 && i < WW ? pw0 : 0, nw = i + 1 < WW ? nw0 : 0;
        const uint64_t s = w & ~((w << 1) | (pw >> 63));
        const uint64_t e = w & ~((w >> 1) | (nw << 63));
        const int cs = __popcll(s), ce = __popcll(e);
        int is = cs, ie = ce;
#pragma unroll
        for (int d = 1; d < CGW; d <<= 1) {
            const int ts = __shfl_up(is, d, CGW), te = __shfl_up(ie, d, CGW);
            if (sl >= d) { is += ts; ie += te; }
        }
        if (i < WW) {
            st[i] = s;
            en[i] = e;
            ps[i] = (uint16_t)(ns + is - cs);
            pe[i] = (uint16_t)(ne + ie - ce);
        }
        ns += __shfl(is, CGW - 1, CGW);
        ne += __shfl(ie, CGW - 1, CGW);
        m += (unsigned long long)__popcll(w);
    }
    if (sl == 0) {
        ps[WW] = (uint16_t)ns;
        pe[WW] = (uint16_t)ne;
    }
    if (motion) *motion = m;
    return ns;
}

__device__ __forceinline__ int build_row_idx(const uint64_t* row, int WW, int W, uint64_t* st, uint64_t* en,
                                             uint16_t* ps, uint16_t* pe, unsigned long long* motion)
{
    return build_row_idx_g<64>(row, WW, W, st, en, ps, pe, motion);
}

// Unions between the runs (8-connected) and the gaps (4-connected) of two
// consecutive rows r0 (above) and r1, by rank queries on their run indexes:
//   run i = [a,b] touches runs j of r1 with re1[j] >= a-1 and rs1[j] <= b+1;
//   gap i = [a,b] overlaps gaps j of r1 with rs1[j] >= a+1 (or j = n1) and
//   re1[j-1] <= b-1 (or j = 0).
template <int CGW = 64, typename FG, typename BG>
__device__ __forceinline__ void row_pair_unions(int W, int WW, const RowIdx& r0, int n0, const RowIdx& r1, FG fg,
                                                BG bg)
{
    const int lane = threadIdx.x & (CGW - 1);
    for (int i = lane; i < n0; i += CGW) {
        const int a = select_k(r0.st, r0.ps, WW, i), b = select_k(r0.en, r0.pe, WW, i);
        const int j0 = rank_le(r1.en, r1.pe, WW, a - 2), j1 = rank_le(r1.st, r1.ps, WW, b + 1);
        for (int j = j0; j < j1; ++j) fg(i, j);
    }
    for (int i = lane; i <= n0; i += CGW) {
        const int a = i == 0 ? 0 : select_k(r0.en, r0.pe, WW, i - 1) + 1;
        const int b = i == n0 ? W - 1 : select_k(r0.st, r0.ps, WW, i) - 1;
        if (a > b) continue;
        const int j0 = rank_le(r1.st, r1.ps, WW, a), j1 = rank_le(r1.en, r1.pe, WW, b - 1);
        for (int j = j0; j <= j1; ++j) bg(i, j);
    }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// A per-lane 32-bit byte offset re-read where it is used: keeps (wave-uniform
// base + zext(offset)) inside a loop body, so the access selects the SGPR-base
// + VGPR-offset form (global_load/store ... v_off, s[base]) instead of one
// 64-bit VALU add per access (LICM otherwise hoists the zext out of the loop
// and the addition becomes a 64-bit VGPR pair per access).
__device__ __forceinline__ uint32_t voff(uint32_t o)
{
    asm volatile("" : "+v"(o));
    return o;
}

// RN_f32(t / q) from one double product: d = RN53(t * RN53(1/q)) is within
// 2^-52 (relative) of t/q, while a float quotient t/q is never a float rounding
// midpoint (that would need 25 significant bits) and, when not equal to one,
// lies at least 2^-49 (relative) away from it — so RN24(d) == RN24(t/q) for all
// finite t and nonzero q. Three instructions instead of the IEEE division
// sequence, bit-identical results.
__device__ __forceinline__ float div_rn(float t, double qinv) { return (float)((double)t * qinv); }

template <int B>
__device__ __forceinline__ void block_dct_quant(float (&X)[B * B], const DctMat& M, float q, double qinv)
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
            X[k * B + l] = __builtin_rintf(div_rn(t, qinv)) * q;
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

// block_dct_quant with every dot product evaluated as before (first product,
// then fmaf in index order) but two independent outputs per v_pk_mul_f32 /
// v_pk_fma_f32, and the quantiser division as div_rn. Bit-identical.
template <int B>
__device__ __forceinline__ void block_dct_quant_pk(float (&X)[B * B], const DctMat& M, float q, double qinv)
{
    float T[B * B];
#pragma unroll
    for (int i = 0; i < B; ++i)
#pragma unroll
        for (int k = 0; k < B; k += 2) {
            const f32x2* mt = reinterpret_cast<const f32x2*>(M.mt + k);   // (M[k][n], M[k+1][n]) at mt[n*B/2]
            f32x2 t = (f32x2)(X[i * B]) * mt[0];
#pragma unroll
            for (int n = 1; n < B; ++n) t = __builtin_elementwise_fma((f32x2)(X[i * B + n]), mt[n * B / 2], t);
            T[i * B + k] = t.x;
            T[i * B + k + 1] = t.y;
        }
#pragma unroll
    for (int k = 0; k < B; ++k)
#pragma unroll
        for (int l = 0; l < B; l += 2) {
            f32x2 t = (f32x2)(M.m[k * B]) * (f32x2){T[l], T[l + 1]};
#pragma unroll
            for (int i = 1; i < B; ++i)
                t = __builtin_elementwise_fma((f32x2)(M.m[k * B + i]), (f32x2){T[i * B + l], T[i * B + l + 1]}, t);
            X[k * B + l] = __builtin_rintf(div_rn(t.x, qinv)) * q;
            X[k * B + l + 1] = __builtin_rintf(div_rn(t.y, qinv)) * q;
        }
#pragma unroll
    for (int k = 0; k < B; ++k)
#pragma unroll
        for (int n = 0; n < B; n += 2) {
            const f32x2* mp = reinterpret_cast<const f32x2*>(M.m + n);    // (M[l][n], M[l][n+1]) at mp[l*B/2]
            f32x2 t = (f32x2)(X[k * B]) * mp[0];
#pragma unroll
            for (int l = 1; l < B; ++l) t = __builtin_elementwise_fma((f32x2)(X[k * B + l]), mp[l * B / 2], t);
            T[k * B + n] = t.x;
            T[k * B + n + 1] = t.y;
        }
#pragma unroll
    for (int i = 0; i < B; ++i)
#pragma unroll
        for (int n = 0; n < B; n += 2) {
            f32x2 t = (f32x2)(M.m[i]) * (f32x2){T[n], T[n + 1]};
#pragma unroll
            for (int k = 1; k < B; ++k)
                t = __builtin_elementwise_fma((f32x2)(M.m[k * B + i]), (f32x2){T[k * B + n], T[k * B + n + 1]}, t);
            X[i * B + n] = t.x;
            X[i * B + n + 1] = t.y;
        }
}

// Y (BGR2YCrCb / BGR2GRAY luma) of 4 packed BGR px as four u32, via v_dot4
// (see gray4_dot).
__device__ __forceinline__ void luma4(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t (&y)[4])
{
    constexpr uint32_t LO = 76u | (145u << 8) | (35u << 16);
    constexpr uint32_t HI = 7u | (37u << 8) | (19u << 16);
    const uint32_t p[4] = {d0, __builtin_amdgcn_alignbyte(d1, d0, 3), __builtin_amdgcn_alignbyte(d2, d1, 2), d2 >> 8};
#pragma unroll
    for (int j = 0; j < 4; ++j)
        y[j] = ((__builtin_amdgcn_udot4(p[j], HI, 0u, false) << 8) + __builtin_amdgcn_udot4(p[j], LO, 8192u, false)) >> 14;
}

// 4 bytes v0..v3 (low byte of each u32) -> the 3 dwords of (v0 v0 v0)(v1 v1 v1)
// (v2 v2 v2)(v3 v3 v3) packed BGR, i.e. 4 gray pixels as BGR.
__device__ __forceinline__ void gray_bgr4(uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3, uint32_t* out)
{
    const uint32_t V = __builtin_amdgcn_perm(__builtin_amdgcn_perm(v3, v2, 0x0c0c0400u),
                                             __builtin_amdgcn_perm(v1, v0, 0x0c0c0400u), 0x05040100u);
    out[0] = __builtin_amdgcn_perm(V, V, 0x01000000u);
    out[1] = __builtin_amdgcn_perm(V, V, 0x02020101u);
    out[2] = __builtin_amdgcn_perm(V, V, 0x03030302u);
}

__device__ __forceinline__ int descale14(int v) { return (v + 8192) >> 14; }
__device__ __forceinline__ uint32_t satu8(int v) { return (uint32_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

}  // namespace dvc
