// fd_kernels.hip — gfx950 (MI355X / CDNA4) kernels of the frame-differencing
// per-frame worker (reference: frame_differencing.py:85-138).
//
// One frame = seven launches on the feed's stream:
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

#include "fd_kernels.h"

namespace dvc {

// Cumulative counters live in 64 slots x 4 (frames, motion px, components,
// static blocks) so concurrent workgroups do not all hit one address; the host
// sums the slots.
#define STAT_SLOT(i) ((unsigned)(i) & 63u)

// ---------------------------------------------------------------- helpers ---
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
__device__ uint32_t uf_find(uint32_t* par, uint32_t x)
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

__device__ void uf_union(uint32_t* par, uint32_t a, uint32_t b)
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

// ------------------------------------------------------------ prime (fd:77) -
__global__ void __launch_bounds__(256) k_gray(const uint8_t* __restrict__ bgr, int pitch,
                                              uint8_t* __restrict__ gray, int W, int H)
{
    int q = blockIdx.x * 256 + threadIdx.x;  // quad index in the row
    int y = blockIdx.y;
    if (4 * q >= W) return;
    const uint32_t* p = reinterpret_cast<const uint32_t*>(bgr + (size_t)y * pitch + 12 * q);
    *reinterpret_cast<uint32_t*>(gray + (size_t)y * W + 4 * q) = gray4(p[0], p[1], p[2]);
}

__global__ void __launch_bounds__(256) k_hblur_q8(const uint8_t* __restrict__ src, uint32_t* __restrict__ tmp,
                                                  int W, int H, GaussTaps k)
{
    int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    int r = k.n / 2;
    uint32_t s = 0;
    for (int j = 0; j < k.n; ++j) s += (uint32_t)k.t[j] * src[(size_t)y * W + reflect101(x + j - r, W)];
    tmp[(size_t)y * W + x] = s;
}

__global__ void __launch_bounds__(256) k_vblur_q8(const uint32_t* __restrict__ tmp, uint8_t* __restrict__ dst,
                                                  int W, int H, GaussTaps k)
{
    int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    int r = k.n / 2;
    uint64_t s = 0;
    for (int i = 0; i < k.n; ++i) s += (uint64_t)k.t[i] * tmp[(size_t)reflect101(y + i - r, H) * W + x];
    dst[(size_t)y * W + x] = (uint8_t)((s + 32768u) >> 16);
}

// ------------------------------------------------------------------ front ---
// Tile: 256 px (64 lanes x 4 px) x 16 rows; 4 waves. Gray halo 2 px / 2 rows,
// loaded as 66 quads x 20 rows with BORDER_REFLECT_101 at the image edges.
// Every BGR and previous-gray load of a thread is issued before the first use
// (fully unrolled), so a workgroup keeps ~6 KB of HBM reads in flight.
constexpr int FT_W = 256, FT_H = 16, FT_Q = FT_W / 4 + 2, FT_R = FT_H + 4;
constexpr int FT_ITEMS = FT_R * FT_Q, FT_NIT = (FT_ITEMS + 255) / 256;

__global__ void __launch_bounds__(256) k_front(const uint8_t* __restrict__ bgr, int pitch,
                                               const uint8_t* __restrict__ prev, uint8_t* __restrict__ cur,
                                               uint64_t* __restrict__ mbits, int W, int H, int WW, int ithresh)
{
    __shared__ uint32_t sg[FT_R][FT_Q];        // gray quads
    __shared__ uint2 sh[FT_R][FT_W / 4];       // horizontal Q8 sums, 4 x u16 per quad
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int x0 = blockIdx.x * FT_W, y0 = blockIdx.y * FT_H;
    const int x = x0 + 4 * lane;

    // previous gray of this lane's 4 output rows (independent of everything else)
    uint32_t pv[FT_H / 4];
#pragma unroll
    for (int i = 0; i < FT_H / 4; ++i) {
        const int y = y0 + wave + 4 * i;
        pv[i] = (y < H && x < W) ? *reinterpret_cast<const uint32_t*>(prev + (size_t)y * W + x) : 0u;
    }
    uint32_t v0[FT_NIT], v1[FT_NIT], v2[FT_NIT];
#pragma unroll
    for (int i = 0; i < FT_NIT; ++i) {
        const int it = tid + 256 * i;
        v0[i] = v1[i] = v2[i] = 0;
        if (it < FT_ITEMS) {
            const int r = it / FT_Q, qq = it - r * FT_Q;
            int gy = y0 - 2 + r;
            if (gy < 0 || gy >= H) gy = reflect101(gy, H);
            const int gx = x0 + 4 * (qq - 1);
            if (gx >= 0 && gx + 3 < W) {
                const uint32_t* p = reinterpret_cast<const uint32_t*>(bgr + (size_t)gy * pitch + 3 * gx);
                v0[i] = p[0];
                v1[i] = p[1];
                v2[i] = p[2];
            }
        }
    }
#pragma unroll
    for (int i = 0; i < FT_NIT; ++i) {
        const int it = tid + 256 * i;
        if (it < FT_ITEMS) {
            const int r = it / FT_Q, qq = it - r * FT_Q;
            const int gx = x0 + 4 * (qq - 1);
            uint32_t gq;
            if (gx >= 0 && gx + 3 < W) {
                gq = gray4(v0[i], v1[i], v2[i]);
            } else if (gx >= W + 2) {
                gq = 0;  // beyond every 5-tap window of an in-image pixel: never read
            } else {  // image edge: BORDER_REFLECT_101 per pixel
                int gy = y0 - 2 + r;
                if (gy < 0 || gy >= H) gy = reflect101(gy, H);
                const uint8_t* row = bgr + (size_t)gy * pitch;
                gq = 0;
                for (int j = 0; j < 4; ++j) {
                    const uint8_t* s = row + 3 * reflect101(gx + j, W);
                    gq |= gray_px(s[0], s[1], s[2]) << (8 * j);
                }
            }
            sg[r][qq] = gq;
        }
    }
    __syncthreads();

#pragma unroll
    for (int i = 0; i < (FT_R * 64 + 255) / 256; ++i) {
        const int it = tid + 256 * i;
        if (it < FT_R * 64) {
            const int r = it >> 6, q = it & 63;
            const uint32_t a = sg[r][q], b = sg[r][q + 1], c = sg[r][q + 2];
            const uint32_t p[8] = {(a >> 16) & 255, a >> 24, b & 255, (b >> 8) & 255, (b >> 16) & 255, b >> 24,
                                   c & 255, (c >> 8) & 255};
            uint32_t h[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) h[j] = p[j] + 4 * p[j + 1] + 6 * p[j + 2] + 4 * p[j + 3] + p[j + 4];
            sh[r][q] = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
        }
    }
    __syncthreads();

#pragma unroll
    for (int i = 0; i < FT_H / 4; ++i) {
        const int rr = wave + 4 * i, y = y0 + rr;
        const uint2 a0 = sh[rr][lane], a1 = sh[rr + 1][lane], a2 = sh[rr + 2][lane], a3 = sh[rr + 3][lane],
                    a4 = sh[rr + 4][lane];
        // 16-bit lanes: sum <= 16 * 4080 = 65280, packed adds cannot carry across halves
        const uint32_t sx = a0.x + 4 * a1.x + 6 * a2.x + 4 * a3.x + a4.x;
        const uint32_t sy = a0.y + 4 * a1.y + 6 * a2.y + 4 * a3.y + a4.y;
        const uint32_t g = (((sx & 0xffff) + 128) >> 8) | ((((sx >> 16) + 128) >> 8) << 8) |
                           ((((sy & 0xffff) + 128) >> 8) << 16) | ((((sy >> 16) + 128) >> 8) << 24);
        uint32_t nib = 0;
        if (y < H && x < W) {
            *reinterpret_cast<uint32_t*>(cur + (size_t)y * W + x) = g;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int da = (g >> (8 * j)) & 255, db = (pv[i] >> (8 * j)) & 255;
                const int d = da > db ? da - db : db - da;
                nib |= (uint32_t)(d > ithresh) << j;
            }
        }
        unsigned long long w = (unsigned long long)nib << (4 * (lane & 15));
        w |= __shfl_xor(w, 1, 64);
        w |= __shfl_xor(w, 2, 64);
        w |= __shfl_xor(w, 4, 64);
        w |= __shfl_xor(w, 8, 64);
        const int wi = (x0 >> 6) + (lane >> 4);
        if ((lane & 15) == 0 && y < H && wi < WW) mbits[(size_t)y * WW + wi] = w;
    }
}

// ------------------------------------------------------------------- band ---
// One workgroup per band of BH rows (one wave per row): extract the row's
// foreground runs straight from the bit mask, then union-find in LDS over the
// band's runs (8-connected) and gaps (4-connected; gaps on the image border
// joined to the OUTSIDE node), flatten, and publish every run/gap's band-local
// root as a global id. Local ids: 0 = OUTSIDE, fg (r,k) = 1 + r*CAP + k,
// gap (r,k) = 1 + BH*CAP + r*(CAP+1) + k. Dynamic LDS: local parents.
__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ uint32_t lfind(uint32_t* lp, uint32_t x)
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

__device__ void lunion(uint32_t* lp, uint32_t a, uint32_t b)
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

__global__ void __launch_bounds__(1024) k_band(const uint64_t* __restrict__ mbits, RowGeom g, int BH,
                                               uint16_t* __restrict__ rs, uint16_t* __restrict__ re,
                                               uint32_t* __restrict__ nfg, uint32_t* __restrict__ fpar,
                                               uint32_t* __restrict__ gpar, uint32_t* __restrict__ area2,
                                               unsigned long long* __restrict__ stats)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t lp[];
    __shared__ int s_n[32];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int y0 = blockIdx.x * BH, y = y0 + wave;
    const bool act = y < g.H;
    const uint32_t CAP = (uint32_t)g.CAP, FG0 = 1, GP0 = 1 + (uint32_t)BH * CAP;
    const uint32_t base = (uint32_t)y * CAP;

    // ---- phase 1: runs of row y (bit tricks + wave scan), written to global
    int n = 0;
    bool left_bg = true, right_bg = true;
    unsigned long long motion = 0;
    if (act) {
        const uint64_t* row = mbits + (size_t)y * g.WW;
        int ne = 0;
        for (int b0 = 0; b0 < g.WW; b0 += 64) {
            const int i = b0 + lane;
            uint64_t w = 0, pw = 0, nw = 0;
            if (i < g.WW) {
                w = row[i];
                pw = i > 0 ? row[i - 1] : 0;
                nw = i + 1 < g.WW ? row[i + 1] : 0;
            }
            uint64_t st = w & ~((w << 1) | (pw >> 63));
            uint64_t en = w & ~((w >> 1) | (nw << 63));
            const int cs = __popcll(st), ce = __popcll(en);
            const int ps = wave_incl_scan(cs), pe = wave_incl_scan(ce);
            int ks = n + ps - cs, ke = ne + pe - ce;
            while (st) { rs[base + ks++] = (uint16_t)(i * 64 + __ffsll((unsigned long long)st) - 1); st &= st - 1; }
            while (en) { re[base + ke++] = (uint16_t)(i * 64 + __ffsll((unsigned long long)en) - 1); en &= en - 1; }
            n += __shfl(ps, 63, 64);
            ne += __shfl(pe, 63, 64);
            motion += (unsigned long long)__popcll(w);
        }
        left_bg = !(row[0] & 1ull);
        right_bg = !((row[(g.W - 1) >> 6] >> ((g.W - 1) & 63)) & 1ull);
        for (int k = lane; k < n; k += 64) lp[FG0 + wave * CAP + k] = FG0 + wave * CAP + k;
        for (int k = lane; k <= n; k += 64) {
            const bool nonempty = (k == 0) ? left_bg : (k == n ? right_bg : true);
            const bool border = y == 0 || y == g.H - 1 || k == 0 || k == n;
            const uint32_t id = GP0 + wave * (CAP + 1) + k;
            lp[id] = (nonempty && border) ? 0u : id;
        }
        if (lane == 0) s_n[wave] = n;
    }
    if (threadIdx.x == 0) lp[0] = 0;
    for (int d = 32; d >= 1; d >>= 1) motion += __shfl_xor(motion, d, 64);
    if (lane == 0 && motion) atomicAdd(stats + STAT_SLOT(y) * 4 + 1, motion);
    __syncthreads();

    // ---- phase 2: unions between the band's consecutive rows, in LDS
    if (act && wave + 1 < BH && y + 1 < g.H) {
        const int n1 = s_n[wave + 1];
        const uint32_t f0 = FG0 + wave * CAP, f1 = f0 + CAP;
        const uint32_t q0 = GP0 + wave * (CAP + 1), q1 = q0 + CAP + 1;
        row_pair_unions(g, rs + base, re + base, n, rs + base + CAP, re + base + CAP, n1,
                        [&](int i, int j) { lunion(lp, f0 + i, f1 + j); },
                        [&](int i, int j) { lunion(lp, q0 + i, q1 + j); });
    }
    __syncthreads();

    // ---- phase 3: flatten; publish band-local roots as global ids (root = min id)
    if (act) {
        for (int k = lane; k < n; k += 64) {
            const uint32_t r = lfind(lp, FG0 + wave * CAP + k) - FG0;
            fpar[base + k] = (uint32_t)(y0 + r / CAP) * CAP + r % CAP;
            area2[base + k] = 0;
        }
        const uint32_t gbase = 1u + (uint32_t)y * (CAP + 1);
        for (int k = lane; k <= n; k += 64) {
            const uint32_t r = lfind(lp, GP0 + wave * (CAP + 1) + k);
            uint32_t gid;
            if (r == 0) gid = 0;
            else {
                const uint32_t rr = r - GP0;
                gid = 1u + (uint32_t)(y0 + rr / (CAP + 1)) * (CAP + 1) + rr % (CAP + 1);
            }
            gpar[gbase + k] = gid;
        }
        if (lane == 0) nfg[y] = (uint32_t)n;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) gpar[0] = 0;  // the OUTSIDE node is its own root
}

// ------------------------------------------------------------------ merge ---
// One wave per band seam (rows b*BH-1 and b*BH): global unions of the band
// roots, with monotone atomicMin links (uf_union).
__global__ void __launch_bounds__(64) k_merge(RowGeom g, int BH, const uint16_t* __restrict__ rs,
                                              const uint16_t* __restrict__ re, const uint32_t* __restrict__ nfg,
                                              uint32_t* fpar, uint32_t* gpar)
{
    const int y = (blockIdx.x + 1) * BH - 1;
    if (y + 1 >= g.H) return;
    const uint32_t b0 = (uint32_t)y * g.CAP, b1 = b0 + g.CAP;
    const uint32_t g0 = 1u + (uint32_t)y * (g.CAP + 1), g1 = g0 + (g.CAP + 1);
    row_pair_unions(g, rs + b0, re + b0, (int)nfg[y], rs + b1, re + b1, (int)nfg[y + 1],
                    [&](int i, int j) { uf_union(fpar, b0 + i, b1 + j); },
                    [&](int i, int j) { uf_union(gpar, g0 + i, g1 + j); });
}

// ------------------------------------------------------------------ paint ---
// One wave per row: the kept (filtered) mask, fd:101-104 — every run of a kept
// component plus the holes between its runs (drawContours FILLED).
__global__ void __launch_bounds__(64) k_paint(RowGeom g, const uint16_t* __restrict__ rs,
                                              const uint16_t* __restrict__ re, const uint32_t* __restrict__ nfg,
                                              const uint32_t* __restrict__ fpar, const uint8_t* __restrict__ gE,
                                              const uint32_t* __restrict__ area2, int64_t min_area2,
                                              uint64_t* __restrict__ kbits)
{
    extern __shared__ __attribute__((aligned(16))) unsigned long long s_k[];
    const int y = blockIdx.x, lane = threadIdx.x;
    for (int w = lane; w < g.WW; w += 64) s_k[w] = 0ull;
    __syncthreads();
    const int n = (int)nfg[y];
    const uint32_t base = (uint32_t)y * g.CAP;
    const uint8_t* ge = gE + (size_t)y * (g.CAP + 1);
    for (int k = lane; k < n; k += 64) {
        const uint32_t root = fpar[base + k];
        if (!((int64_t)area2[root] > min_area2)) continue;  // contourArea > min_area
        const int e = re[base + k];
        paint_bits(s_k, 0, g.WW, rs[base + k], e);
        if (k + 1 < n && !ge[k + 1]) paint_bits(s_k, 0, g.WW, e + 1, (int)rs[base + k + 1] - 1);
    }
    __syncthreads();
    for (int w = lane; w < g.WW; w += 64) kbits[(size_t)y * g.WW + w] = s_k[w];
}

// ---------------------------------------------------------------- resolve ---
// One wave per row. Dynamic LDS: CAP u32 roots + WW u64 filled row.
__global__ void __launch_bounds__(64) k_resolve(RowGeom g, const uint16_t* __restrict__ rs,
                                                const uint16_t* __restrict__ re, const uint32_t* __restrict__ nfg,
                                                uint32_t* fpar, uint32_t* gpar, uint8_t* __restrict__ gE,
                                                const uint64_t* __restrict__ mbits, uint64_t* __restrict__ fbits)
{
    extern __shared__ __attribute__((aligned(16))) unsigned long long s_r[];
    unsigned long long* s_f = s_r;
    uint32_t* s_root = reinterpret_cast<uint32_t*>(s_r + g.WW);
    const int y = blockIdx.x, lane = threadIdx.x;
    const int n = (int)nfg[y];
    const uint32_t base = (uint32_t)y * g.CAP, gbase = 1u + (uint32_t)y * (g.CAP + 1);
    for (int w = lane; w < g.WW; w += 64) s_f[w] = mbits[(size_t)y * g.WW + w];
    for (int k = lane; k < n; k += 64) s_root[k] = uf_find(fpar, base + k);
    __syncthreads();
    for (int k = lane; k <= n; k += 64) {
        int a = k == 0 ? 0 : (int)re[base + k - 1] + 1;
        int b = k == n ? g.W - 1 : (int)rs[base + k] - 1;
        uint8_t e = 1;
        if (a <= b) {
            uint32_t r = uf_find(gpar, gbase + k);
            atomicMin(gpar + gbase + k, r);
            e = r == 0;
            if (!e) {  // a hole: interior gap, both neighbours are runs of this row
                uf_union(fpar, s_root[k - 1], s_root[k]);
                paint_bits(s_f, 0, g.WW, a, b);
            }
        }
        gE[(size_t)y * (g.CAP + 1) + k] = e;
    }
    __syncthreads();
    for (int w = lane; w < g.WW; w += 64) fbits[(size_t)y * g.WW + w] = s_f[w];
}

// ------------------------------------------------------------------- area ---
// One wave per row y; F row y+1 staged in LDS. 2*area per filled run:
//   2*popc(F'[s..e]) - F'(s) - F'(e) + [F'(s-1)&F'(s)] + [F'(e)&F'(e+1)]
// (F' = row y+1), split additively over the runs and holes of the filled run.
__global__ void __launch_bounds__(64) k_area(RowGeom g, const uint16_t* __restrict__ rs,
                                             const uint16_t* __restrict__ re, const uint32_t* __restrict__ nfg,
                                             uint32_t* fpar, const uint8_t* __restrict__ gE,
                                             const uint64_t* __restrict__ fbits, uint32_t* __restrict__ area2,
                                             unsigned long long* __restrict__ stats)
{
    extern __shared__ __attribute__((aligned(16))) unsigned long long s_b[];
    const int y = blockIdx.x, lane = threadIdx.x;
    const int n = (int)nfg[y];
    const bool last = y == g.H - 1;
    for (int w = lane; w < g.WW; w += 64) s_b[w] = last ? 0ull : fbits[(size_t)(y + 1) * g.WW + w];
    __syncthreads();
    const uint32_t base = (uint32_t)y * g.CAP;
    const uint8_t* ge = gE + (size_t)y * (g.CAP + 1);
    const uint64_t* b = reinterpret_cast<const uint64_t*>(s_b);
    int comps = 0;
    for (int k = lane; k < n; k += 64) {
        uint32_t id = base + k;
        uint32_t r = uf_find(fpar, id);
        atomicMin(fpar + id, r);
        comps += r == id;
        if (last) continue;
        int s = rs[id], e = re[id];
        int c = 2 * popc_range(b, s, e);
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
        if (c) atomicAdd(area2 + r, (uint32_t)c);
    }
    for (int d = 32; d >= 1; d >>= 1) comps += __shfl_xor(comps, d, 64);
    if (lane == 0 && comps) atomicAdd(stats + STAT_SLOT(y) * 4 + 2, (unsigned long long)comps);
}

// ------------------------------------------------------------------- back ---
// Tile: 64 blocks across (64*B px) x 4 block rows (4*B rows), one wave per
// block row, one lane per BxB block. Kept-mask window rows [y0-anchor,
// y0+4B-1+ksize-1-anchor], words [x0/64-1, x0/64+B] in LDS.
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

template <int B>
__global__ void __launch_bounds__(256) k_back(BackArgs a)
{
    constexpr int TW = 64 * B, TH = 4 * B, NWD = B + 2, MAXR = TH + 63;
    __shared__ unsigned long long s_k[MAXR][NWD];   // kept (filtered) mask window
    __shared__ unsigned long long s_h[MAXR][B];     // horizontally dilated
    __shared__ unsigned long long s_v[TH][B];       // dilated
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int x0 = blockIdx.x * TW, y0 = blockIdx.y * TH;
    const int k = a.ksize, an = a.anchor, NR = TH + k - 1;
    const int wx0 = (x0 >> 6) - 1;

    // this lane's BxB block of BGR and accumulated mask: issued first, so the HBM
    // latency hides under the kept-mask/dilation phases below
    const int bx = x0 + lane * B, by = y0 + wave * B;
    const bool active = bx < a.g.W && by < a.g.H;
    uint32_t px[B][3 * B / 4];   // BGR, B px per row = 3B/4 dwords
    uint32_t acv[B][B / 4];
    if (active) {
#pragma unroll
        for (int i = 0; i < B; ++i) {
            const uint32_t* src = reinterpret_cast<const uint32_t*>(a.bgr + (size_t)(by + i) * a.pitch + 3 * bx);
#pragma unroll
            for (int d = 0; d < 3 * B / 4; ++d) px[i][d] = src[d];
            const uint32_t* ac = reinterpret_cast<const uint32_t*>(a.acc + (size_t)(by + i) * a.g.W + bx);
#pragma unroll
            for (int d = 0; d < B / 4; ++d) acv[i][d] = ac[d];
        }
    }

    // kept-mask window (k_paint): rows outside the image and words outside the row are 0
    for (int i = tid; i < NR * NWD; i += 256) {
        const int r = i / NWD, c = i % NWD, gy = y0 - an + r, gw = wx0 + c;
        s_k[r][c] = (gy >= 0 && gy < a.g.H && gw >= 0 && gw < a.g.WW) ? a.kbits[(size_t)gy * a.g.WW + gw] : 0ull;
    }
    __syncthreads();
    // horizontal dilation: out bit x = OR src bits x-an .. x+k-1-an
    for (int i = tid; i < NR * B; i += 256) {
        int r = i / B, c = i % B + 1;
        uint64_t pv = s_k[r][c - 1], cv = s_k[r][c], nv = s_k[r][c + 1];
        uint64_t o = 0;
        for (int off = -an; off <= k - 1 - an; ++off) {
            if (off == 0) o |= cv;
            else if (off > 0) o |= (cv >> off) | (nv << (64 - off));
            else o |= (cv << -off) | (pv >> (64 + off));
        }
        s_h[r][c - 1] = o;
    }
    __syncthreads();
    for (int i = tid; i < TH * B; i += 256) {
        int rr = i / B, c = i % B;
        uint64_t o = 0;
        for (int j = 0; j < k; ++j) o |= s_h[rr + j][c];
        s_v[rr][c] = o;
    }
    __syncthreads();
    if (a.dbg_dil) {
        for (int i = tid; i < TH * B; i += 256) {
            int rr = i / B, c = i % B, gy = y0 + rr, gw = (x0 >> 6) + c;
            if (gy < a.g.H && gw < a.g.WW) a.dbg_dil[(size_t)gy * a.g.WW + gw] = s_v[rr][c];
        }
    }

    // per-block work: wave -> block row, lane -> block
    bool is_static = false;
    if (active) {
        const int W = a.g.W;
        uint32_t accn[B][B / 4];
        bool zero = true;
#pragma unroll
        for (int i = 0; i < B; ++i) {
            uint64_t dw = s_v[wave * B + i][(lane * B) >> 6] >> ((lane * B) & 63);
#pragma unroll
            for (int d = 0; d < B / 4; ++d) {
                uint32_t av = acv[i][d], nv = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float dil = (float)(((dw >> (4 * d + j)) & 1ull) ? 255 : 0);
                    float t = __builtin_fmaf((float)((av >> (8 * j)) & 255), a.alpha, __builtin_fmaf(dil, a.beta, a.gamma));
                    float rr = __builtin_rintf(t);
                    uint32_t v = rr < 0.f ? 0u : (rr > 255.f ? 255u : (uint32_t)rr);
                    nv |= v << (8 * j);
                }
                accn[i][d] = nv;
                zero = zero && nv == 0;
            }
        }
        is_static = zero;
        // accumulated mask + overlay (fd:107, 110-111)
#pragma unroll
        for (int i = 0; i < B; ++i) {
            const int yy = by + i;
            uint32_t* ac = reinterpret_cast<uint32_t*>(a.acc + (size_t)yy * W + bx);
#pragma unroll
            for (int d = 0; d < B / 4; ++d) ac[d] = accn[i][d];
            if (a.overlay) {
                uint8_t ob[3 * B];
#pragma unroll
                for (int j = 0; j < B; ++j) {
                    uint32_t av = (accn[i][j >> 2] >> (8 * (j & 3))) & 255;
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        int bi = 3 * j + c;
                        uint32_t v = (px[i][bi >> 2] >> (8 * (bi & 3))) & 255;
                        ob[bi] = av > 127 ? (c == 2 ? 255 : 0) : (uint8_t)v;
                    }
                }
                uint32_t* o = reinterpret_cast<uint32_t*>(a.overlay + (size_t)yy * a.opitch + 3 * bx);
#pragma unroll
                for (int d = 0; d < 3 * B / 4; ++d)
                    o[d] = ob[4 * d] | (ob[4 * d + 1] << 8) | (ob[4 * d + 2] << 16) | ((uint32_t)ob[4 * d + 3] << 24);
            }
        }
        // YCrCb, static-block DCT quantisation, YCrCb -> BGR (fd:115-130)
        if (a.compressed) {
            uint8_t Y[B][B], Cr[B][B], Cb[B][B];
#pragma unroll
            for (int i = 0; i < B; ++i)
#pragma unroll
                for (int j = 0; j < B; ++j) {
                    int b = (px[i][(3 * j) >> 2] >> (8 * ((3 * j) & 3))) & 255;
                    int gg = (px[i][(3 * j + 1) >> 2] >> (8 * ((3 * j + 1) & 3))) & 255;
                    int r = (px[i][(3 * j + 2) >> 2] >> (8 * ((3 * j + 2) & 3))) & 255;
                    int yv = descale14(b * 1868 + gg * 9617 + r * 4899);
                    Y[i][j] = (uint8_t)satu8(yv);
                    Cr[i][j] = (uint8_t)satu8(descale14((r - yv) * 11682 + (128 << 14)));
                    Cb[i][j] = (uint8_t)satu8(descale14((b - yv) * 9241 + (128 << 14)));
                }
            if (is_static) {
                float X[B * B];
#pragma unroll
                for (int i = 0; i < B; ++i)
#pragma unroll
                    for (int j = 0; j < B; ++j) X[i * B + j] = (float)Y[i][j] - 128.0f;
                block_dct_quant<B>(X, a.M, a.quant);
#pragma unroll
                for (int i = 0; i < B; ++i)
#pragma unroll
                    for (int j = 0; j < B; ++j) {
                        float v = X[i * B + j] + 128.0f;
                        v = v < 0.f ? 0.f : (v > 255.f ? 255.f : v);
                        Y[i][j] = (uint8_t)(uint32_t)v;
                    }
            }
#pragma unroll
            for (int i = 0; i < B; ++i) {
                uint8_t ob[3 * B];
#pragma unroll
                for (int j = 0; j < B; ++j) {
                    int yv = Y[i][j];
                    if (is_static) {
                        ob[3 * j] = ob[3 * j + 1] = ob[3 * j + 2] = (uint8_t)yv;
                    } else {
                        int cr = Cr[i][j] - 128, cb = Cb[i][j] - 128;
                        ob[3 * j] = (uint8_t)satu8(yv + descale14(cb * 29049));
                        ob[3 * j + 1] = (uint8_t)satu8(yv + descale14(cb * -5636 + cr * -11698));
                        ob[3 * j + 2] = (uint8_t)satu8(yv + descale14(cr * 22987));
                    }
                }
                uint32_t* o = reinterpret_cast<uint32_t*>(a.compressed + (size_t)(by + i) * a.opitch + 3 * bx);
#pragma unroll
                for (int d = 0; d < 3 * B / 4; ++d)
                    o[d] = ob[4 * d] | (ob[4 * d + 1] << 8) | (ob[4 * d + 2] << 16) | ((uint32_t)ob[4 * d + 3] << 24);
            }
        }
    }
    unsigned long long bal = __ballot(active && is_static);
    if (lane == 0 && bal)
        atomicAdd(a.stats + STAT_SLOT(blockIdx.x * 4 + blockIdx.y * 7 + wave) * 4 + 3, (unsigned long long)__popcll(bal));
}

// --------------------------------------------------------------- launchers --
hipError_t launch_prime(const uint8_t* bgr, int pitch, uint8_t* gray_tmp, uint32_t* tmp32, uint8_t* out,
                        int W, int H, const GaussTaps& k, hipStream_t s)
{
    dim3 gq((W / 4 + 255) / 256, H), gp((W + 255) / 256, H);
    hipLaunchKernelGGL(k_gray, gq, dim3(256), 0, s, bgr, pitch, gray_tmp, W, H);
    hipLaunchKernelGGL(k_hblur_q8, gp, dim3(256), 0, s, gray_tmp, tmp32, W, H, k);
    hipLaunchKernelGGL(k_vblur_q8, gp, dim3(256), 0, s, tmp32, out, W, H, k);
    return hipGetLastError();
}

hipError_t launch_front(const uint8_t* bgr, int pitch, const uint8_t* prev, uint8_t* cur, uint64_t* mbits,
                        const RowGeom& g, int ithresh, hipStream_t s)
{
    dim3 grid((g.W + FT_W - 1) / FT_W, (g.H + FT_H - 1) / FT_H);
    hipLaunchKernelGGL(k_front, grid, dim3(256), 0, s, bgr, pitch, prev, cur, mbits, g.W, g.H, g.WW, ithresh);
    return hipGetLastError();
}

// Rows per band: the band's local parents (BH x (2 CAP + 1) u32) must fit LDS.
int band_rows(const RowGeom& g)
{
    int bh = 16;
    while (bh > 1 && (size_t)bh * (2 * g.CAP + 1) * 4 + 16 > 128 * 1024) bh >>= 1;
    return bh;
}

hipError_t launch_ccl(const CclBufs& c, const RowGeom& g, int64_t min_area2, hipStream_t s)
{
    const int BH = band_rows(g), nb = (g.H + BH - 1) / BH;
    const size_t lds = ((size_t)BH * (2 * g.CAP + 1) + 1) * 4;
    hipLaunchKernelGGL(k_band, dim3(nb), dim3(64 * BH), lds, s, c.mbits, g, BH, c.rs, c.re, c.nfg, c.fpar, c.gpar,
                       c.area2, c.stats);
    if (nb > 1) hipLaunchKernelGGL(k_merge, dim3(nb - 1), dim3(64), 0, s, g, BH, c.rs, c.re, c.nfg, c.fpar, c.gpar);
    hipLaunchKernelGGL(k_resolve, dim3(g.H), dim3(64), 8 * g.WW + 4 * g.CAP + 16, s, g, c.rs, c.re, c.nfg,
                       c.fpar, c.gpar, c.gE, c.mbits, c.fbits);
    hipLaunchKernelGGL(k_area, dim3(g.H), dim3(64), 8 * g.WW, s, g, c.rs, c.re, c.nfg, c.fpar, c.gE, c.fbits,
                       c.area2, c.stats);
    hipLaunchKernelGGL(k_paint, dim3(g.H), dim3(64), 8 * g.WW, s, g, c.rs, c.re, c.nfg, c.fpar, c.gE, c.area2,
                       min_area2, c.kbits);
    return hipGetLastError();
}

hipError_t launch_back(const BackArgs& a, int block, hipStream_t s)
{
    if (block == 4) {
        dim3 grid((a.g.W + 255) / 256, (a.g.H + 15) / 16);
        hipLaunchKernelGGL(k_back<4>, grid, dim3(256), 0, s, a);
    } else {
        dim3 grid((a.g.W + 511) / 512, (a.g.H + 31) / 32);
        hipLaunchKernelGGL(k_back<8>, grid, dim3(256), 0, s, a);
    }
    return hipGetLastError();
}

}  // namespace dvc
