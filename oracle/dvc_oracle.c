/*
 * dvc_oracle.c — CPU ORACLE. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / CPU baseline. The product path
 * (dynamic-video-compression-surveillance_amd/) never links, loads or falls
 * back to it.
 *
 * A plain-C, single-threaded restatement of the reference's frame-differencing
 * per-frame worker, frame_differencing.py:67-133, with every OpenCV 4.11 call it
 * makes restated from the published algorithm (opencv-python==4.11.0.86,
 * requirements.txt:2 — not present in this container, so those semantics are
 * "OCV-unverified" here). Each function cites the
 * reference line it follows.
 *
 * Parity anchoring: the numpy-side semantics of the reference loop (mean()==0
 * gating, np.round half-to-even, float32 division, clip, truncating uint8
 * assignment, the overlay) are pinned by golden vectors captured by running the
 * UNMODIFIED reference orchestration under a cv2 shim (tests/golden/
 * make_golden.py); the contour filter here (pixel formulation) is pinned against
 * the literal Suzuki-Abe border follower + shoelace + polygon fill in
 * contours_literal.c.
 *
 * Compile with -ffp-contract=off: every fused multiply-add below is an explicit
 * fmaf() so the arithmetic order is the one the HIP kernels use.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/dvc.h"
#include "dvc_oracle.h"

/* ------------------------------------------------------------------------- */
/* OpenCV fixed-point constants (imgproc color conversions, yuv_shift = 14).   */
enum {
    OC_YUV_SHIFT = 14,
    OC_B2Y = 1868, OC_G2Y = 9617, OC_R2Y = 4899,      /* BGR2GRAY, BGR2YCrCb Y  */
    OC_YCRI = 11682, OC_YCBI = 9241,                  /* BGR2YCrCb Cr, Cb        */
    OC_CR2RI = 22987, OC_CR2GI = -11698,              /* YCrCb2BGR               */
    OC_CB2GI = -5636, OC_CB2BI = 29049,
};

static inline uint8_t sat_u8i(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }
static inline int descale14(int v) { return (v + (1 << (OC_YUV_SHIFT - 1))) >> OC_YUV_SHIFT; }

int oc_reflect101(int x, int n)
{
    if (n == 1) return 0;
    while (x < 0 || x >= n) {
        if (x < 0) x = -x;
        else x = 2 * n - 2 - x;
    }
    return x;
}

/* cvtColor(BGR2GRAY) 8U, fd:75,92: Y = (1868 B + 9617 G + 4899 R + 2^13) >> 14. */
void oc_bgr2gray(const uint8_t* bgr, size_t pitch, int W, int H, uint8_t* gray)
{
    for (int y = 0; y < H; ++y) {
        const uint8_t* s = bgr + (size_t)y * pitch;
        for (int x = 0; x < W; ++x) {
            int b = s[3 * x], g = s[3 * x + 1], r = s[3 * x + 2];
            gray[(size_t)y * W + x] = (uint8_t)descale14(b * OC_B2Y + g * OC_G2Y + r * OC_R2Y);
        }
    }
}

/*
 * getGaussianKernelBitExact + getGaussianKernelFixedPoint_ED (fraction bits 8),
 * as used by GaussianBlur for 8U (fd:77 with (25,25),30; fd:93 with (5,5),0).
 * sigma <= 0 with n in {1,3,5,7} uses OpenCV's small binomial tables.
 */
int oc_gauss_kernel_q8(int n, double sigma, uint16_t* taps)
{
    if (n < 1 || n > 63 || (n & 1) == 0) return -1;
    double k[64];
    oc_gauss_kernel_f64(n, sigma, k);
    /* error-diffused rounding to Q8, mirrored, centre = 256 - sum(sides) */
    int n2 = n / 2;
    double err = 0.0;
    int64_t sum = 0;
    for (int i = 0; i < n2; ++i) {
        double adj = k[i] * 256.0 + err;
        double v0 = nearbyint(adj); /* cvRound(softdouble): round half to even */
        err = adj - v0;
        taps[i] = (uint16_t)v0;
        taps[n - 1 - i] = (uint16_t)v0;
        sum += (int64_t)v0;
    }
    sum *= 2;
    taps[n2] = (uint16_t)(256 - sum);
    return 0;
}

/* getGaussianKernelBitExact in double (the float kernels of getGaussianKernel
 * are these values cast to float). n odd <= 63. */
void oc_gauss_kernel_f64(int n, double sigma, double* k)
{
    if (sigma <= 0 && n <= 7) {
        static const double t1[] = {1.0};
        static const double t3[] = {0.25, 0.5, 0.25};
        static const double t5[] = {0.0625, 0.25, 0.375, 0.25, 0.0625};
        static const double t7[] = {0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125};
        const double* t = n == 1 ? t1 : n == 3 ? t3 : n == 5 ? t5 : t7;
        for (int i = 0; i < n; ++i) k[i] = t[i];
    } else {
        /* sigmaX = sigma > 0 ? sigma : mulAdd(n, 0.15, 0.35) */
        double sigmaX = sigma > 0 ? sigma : fma((double)n, 0.15, 0.35);
        double scale2X = -0.125 / (sigmaX * sigmaX);
        int n2 = (n - 1) / 2;
        double values[32];
        double sum = 0.0;
        for (int i = 0, x = 1 - n; i < n2; ++i, x += 2) {
            double t = exp((double)(x * x) * scale2X);
            values[i] = t;
            sum += t;
        }
        sum *= 2.0;
        sum += 1.0;
        double mul1 = 1.0 / sum;
        for (int i = 0; i < n2; ++i) {
            double t = values[i] * mul1;
            k[i] = t;
            k[n - 1 - i] = t;
        }
        k[n2] = 1.0 * mul1;
    }
}

/*
 * GaussianBlurFixedPoint<uint8_t, ufixedpoint16> with BORDER_REFLECT_101:
 * horizontal pass in Q8 (exact in 16 bits), vertical pass in Q16,
 * out = (sum_i ky_i * (sum_j kx_j * x) + 2^15) >> 16.
 */
void oc_gaussian_q8(const uint8_t* src, int W, int H, const uint16_t* kx, int n, uint8_t* dst)
{
    int r = n / 2;
    uint32_t* hrow = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)W * H);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            uint32_t s = 0;
            for (int j = 0; j < n; ++j)
                s += (uint32_t)kx[j] * src[(size_t)y * W + oc_reflect101(x + j - r, W)];
            hrow[(size_t)y * W + x] = s;
        }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            uint64_t s = 0;
            for (int i = 0; i < n; ++i)
                s += (uint64_t)kx[i] * hrow[(size_t)oc_reflect101(y + i - r, H) * W + x];
            dst[(size_t)y * W + x] = (uint8_t)((s + 32768u) >> 16);
        }
    free(hrow);
}

/* absdiff (fd:96) + threshold(THRESH_BINARY, 255) on 8U (fd:97): OpenCV floors
 * the threshold for 8U, ithresh < 0 -> all 255, ithresh >= 255 -> all 0. */
void oc_absdiff_threshold(const uint8_t* a, const uint8_t* b, size_t n, int ithresh, uint8_t* m)
{
    for (size_t i = 0; i < n; ++i) {
        int d = a[i] > b[i] ? a[i] - b[i] : b[i] - a[i];
        m[i] = d > ithresh ? 255 : 0;
    }
}

/* ------------------------------------------------------------------------- */
/*
 * Contour-area filter, fd:100-104, pixel formulation:
 *   E  = background pixels 4-connected to the (zero-padded) image border
 *   R_i= 8-connected components of not-E (= each external component with
 *        every hole, and everything nested in a hole, filled — exactly the
 *        pixels drawContours(FILLED) paints for its external contour)
 *   2*contourArea(R_i) = 2*#{2x2 windows with 4 px in R_i} + #{windows with 3}
 *   keep R_i iff 2*area > min_area2.
 * Proven equal to the literal Suzuki-Abe path (contours_literal.c) by
 * tests/test_oracle_contours.py.
 * filled (nullable) receives not-E as {0,255}. Returns the number of R_i.
 */
int64_t oc_contour_filter(const uint8_t* mask, int W, int H, int64_t min_area2,
                          uint8_t* filtered, uint8_t* filled)
{
    size_t N = (size_t)W * H;
    uint8_t* ext = (uint8_t*)calloc(N, 1);       /* 1 = in E */
    int32_t* stack = (int32_t*)malloc(sizeof(int32_t) * (N + 1));
    int32_t* label = (int32_t*)malloc(sizeof(int32_t) * N);
    size_t sp = 0;
    /* seed E with border background pixels */
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            if (y != 0 && y != H - 1 && x != 0 && x != W - 1) continue;
            size_t i = (size_t)y * W + x;
            if (!mask[i] && !ext[i]) { ext[i] = 1; stack[sp++] = (int32_t)i; }
        }
    while (sp) {
        int32_t i = stack[--sp];
        int x = i % W, y = i / W;
        const int dx[4] = {1, -1, 0, 0}, dy[4] = {0, 0, 1, -1};
        for (int d = 0; d < 4; ++d) {
            int nx = x + dx[d], ny = y + dy[d];
            if (nx < 0 || ny < 0 || nx >= W || ny >= H) continue;
            size_t j = (size_t)ny * W + nx;
            if (!mask[j] && !ext[j]) { ext[j] = 1; stack[sp++] = (int32_t)j; }
        }
    }
    /* 8-CC labels of not-E */
    for (size_t i = 0; i < N; ++i) label[i] = -1;
    int64_t nlab = 0;
    for (size_t s = 0; s < N; ++s) {
        if (ext[s] || label[s] >= 0) continue;
        label[s] = (int32_t)nlab;
        stack[sp++] = (int32_t)s;
        while (sp) {
            int32_t i = stack[--sp];
            int x = i % W, y = i / W;
            for (int ddy = -1; ddy <= 1; ++ddy)
                for (int ddx = -1; ddx <= 1; ++ddx) {
                    int nx = x + ddx, ny = y + ddy;
                    if (nx < 0 || ny < 0 || nx >= W || ny >= H) continue;
                    size_t j = (size_t)ny * W + nx;
                    if (!ext[j] && label[j] < 0) { label[j] = (int32_t)nlab; stack[sp++] = (int32_t)j; }
                }
        }
        ++nlab;
    }
    int64_t* area2 = (int64_t*)calloc((size_t)nlab + 1, sizeof(int64_t));
    for (int y = 0; y + 1 < H; ++y)
        for (int x = 0; x + 1 < W; ++x) {
            size_t i = (size_t)y * W + x;
            int32_t l[4] = {label[i], label[i + 1], label[i + W], label[i + W + 1]};
            int c = 0, lab = -1;
            for (int k = 0; k < 4; ++k) if (l[k] >= 0) { ++c; lab = l[k]; }
            if (c == 4) area2[lab] += 2;
            else if (c == 3) area2[lab] += 1;
        }
    for (size_t i = 0; i < N; ++i) {
        if (filled) filled[i] = ext[i] ? 0 : 255;
        filtered[i] = (label[i] >= 0 && area2[label[i]] > min_area2) ? 255 : 0;
    }
    free(area2); free(label); free(stack); free(ext);
    return nlab;
}

/* dilate(src, np.ones((k,k))) with anchor (k/2,k/2), iterations=1, default
 * border (out-of-image ignored), fd:80,106. Separable max. */
void oc_dilate_rect(const uint8_t* src, int W, int H, int k, int anchor, uint8_t* dst)
{
    uint8_t* tmp = (uint8_t*)malloc((size_t)W * H);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            uint8_t m = 0;
            for (int i = 0; i < k; ++i) {
                int sx = x + i - anchor;
                if (sx < 0 || sx >= W) continue;
                uint8_t v = src[(size_t)y * W + sx];
                if (v > m) m = v;
            }
            tmp[(size_t)y * W + x] = m;
        }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            uint8_t m = 0;
            for (int i = 0; i < k; ++i) {
                int sy = y + i - anchor;
                if (sy < 0 || sy >= H) continue;
                uint8_t v = tmp[(size_t)sy * W + x];
                if (v > m) m = v;
            }
            dst[(size_t)y * W + x] = m;
        }
    free(tmp);
}

/* addWeighted 8U, fd:107: saturate_cast<uchar>(fma(a, alpha, fma(b, beta, gamma)))
 * with float32 weights and round-half-to-even (cvRound). */
uint8_t oc_add_weighted_px(uint8_t a, float alpha, uint8_t b, float beta, float gamma)
{
    float t = fmaf((float)a, alpha, fmaf((float)b, beta, gamma));
    float r = rintf(t);
    return r < 0.f ? 0 : (r > 255.f ? 255 : (uint8_t)r);
}

/* cvtColor(BGR2YCrCb) 8U, fd:115. */
void oc_bgr2ycrcb_px(const uint8_t* p, uint8_t* ycc)
{
    int b = p[0], g = p[1], r = p[2];
    int Y = descale14(b * OC_B2Y + g * OC_G2Y + r * OC_R2Y);
    int Cr = descale14((r - Y) * OC_YCRI + (128 << OC_YUV_SHIFT));
    int Cb = descale14((b - Y) * OC_YCBI + (128 << OC_YUV_SHIFT));
    ycc[0] = sat_u8i(Y); ycc[1] = sat_u8i(Cr); ycc[2] = sat_u8i(Cb);
}

/* cvtColor(YCrCb2BGR) 8U, fd:130. */
void oc_ycrcb2bgr_px(const uint8_t* ycc, uint8_t* p)
{
    int Y = ycc[0], Cr = ycc[1] - 128, Cb = ycc[2] - 128;
    int b = Y + descale14(Cb * OC_CB2BI);
    int g = Y + descale14(Cb * OC_CB2GI + Cr * OC_CR2GI);
    int r = Y + descale14(Cr * OC_CR2RI);
    p[0] = sat_u8i(b); p[1] = sat_u8i(g); p[2] = sat_u8i(r);
}

/* Orthonormal DCT-II basis, M[k][n] = c_k cos(pi (2n+1) k / 2B), float32. */
void oc_dct_matrix(int B, float* M)
{
    const double PI = 3.14159265358979323846;
    for (int k = 0; k < B; ++k)
        for (int n = 0; n < B; ++n) {
            double c = k == 0 ? sqrt(1.0 / B) : sqrt(2.0 / B);
            M[k * B + n] = (float)(c * cos(PI * (2 * n + 1) * k / (2.0 * B)));
        }
}

/*
 * cv2.dct / cv2.idct of a float32 block of bh rows x bw columns (fd:122,124;
 * of:165-168). OpenCV transforms the rows (length bw) then the columns (length
 * bh) — a single row or column (bh or bw = 1) is transformed as one 1-D signal
 * and a length-1 transform is the identity — and refuses odd lengths > 1
 * ("Odd-size DCT's are not implemented", cv::error StsNotImplemented): see
 * oc_dct_size_ok. Here each 1-D transform is the orthonormal DCT-II matrix
 * M_n (oc_dct_matrix; M_1 = [1]) applied as a float32 fmaf chain in index order
 * starting from the first product — the same chains the HIP kernels run.
 *   forward  Y = M_bh X M_bw^T : rows T[i][k] = sum_n X[i][n] M_bw[k][n],
 *                                cols Y[k][l] = sum_i M_bh[k][i] T[i][l]
 *   inverse  X = M_bh^T Y M_bw : rows T[k][n] = sum_l Y[k][l] M_bw[l][n],
 *                                cols X[i][n] = sum_k M_bh[k][i] T[k][n]
 */
int oc_dct_size_ok(int bh, int bw) { return !((bh > 1 && (bh & 1)) || (bw > 1 && (bw & 1))); }

void oc_dct2d_rect(const float* X, int bh, int bw, const float* Mh, const float* Mw, float* Y)
{
    float* T = (float*)malloc(sizeof(float) * (size_t)bh * bw);
    for (int i = 0; i < bh; ++i)
        for (int k = 0; k < bw; ++k) {
            float t = X[i * bw] * Mw[k * bw];
            for (int n = 1; n < bw; ++n) t = fmaf(X[i * bw + n], Mw[k * bw + n], t);
            T[i * bw + k] = t;
        }
    for (int k = 0; k < bh; ++k)
        for (int l = 0; l < bw; ++l) {
            float t = Mh[k * bh] * T[l];
            for (int i = 1; i < bh; ++i) t = fmaf(Mh[k * bh + i], T[i * bw + l], t);
            Y[k * bw + l] = t;
        }
    free(T);
}

void oc_idct2d_rect(const float* Y, int bh, int bw, const float* Mh, const float* Mw, float* X)
{
    float* T = (float*)malloc(sizeof(float) * (size_t)bh * bw);
    for (int k = 0; k < bh; ++k)
        for (int n = 0; n < bw; ++n) {
            float t = Y[k * bw] * Mw[n];
            for (int l = 1; l < bw; ++l) t = fmaf(Y[k * bw + l], Mw[l * bw + n], t);
            T[k * bw + n] = t;
        }
    for (int i = 0; i < bh; ++i)
        for (int n = 0; n < bw; ++n) {
            float t = Mh[i] * T[n];
            for (int k = 1; k < bh; ++k) t = fmaf(Mh[k * bh + i], T[k * bw + n], t);
            X[i * bw + n] = t;
        }
    free(T);
}

/* Square B x B forms (kept for the golden shim and the OF path). */
void oc_dct2d(const float* X, int B, const float* M, float* Y) { oc_dct2d_rect(X, B, B, M, M, Y); }
void oc_idct2d(const float* Y, int B, const float* M, float* X) { oc_idct2d_rect(Y, B, B, M, M, X); }

/*
 * One static block, fd:121-125 (and of:162-168): Y - 128 -> cv2.dct ->
 * np.round(./q)*q (float32 quotient, half-to-even) -> cv2.idct -> +128 ->
 * np.clip(0, 255) -> truncating uint8 assignment. bh x bw block (partial blocks
 * at the right / bottom edge are their slice, fd:121). Caller checks
 * oc_dct_size_ok first.
 */
void oc_block_quant_rect(const uint8_t* in, int stride, int bh, int bw, const float* Mh, const float* Mw, float q,
                         uint8_t* out, int ostride)
{
    size_t n = (size_t)bh * bw;
    float* X = (float*)calloc(n ? n : 1, sizeof(float));
    float* Y = (float*)calloc(n ? n : 1, sizeof(float));
    for (int i = 0; i < bh; ++i)
        for (int j = 0; j < bw; ++j) X[i * bw + j] = (float)in[i * stride + j] - 128.0f;
    oc_dct2d_rect(X, bh, bw, Mh, Mw, Y);
    for (size_t i = 0; i < n; ++i) Y[i] = rintf(Y[i] / q) * q;
    oc_idct2d_rect(Y, bh, bw, Mh, Mw, X);
    for (int i = 0; i < bh; ++i)
        for (int j = 0; j < bw; ++j) {
            float v = X[i * bw + j] + 128.0f;
            v = v < 0.f ? 0.f : (v > 255.f ? 255.f : v);
            out[i * ostride + j] = (uint8_t)v; /* truncation, as numpy's cast */
        }
    free(X);
    free(Y);
}

void oc_block_quant(const uint8_t* in, int stride, int B, const float* M, float q, uint8_t* out, int ostride)
{
    oc_block_quant_rect(in, stride, B, B, M, M, q, out, ostride);
}

/* ------------------------------------------------------------------------- */
/*
 * cv2.resize(frame, (dw, dh)) of 8-bit BGR with the default INTER_LINEAR
 * (fd:74, fd:91), restated from OpenCV 4.11 imgproc/src/resize.cpp:
 *  - dsize == ssize: a copy;
 *  - exact 2x downscale (scale_x == scale_y == 2.0): INTER_LINEAR becomes the
 *    fast INTER_AREA path, (a + b + c + d + 2) >> 2 per 2x2 block and channel;
 *  - otherwise resizeGeneric_ with fixed-point coefficients (INTER_RESIZE_COEF_
 *    BITS = 11): per output column fx = (float)((dx + 0.5) * scale_x - 0.5),
 *    sx = floor(fx), fx -= sx, clamped at the borders (fx = 0), alpha =
 *    (cvRound((1 - fx) * 2048), cvRound(fx * 2048)); rows likewise. Horizontal
 *    pass exact in int32: S = src[sx] * a0 + src[sx + 1] * a1. Vertical pass of
 *    each output row element x (x counts bytes, 3 per pixel):
 *      SIMD prefix (VResizeLinearVec_32s8u, 128-bit baseline: x below the end
 *      of its 16- and 8-lane loops): ((S0 >> 4) * b0 >> 16) + ((S1 >> 4) * b1
 *      >> 16), then (v + 2) >> 2 saturated;
 *      scalar tail: (S0 * b0 + S1 * b1 + 2^21) >> 22 saturated.
 * The SIMD width of the opencv-python build decides the split: parity with
 * real OpenCV is unpinned here; the HIP kernel restates
 * exactly this.
 */
static int oc_cvround_f(float v) { return (int)nearbyintf(v); }

static void oc_linear_tab(int ssize, int dsize, int* ofs, int* a0, int* a1)
{
    double inv = (double)dsize / ssize, scale = 1. / inv;
    for (int d = 0; d < dsize; ++d) {
        float f = (float)((d + 0.5) * scale - 0.5);
        int sx = (int)floorf(f);
        f -= (float)sx;
        if (sx < 0) { f = 0.f; sx = 0; }
        if (sx >= ssize - 1) { f = 0.f; sx = ssize - 1; }
        int c0 = oc_cvround_f((1.f - f) * 2048.f), c1 = oc_cvround_f(f * 2048.f);
        ofs[d] = sx;
        a0[d] = c0 < -32768 ? -32768 : (c0 > 32767 ? 32767 : c0);
        a1[d] = c1 < -32768 ? -32768 : (c1 > 32767 ? 32767 : c1);
    }
}

int oc_resize_simd_end(int width)
{
    int x = 0;
    while (x <= width - 16) x += 16;
    while (x < width - 8) x += 8;
    return x;
}

void oc_resize_bgr(const uint8_t* src, size_t spitch, int sw, int sh, uint8_t* dst, size_t dpitch, int dw, int dh)
{
    if (sw == dw && sh == dh) {
        for (int y = 0; y < sh; ++y) memcpy(dst + (size_t)y * dpitch, src + (size_t)y * spitch, (size_t)3 * sw);
        return;
    }
    double scx = 1. / ((double)dw / sw), scy = 1. / ((double)dh / sh);   /* cv::resize's scale_x, scale_y */
    if (fabs(scx - 2.0) < 2.220446049250313e-16 && fabs(scy - 2.0) < 2.220446049250313e-16) {
        for (int y = 0; y < dh; ++y)
            for (int x = 0; x < 3 * dw; ++x) {
                int c = x % 3, sx = 2 * (x / 3);
                const uint8_t* r0 = src + (size_t)(2 * y) * spitch;
                const uint8_t* r1 = r0 + spitch;
                int s = r0[3 * sx + c] + r0[3 * sx + 3 + c] + r1[3 * sx + c] + r1[3 * sx + 3 + c];
                dst[(size_t)y * dpitch + x] = (uint8_t)((s + 2) >> 2);
            }
        return;
    }
    int *xo = (int*)malloc(sizeof(int) * dw * 3), *xa = xo + dw, *xb = xa + dw;
    int *yo = (int*)malloc(sizeof(int) * dh * 3), *ya = yo + dh, *yb = ya + dh;
    oc_linear_tab(sw, dw, xo, xa, xb);
    oc_linear_tab(sh, dh, yo, ya, yb);
    int wb = 3 * dw, xs = oc_resize_simd_end(wb);
    for (int y = 0; y < dh; ++y) {
        const uint8_t* r0 = src + (size_t)yo[y] * spitch;
        const uint8_t* r1 = src + (size_t)(yo[y] + 1 < sh ? yo[y] + 1 : sh - 1) * spitch;
        int b0 = ya[y], b1 = yb[y];
        for (int x = 0; x < wb; ++x) {
            int d = x / 3, c = x % 3, sx = xo[d], sx1 = sx + 1 < sw ? sx + 1 : sx;
            int S0 = r0[3 * sx + c] * xa[d] + r0[3 * sx1 + c] * xb[d];
            int S1 = r1[3 * sx + c] * xa[d] + r1[3 * sx1 + c] * xb[d];
            int v;
            if (x < xs) {
                int h0 = ((S0 >> 4) * b0) >> 16, h1 = ((S1 >> 4) * b1) >> 16;
                v = (h0 + h1 + 2) >> 2;
            } else {
                v = (int)(((int64_t)S0 * b0 + (int64_t)S1 * b1 + (1 << 21)) >> 22);
            }
            dst[(size_t)y * dpitch + x] = sat_u8i(v);
        }
    }
    free(xo);
    free(yo);
}

/* ------------------------------------------------------------------------- */
/* The per-feed worker (fd:67-133).                                           */
struct oc_fd {
    dvc_fd_params p;
    int primed, failed;
    int sw, sh;                 /* source frame size (resized to p.width x p.height, fd:74,91) */
    uint16_t k5[5];
    uint16_t kp[64];
    float *Mb, *Mw, *Mh;        /* DCT bases of length B, W % B, H % B */
    uint8_t *prev, *gray, *cur, *motion, *filtered, *filled, *dil, *acc, *ycc, *scaled, *Yb, *Yq;
    dvc_fd_stats st;
    int use_literal;
};

oc_fd* oc_fd_create(const dvc_fd_params* p, int use_literal)
{
    if (p->width < 1 || p->height < 1 || p->block < 1 || p->block > 1024 || p->ksize < 1 || p->ksize > 1023)
        return NULL;
    if (p->src_width < 0 || p->src_height < 0) return NULL;
    oc_fd* h = (oc_fd*)calloc(1, sizeof(oc_fd));
    h->p = *p;
    h->use_literal = use_literal;
    h->sw = p->src_width ? p->src_width : p->width;
    h->sh = p->src_height ? p->src_height : p->height;
    oc_gauss_kernel_q8(5, 0.0, h->k5);
    if (oc_gauss_kernel_q8(p->prime_ksize, p->prime_sigma, h->kp) != 0) { free(h); return NULL; }
    int B = p->block, bw = p->width % B, bh = p->height % B;
    h->Mb = (float*)malloc(sizeof(float) * B * B);
    h->Mw = (float*)malloc(sizeof(float) * (bw ? bw * bw : 1));
    h->Mh = (float*)malloc(sizeof(float) * (bh ? bh * bh : 1));
    oc_dct_matrix(B, h->Mb);
    if (bw) oc_dct_matrix(bw, h->Mw);
    if (bh) oc_dct_matrix(bh, h->Mh);
    size_t N = (size_t)p->width * p->height;
    h->prev = (uint8_t*)calloc(N, 1); h->gray = (uint8_t*)calloc(N, 1);
    h->cur = (uint8_t*)calloc(N, 1); h->motion = (uint8_t*)calloc(N, 1);
    h->filtered = (uint8_t*)calloc(N, 1); h->filled = (uint8_t*)calloc(N, 1);
    h->dil = (uint8_t*)calloc(N, 1); h->acc = (uint8_t*)calloc(N, 1);
    h->ycc = (uint8_t*)calloc(N * 3, 1);
    h->scaled = (uint8_t*)calloc(N * 3, 1);
    h->Yb = (uint8_t*)calloc((size_t)B * B, 1); h->Yq = (uint8_t*)calloc((size_t)B * B, 1);
    return h;
}

void oc_fd_destroy(oc_fd* h)
{
    if (!h) return;
    free(h->prev); free(h->gray); free(h->cur); free(h->motion); free(h->filtered);
    free(h->filled); free(h->dil); free(h->acc); free(h->ycc); free(h->scaled);
    free(h->Yb); free(h->Yq); free(h->Mb); free(h->Mw); free(h->Mh); free(h);
}

/* cv2.resize(frame, (scaled_width, scaled_height)) (fd:74, fd:91): the frame
 * itself when the sizes agree, else the resized copy. */
static const uint8_t* oc_fd_input(oc_fd* h, const uint8_t* bgr, size_t* pitch)
{
    int W = h->p.width, H = h->p.height;
    if (h->sw == W && h->sh == H) return bgr;
    oc_resize_bgr(bgr, *pitch, h->sw, h->sh, h->scaled, (size_t)3 * W, W, H);
    *pitch = (size_t)3 * W;
    return h->scaled;
}

/* fd:67-81 */
int oc_fd_prime(oc_fd* h, const uint8_t* bgr, size_t pitch)
{
    int W = h->p.width, H = h->p.height;
    bgr = oc_fd_input(h, bgr, &pitch);                                      /* fd:74 */
    oc_bgr2gray(bgr, pitch, W, H, h->gray);                                 /* fd:75 */
    oc_gaussian_q8(h->gray, W, H, h->kp, h->p.prime_ksize, h->prev);        /* fd:77 */
    memset(h->acc, 0, (size_t)W * H);                                       /* fd:81 */
    memset(&h->st, 0, sizeof(h->st));
    h->primed = 1;
    h->failed = 0;
    return 0;
}

/* fd:91-133. Returns DVC_E_ODD_DCT when a static block has an odd side > 1
 * (cv2.dct raises, fd:122; the reference's try/except ends the loop, fd:140):
 * the overlay of that frame is written (fd:112 precedes the block loop), the
 * compressed frame is not, the frame is not counted and the worker stops. */
int oc_fd_step(oc_fd* h, const uint8_t* bgr, size_t pitch, uint8_t* overlay,
               uint8_t* compressed, uint8_t* acc_out)
{
    if (!h->primed || h->failed) return DVC_E_STATE;
    const dvc_fd_params* p = &h->p;
    int W = p->width, H = p->height, B = p->block;
    size_t N = (size_t)W * H;
    bgr = oc_fd_input(h, bgr, &pitch);                                     /* fd:91 */
    oc_bgr2gray(bgr, pitch, W, H, h->gray);                               /* fd:92 */
    oc_gaussian_q8(h->gray, W, H, h->k5, 5, h->cur);                       /* fd:93 */
    oc_absdiff_threshold(h->prev, h->cur, N, p->ithresh, h->motion);       /* fd:96-97 */
    int64_t ncomp;
    if (h->use_literal)                                                    /* fd:100-104 */
        ncomp = oc_contour_filter_literal(h->motion, W, H, p->min_area2, h->filtered);
    else
        ncomp = oc_contour_filter(h->motion, W, H, p->min_area2, h->filtered, h->filled);
    oc_dilate_rect(h->filtered, W, H, p->ksize, p->anchor, h->dil);        /* fd:106 */
    for (size_t i = 0; i < N; ++i)                                         /* fd:107 */
        h->acc[i] = oc_add_weighted_px(h->acc[i], p->alpha, h->dil[i], p->beta, p->gamma);
    for (int y = 0; y < H; ++y) {                                          /* fd:110-111, 115 */
        const uint8_t* s = bgr + (size_t)y * pitch;
        for (int x = 0; x < W; ++x) {
            size_t i = (size_t)y * W + x;
            uint8_t* o = overlay ? overlay + 3 * i : NULL;
            if (o) {
                if (h->acc[i] > 127) { o[0] = 0; o[1] = 0; o[2] = 255; }
                else { o[0] = s[3 * x]; o[1] = s[3 * x + 1]; o[2] = s[3 * x + 2]; }
            }
            oc_bgr2ycrcb_px(s + 3 * x, h->ycc + 3 * i);
        }
    }
    if (acc_out) memcpy(acc_out, h->acc, N);
    /* fd:117-127: B x B blocks in row-major order; the right / bottom edge blocks
     * are their partial slices (fd:120-121) */
    uint64_t nstatic = 0;
    for (int by = 0; by < H; by += B)
        for (int bx = 0; bx < W; bx += B) {
            int bh = by + B <= H ? B : H - by, bw = bx + B <= W ? B : W - bx;
            int zero = 1;
            for (int i = 0; i < bh && zero; ++i)
                for (int j = 0; j < bw; ++j)
                    if (h->acc[(size_t)(by + i) * W + bx + j]) { zero = 0; break; }
            if (!zero) continue;                                           /* fd:120 mean() == 0 */
            if (!oc_dct_size_ok(bh, bw)) { h->failed = 1; return DVC_E_ODD_DCT; }
            ++nstatic;
            for (int i = 0; i < bh; ++i)
                for (int j = 0; j < bw; ++j) h->Yb[i * bw + j] = h->ycc[3 * ((size_t)(by + i) * W + bx + j)];
            oc_block_quant_rect(h->Yb, bw, bh, bw, bh == B ? h->Mb : h->Mh, bw == B ? h->Mb : h->Mw, p->quant,
                                h->Yq, bw);
            for (int i = 0; i < bh; ++i)
                for (int j = 0; j < bw; ++j) {
                    uint8_t* c = h->ycc + 3 * ((size_t)(by + i) * W + bx + j);
                    c[0] = h->Yq[i * bw + j]; c[1] = 128; c[2] = 128;      /* fd:125-127 */
                }
        }
    if (compressed)                                                         /* fd:129-130 */
        for (size_t i = 0; i < N; ++i) oc_ycrcb2bgr_px(h->ycc + 3 * i, compressed + 3 * i);
    uint8_t* t = h->prev; h->prev = h->cur; h->cur = t;                    /* fd:133 */
    uint64_t nm = 0;
    for (size_t i = 0; i < N; ++i) nm += h->motion[i] != 0;
    h->st.frames += 1; h->st.motion_px += nm; h->st.components += (uint64_t)ncomp;
    h->st.static_blocks += nstatic;
    return 0;
}

int oc_fd_read_plane(oc_fd* h, int plane, uint8_t* dst)
{
    size_t N = (size_t)h->p.width * h->p.height;
    const uint8_t* s = plane == DVC_PLANE_GRAY ? h->prev :           /* swapped: prev = last cur */
                       plane == DVC_PLANE_MOTION ? h->motion :
                       plane == DVC_PLANE_FILTERED ? h->filtered :
                       plane == DVC_PLANE_ACC ? h->acc :
                       plane == DVC_PLANE_DILATED ? h->dil :
                       plane == 5 ? h->filled : NULL;
    if (!s) return DVC_E_INVALID;
    memcpy(dst, s, N);
    return 0;
}

void oc_fd_get_stats(oc_fd* h, dvc_fd_stats* out) { *out = h->st; }

/* Test hook: load a feed state (the previous blurred gray, fd:133, and the
 * accumulated mask, fd:107) taken from another implementation mid-sequence, so
 * the next oc_fd_step checks one transition of a long run without replaying
 * every earlier frame. */
void oc_fd_set_state(oc_fd* h, const uint8_t* prev_gray, const uint8_t* acc)
{
    size_t N = (size_t)h->p.width * h->p.height;
    memcpy(h->prev, prev_gray, N);
    memcpy(h->acc, acc, N);
    h->primed = 1;
    h->failed = 0;
}
