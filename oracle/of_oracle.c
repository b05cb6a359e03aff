/*
 * of_oracle.c — CPU ORACLE. TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference's optical-flow path,
 * motion_compression_opt.py:29-193, with the two passes fused per frame (the
 * reference hands the mask over through lossy mp4v files, of:99-100,121-122;
 * here the exact mask goes straight to the compression stage):
 *
 *   gray (of:60,71) -> calcOpticalFlowFarneback(prev, gray, 0.3, 2, 9, 2, 5, 1.1, 0)
 *   (of:72-81) -> |flow| > 0.5 (of:82-83) -> vote over the last `window` masks,
 *   count*255 >= alpha*L*255 (of:84-86) -> MORPH_CLOSE then MORPH_OPEN with the
 *   morph_kernel x morph_kernel ellipse (of:62,89-90; default 2 = [[0,1],[1,1]])
 *   -> union of the external contours'
 *   bounding rectangles grown by one pixel right/down (of:93-97) -> on every full
 *   8x8 block whose mask is all zero: DCT quantisation of Y, Cr and Cb
 *   (of:156-168), YCrCb->BGR (of:170-171), then BGR->gray->BGR (of:174-183).
 *
 * Farneback follows OpenCV 4.11 optflowgf.cpp (pyramid of blurred + bilinearly
 * resized float images, FarnebackPolyExp, FarnebackUpdateMatrices,
 * FarnebackUpdateFlow_Blur with the box window; flags = 0), restated in plain
 * C. The 9x9 box sums of the update step follow OpenCV's running sums
 * (oc_update_flow_box_sliding) unless the handle asks for direct per-pixel
 * double sums (DVC_FLAG_OF_DIRECT_SUMS, oc_update_flow_box), and every float
 * expression is evaluated without contraction (-ffp-contract=off). The HIP
 * kernels implement both orders the same way, so each pair agrees to the last
 * bit; agreement with cv2 itself is "OCV-unverified" (no cv2 here).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/dvc.h"
#include "dvc_oracle.h"

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* GaussianBlur of a float image, separable, BORDER_REFLECT_101; symmetric taps
 * summed centre first, then k[r+i] * (s[x-i] + s[x+i]) for i = 1..r. */
void oc_blur_f32(const float* src, int W, int H, const float* k, int n, float* dst)
{
    int r = n / 2;
    float* tmp = (float*)malloc(sizeof(float) * (size_t)W * H);
    for (int y = 0; y < H; ++y) {
        const float* s = src + (size_t)y * W;
        for (int x = 0; x < W; ++x) {
            float acc = k[r] * s[x];
            for (int i = 1; i <= r; ++i) acc += k[r + i] * (s[oc_reflect101(x - i, W)] + s[oc_reflect101(x + i, W)]);
            tmp[(size_t)y * W + x] = acc;
        }
    }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            float acc = k[r] * tmp[(size_t)y * W + x];
            for (int i = 1; i <= r; ++i)
                acc += k[r + i] * (tmp[(size_t)oc_reflect101(y - i, H) * W + x] + tmp[(size_t)oc_reflect101(y + i, H) * W + x]);
            dst[(size_t)y * W + x] = acc;
        }
    free(tmp);
}

/* resize INTER_LINEAR of a float image with cn interleaved channels. */
void oc_resize_linear_f32(const float* src, int sw, int sh, int cn, float* dst, int dw, int dh)
{
    double sx_scale = (double)sw / dw, sy_scale = (double)sh / dh;
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * sy_scale - 0.5);
        int sy = (int)floorf(fy);
        fy -= (float)sy;
        if (sy < 0) { fy = 0.f; sy = 0; }
        if (sy >= sh - 1) { fy = 0.f; sy = sh - 1; }
        int sy1 = sy + 1 < sh ? sy + 1 : sh - 1;
        float b0 = 1.f - fy, b1 = fy;
        for (int dx = 0; dx < dw; ++dx) {
            float fx = (float)((dx + 0.5) * sx_scale - 0.5);
            int sx = (int)floorf(fx);
            fx -= (float)sx;
            if (sx < 0) { fx = 0.f; sx = 0; }
            if (sx >= sw - 1) { fx = 0.f; sx = sw - 1; }
            int sx1 = sx + 1 < sw ? sx + 1 : sw - 1;
            float a0 = 1.f - fx, a1 = fx;
            for (int c = 0; c < cn; ++c) {
                const float* r0 = src + (size_t)sy * sw * cn;
                const float* r1 = src + (size_t)sy1 * sw * cn;
                float t0 = r0[sx * cn + c] * a0 + r0[sx1 * cn + c] * a1;
                float t1 = r1[sx * cn + c] * a0 + r1[sx1 * cn + c] * a1;
                dst[((size_t)dy * dw + dx) * cn + c] = t0 * b0 + t1 * b1;
            }
        }
    }
}

/* FarnebackPrepareGaussian: g, xg, xxg (float, 2n+1 taps, index x+n) and the
 * needed entries of the inverse of the 6x6 moment matrix G (Cholesky, double). */
void oc_poly_gauss(int n, double sigma, float* g, float* xg, float* xxg, double* ig)
{
    if (sigma < FLT_EPSILON) sigma = n * 0.3;
    double s = 0.;
    for (int x = -n; x <= n; ++x) {
        g[x + n] = (float)exp(-x * x / (2 * sigma * sigma));
        s += g[x + n];
    }
    s = 1. / s;
    for (int x = -n; x <= n; ++x) {
        g[x + n] = (float)(g[x + n] * s);
        xg[x + n] = (float)(x * g[x + n]);
        xxg[x + n] = (float)(x * x * g[x + n]);
    }
    double G[6][6];
    memset(G, 0, sizeof(G));
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
    /* inverse by Cholesky: G = L L^T, then solve for each unit vector */
    double L[6][6];
    memset(L, 0, sizeof(L));
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j <= i; ++j) {
            double v = G[i][j];
            for (int k = 0; k < j; ++k) v -= L[i][k] * L[j][k];
            L[i][j] = (i == j) ? sqrt(v) : v / L[j][j];
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
    ig[0] = inv[1][1];  /* ig11 */
    ig[1] = inv[0][3];  /* ig03 */
    ig[2] = inv[3][3];  /* ig33 */
    ig[3] = inv[5][5];  /* ig55 */
}

/* FarnebackPolyExp: 5 coefficients per pixel (r2..r6 in OpenCV's numbering),
 * replicated borders. dst has 5 interleaved floats per pixel. */
void oc_poly_exp(const float* src, int W, int H, int n, double sigma, float* dst)
{
    float g[32], xg[32], xxg[32];
    double ig[4];
    oc_poly_gauss(n, sigma, g, xg, xxg, ig);
    float* row = (float*)malloc(sizeof(float) * 3 * (size_t)(W + 2 * n));
    float* r = row + 3 * n;
    for (int y = 0; y < H; ++y) {
        const float* s0 = src + (size_t)y * W;
        for (int x = 0; x < W; ++x) {
            r[3 * x] = s0[x] * g[n];
            r[3 * x + 1] = r[3 * x + 2] = 0.f;
        }
        for (int k = 1; k <= n; ++k) {
            float g0 = g[n + k], g1 = xg[n + k], g2 = xxg[n + k];
            const float* a = src + (size_t)clampi(y - k, 0, H - 1) * W;
            const float* b = src + (size_t)clampi(y + k, 0, H - 1) * W;
            for (int x = 0; x < W; ++x) {
                float p = a[x] + b[x];
                float t0 = r[3 * x] + g0 * p;
                float t1 = r[3 * x + 1] + g1 * (b[x] - a[x]);
                float t2 = r[3 * x + 2] + g2 * p;
                r[3 * x] = t0;
                r[3 * x + 1] = t1;
                r[3 * x + 2] = t2;
            }
        }
        for (int x = 0; x < 3 * n; ++x) {  /* replicate the row ends */
            r[-1 - x] = r[2 - x];
            r[3 * W + x] = r[3 * W + x - 3];
        }
        float* d = dst + (size_t)y * W * 5;
        /* Horizontal part with the C++ types of FarnebackPolyExp: row, g, xg,
         * xxg are float, b1..b6 double. So `row*g0`, `row[a] + row[b]` and
         * `(row[a] -/+ row[b]) * xg[k]` (both operands float) round in float
         * before widening; only `tg * g0` and `tg * xxg[k]` (tg double) are
         * double products. */
        for (int x = 0; x < W; ++x) {
            const float c0 = r[3 * x] * g[n], c1 = r[3 * x + 1] * g[n], c2 = r[3 * x + 2] * g[n];
            double b1 = c0, b2 = 0, b3 = c1, b4 = 0, b5 = c2, b6 = 0;
            for (int k = 1; k <= n; ++k) {
                const float* P = r + 3 * (x + k);
                const float* M = r + 3 * (x - k);
                const float tgf = P[0] + M[0];
                const double tg = tgf;
                b1 += tg * g[n + k];
                b4 += tg * xxg[n + k];
                const float q2 = (P[0] - M[0]) * xg[n + k];
                const float q3 = (P[1] + M[1]) * g[n + k];
                const float q6 = (P[1] - M[1]) * xg[n + k];
                const float q5 = (P[2] + M[2]) * g[n + k];
                b2 += q2;
                b3 += q3;
                b6 += q6;
                b5 += q5;
            }
            d[5 * x + 1] = (float)(b2 * ig[0]);
            d[5 * x] = (float)(b3 * ig[0]);
            d[5 * x + 3] = (float)(b1 * ig[1] + b4 * ig[2]);
            d[5 * x + 2] = (float)(b1 * ig[1] + b5 * ig[2]);
            d[5 * x + 4] = (float)(b6 * ig[3]);
        }
    }
    free(row);
}

/* FarnebackUpdateMatrices for rows [y0, y1). */
void oc_update_matrices(const float* R0, const float* R1, const float* flow, int W, int H, float* M, int y0, int y1)
{
    static const float border[5] = {0.14f, 0.14f, 0.4472f, 0.4472f, 0.4472f};
    for (int y = y0; y < y1; ++y)
        for (int x = 0; x < W; ++x) {
            const float* r0 = R0 + ((size_t)y * W + x) * 5;
            float dx = flow[((size_t)y * W + x) * 2], dy = flow[((size_t)y * W + x) * 2 + 1];
            float fx = (float)x + dx, fy = (float)y + dy;
            int x1 = (int)floorf(fx), y1i = (int)floorf(fy);
            float r2, r3, r4, r5, r6;
            fx -= (float)x1;
            fy -= (float)y1i;
            if ((unsigned)x1 < (unsigned)(W - 1) && (unsigned)y1i < (unsigned)(H - 1)) {
                const float* p = R1 + ((size_t)y1i * W + x1) * 5;
                const float* q = p + (size_t)W * 5;
                float a00 = (1.f - fx) * (1.f - fy), a01 = fx * (1.f - fy), a10 = (1.f - fx) * fy, a11 = fx * fy;
                r2 = a00 * p[0] + a01 * p[5] + a10 * q[0] + a11 * q[5];
                r3 = a00 * p[1] + a01 * p[6] + a10 * q[1] + a11 * q[6];
                r4 = a00 * p[2] + a01 * p[7] + a10 * q[2] + a11 * q[7];
                r5 = a00 * p[3] + a01 * p[8] + a10 * q[3] + a11 * q[8];
                r6 = a00 * p[4] + a01 * p[9] + a10 * q[4] + a11 * q[9];
                r4 = (r0[2] + r4) * 0.5f;
                r5 = (r0[3] + r5) * 0.5f;
                r6 = (r0[4] + r6) * 0.25f;
            } else {
                r2 = r3 = 0.f;
                r4 = r0[2];
                r5 = r0[3];
                r6 = r0[4] * 0.5f;
            }
            r2 = (r0[0] - r2) * 0.5f;
            r3 = (r0[1] - r3) * 0.5f;
            r2 += r4 * dy + r6 * dx;
            r3 += r6 * dy + r5 * dx;
            if ((unsigned)(x - 5) >= (unsigned)(W - 10) || (unsigned)(y - 5) >= (unsigned)(H - 10)) {
                float scale = (x < 5 ? border[x] : 1.f) * (x >= W - 5 ? border[W - x - 1] : 1.f) *
                              (y < 5 ? border[y] : 1.f) * (y >= H - 5 ? border[H - y - 1] : 1.f);
                r2 *= scale; r3 *= scale; r4 *= scale; r5 *= scale; r6 *= scale;
            }
            float* m = M + ((size_t)y * W + x) * 5;
            m[0] = r4 * r4 + r6 * r6;
            m[1] = (r4 + r5) * r6;
            m[2] = r5 * r5 + r6 * r6;
            m[3] = r4 * r2 + r6 * r3;
            m[4] = r6 * r2 + r5 * r3;
        }
}

/* FarnebackUpdateFlow_Blur: box-filtered (replicated borders, double sums:
 * vertical first, rows in order; then horizontal, columns in order) G and h,
 * flow = G^-1 h with the 1e-3 regulariser. */
void oc_update_flow_box(const float* M, int W, int H, int bs, float* flow)
{
    int m = bs / 2;
    double scale = 1. / (bs * bs);
    double* vs = (double*)malloc(sizeof(double) * 5 * (size_t)W);
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x)
            for (int c = 0; c < 5; ++c) {
                double s = 0;
                for (int j = -m; j <= m; ++j) s += M[((size_t)clampi(y + j, 0, H - 1) * W + x) * 5 + c];
                vs[5 * x + c] = s;
            }
        for (int x = 0; x < W; ++x) {
            double h[5] = {0, 0, 0, 0, 0};
            for (int i = -m; i <= m; ++i) {
                const double* v = vs + 5 * clampi(x + i, 0, W - 1);
                for (int c = 0; c < 5; ++c) h[c] += v[c];
            }
            double g11 = h[0] * scale, g12 = h[1] * scale, g22 = h[2] * scale, h1 = h[3] * scale, h2 = h[4] * scale;
            double idet = 1. / (g11 * g22 - g12 * g12 + 1e-3);
            flow[((size_t)y * W + x) * 2] = (float)((g11 * h2 - g12 * h1) * idet);
            flow[((size_t)y * W + x) * 2 + 1] = (float)((g22 * h1 - g12 * h2) * idet);
        }
    }
    free(vs);
}

/* FarnebackUpdateFlow_Blur exactly as OpenCV 4.11 optflowgf.cpp accumulates
 * it: a vertical running sum per column (vsum, double) initialised with row 0
 * times (m + 2) — a FLOAT product — plus rows 1..m-1, then per row
 * vsum += (float)(M[y+m] - M[y-m-1]) (the difference of two floats is rounded
 * to float before the double add); replicated borders of m + 1 columns; a
 * horizontal running sum per row initialised with vsum[0] * (m + 2) plus
 * columns 1..m-1, then g += vsum[x+m] - vsum[x-m-1] (double). Same solve.
 * Selected by oc_of_set_sliding(1); the measured difference to the direct sums
 * is reported by tests/test_of_sliding.py. */
void oc_update_flow_box_sliding(const float* M, int W, int H, int bs, float* flow)
{
    const int m = bs / 2;
    const double scale = 1. / (bs * bs);
    double* buf = (double*)malloc(sizeof(double) * 5 * (size_t)(W + 2 * m + 2));
    double* vsum = buf + (m + 1) * 5;
    const size_t rs = (size_t)W * 5;
    const float* srow0 = M;
    for (size_t x = 0; x < rs; ++x) vsum[x] = srow0[x] * (m + 2);
    for (int y = 1; y < m; ++y) {
        srow0 = M + (size_t)(y < H - 1 ? y : H - 1) * rs;
        for (size_t x = 0; x < rs; ++x) vsum[x] += srow0[x];
    }
    for (int y = 0; y < H; ++y) {
        srow0 = M + (size_t)(y - m - 1 > 0 ? y - m - 1 : 0) * rs;
        const float* srow1 = M + (size_t)(y + m < H - 1 ? y + m : H - 1) * rs;
        for (size_t x = 0; x < rs; ++x) vsum[x] += srow1[x] - srow0[x];
        for (int x = 0; x < (m + 1) * 5; ++x) {
            vsum[-1 - x] = vsum[4 - x];
            vsum[W * 5 + x] = vsum[W * 5 + x - 5];
        }
        double g11 = vsum[0] * (m + 2), g12 = vsum[1] * (m + 2), g22 = vsum[2] * (m + 2);
        double h1 = vsum[3] * (m + 2), h2 = vsum[4] * (m + 2);
        for (int x = 1; x < m; ++x) {
            g11 += vsum[x * 5];
            g12 += vsum[x * 5 + 1];
            g22 += vsum[x * 5 + 2];
            h1 += vsum[x * 5 + 3];
            h2 += vsum[x * 5 + 4];
        }
        float* fl = flow + (size_t)y * W * 2;
        for (int x = 0; x < W; ++x) {
            g11 += vsum[(x + m) * 5] - vsum[(x - m) * 5 - 5];
            g12 += vsum[(x + m) * 5 + 1] - vsum[(x - m) * 5 - 4];
            g22 += vsum[(x + m) * 5 + 2] - vsum[(x - m) * 5 - 3];
            h1 += vsum[(x + m) * 5 + 3] - vsum[(x - m) * 5 - 2];
            h2 += vsum[(x + m) * 5 + 4] - vsum[(x - m) * 5 - 1];
            const double g11_ = g11 * scale, g12_ = g12 * scale, g22_ = g22 * scale;
            const double h1_ = h1 * scale, h2_ = h2 * scale;
            const double idet = 1. / (g11_ * g22_ - g12_ * g12_ + 1e-3);
            fl[x * 2] = (float)((g11_ * h2_ - g12_ * h1_) * idet);
            fl[x * 2 + 1] = (float)((g22_ * h1_ - g12_ * h2_) * idet);
        }
    }
    free(buf);
}

static int oc_sliding = 1;   /* OpenCV's order by default */
void oc_of_set_sliding(int on) { oc_sliding = on; }

/* Pyramid level geometry of calcOpticalFlowFarneback (min_size 32). */
int oc_fb_levels(int W, int H, double pyr_scale, int levels)
{
    double scale = 1;
    int k;
    for (k = 0; k < levels; ++k) {
        scale *= pyr_scale;
        if (W * scale < 32 || H * scale < 32) break;
    }
    return k;
}

/* Blurred, resized, polynomial-expanded image of one pyramid level. */
void oc_fb_level_poly(const uint8_t* gray, int W, int H, double pyr_scale, int k, int poly_n, double poly_sigma,
                      float* R, int* lw, int* lh)
{
    double scale = 1;
    for (int i = 0; i < k; ++i) scale *= pyr_scale;
    double sigma = (1. / scale - 1) * 0.5;
    int sz = ((int)lrint(sigma * 5)) | 1;
    if (sz < 3) sz = 3;
    int w = (int)lrint(W * scale), h = (int)lrint(H * scale);
    double kd[64];
    float kf[64];
    oc_gauss_kernel_f64(sz, sigma, kd);
    for (int i = 0; i < sz; ++i) kf[i] = (float)kd[i];
    float* f = (float*)malloc(sizeof(float) * (size_t)W * H);
    float* b = (float*)malloc(sizeof(float) * (size_t)W * H);
    for (size_t i = 0; i < (size_t)W * H; ++i) f[i] = (float)gray[i];
    oc_blur_f32(f, W, H, kf, sz, b);
    float* I = (float*)malloc(sizeof(float) * (size_t)w * h);
    if (w == W && h == H) memcpy(I, b, sizeof(float) * (size_t)W * H);
    else oc_resize_linear_f32(b, W, H, 1, I, w, h);
    oc_poly_exp(I, w, h, poly_n, poly_sigma, R);
    free(f); free(b); free(I);
    *lw = w;
    *lh = h;
}

/* calcOpticalFlowFarneback(prev, next, flow, pyr_scale, levels, winsize,
 * iterations, poly_n, poly_sigma, 0) -> flow (H x W x 2). */
void oc_farneback(const uint8_t* prev, const uint8_t* next, int W, int H, double pyr_scale, int levels,
                  int winsize, int iterations, int poly_n, double poly_sigma, float* flow_out)
{
    int L = oc_fb_levels(W, H, pyr_scale, levels);
    float* prev_flow = NULL;
    int pw = 0, ph = 0;
    for (int k = L; k >= 0; --k) {
        int w, h;
        float* R0 = (float*)malloc(sizeof(float) * 5 * (size_t)W * H);
        float* R1 = (float*)malloc(sizeof(float) * 5 * (size_t)W * H);
        oc_fb_level_poly(prev, W, H, pyr_scale, k, poly_n, poly_sigma, R0, &w, &h);
        oc_fb_level_poly(next, W, H, pyr_scale, k, poly_n, poly_sigma, R1, &w, &h);
        float* flow = (float*)calloc((size_t)w * h * 2, sizeof(float));
        if (prev_flow) {
            oc_resize_linear_f32(prev_flow, pw, ph, 2, flow, w, h);
            const float up = (float)(1. / pyr_scale);  /* flow *= 1./pyr_scale (float convertTo scale) */
            for (size_t i = 0; i < (size_t)w * h * 2; ++i) flow[i] = flow[i] * up;
            free(prev_flow);
        }
        float* M = (float*)malloc(sizeof(float) * 5 * (size_t)w * h);
        oc_update_matrices(R0, R1, flow, w, h, M, 0, h);
        for (int it = 0; it < iterations; ++it) {
            if (oc_sliding) oc_update_flow_box_sliding(M, w, h, winsize, flow);
            else oc_update_flow_box(M, w, h, winsize, flow);
            if (it < iterations - 1) oc_update_matrices(R0, R1, flow, w, h, M, 0, h);
        }
        free(M); free(R0); free(R1);
        prev_flow = flow;
        pw = w;
        ph = h;
    }
    memcpy(flow_out, prev_flow, sizeof(float) * 2 * (size_t)W * H);
    free(prev_flow);
}

/* getStructuringElement(MORPH_ELLIPSE, (k, k)) (of:62; OpenCV 4.11
 * imgproc/morph.dispatch.cpp): r = c = k/2, inv_r2 = r ? 1/(r*r) : 0; row i
 * has dy = i - r and, when |dy| <= r, ones at columns [max(c - dx, 0),
 * min(c + dx + 1, k)) with dx = saturate_cast<int>(c * sqrt((r*r - dy*dy) *
 * inv_r2)) (cvRound: half to even); k = 1 is MORPH_RECT, the same [[1]].
 * k = 2 gives [[0,1],[1,1]]. el: k*k bytes. */
void oc_ellipse_element(int k, uint8_t* el)
{
    const int r = k / 2, c = k / 2;
    const double inv_r2 = r ? 1. / ((double)r * r) : 0;
    memset(el, 0, (size_t)k * k);
    for (int i = 0; i < k; ++i) {
        const int dy = i - r;
        if (abs(dy) > r) continue;
        const int dx = (int)lrint(c * sqrt((r * r - dy * dy) * inv_r2));
        const int j1 = c - dx > 0 ? c - dx : 0, j2 = c + dx + 1 < k ? c + dx + 1 : k;
        for (int j = j1; j < j2; ++j) el[i * k + j] = 1;
    }
}

/* dilate / erode with a k x k element, anchor (k/2, k/2) (the default (-1,-1)):
 * out(x, y) = max / min over el[i][j] != 0 of src(x + j - k/2, y + i - k/2);
 * out-of-image pixels are ignored (morphologyDefaultBorderValue). */
static void morph_el(const uint8_t* s, int W, int H, const uint8_t* el, int k, int dilate, uint8_t* d)
{
    const int a = k / 2;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            int v = dilate ? 0 : 255;
            for (int i = 0; i < k; ++i) {
                const int yy = y + i - a;
                if (yy < 0 || yy >= H) continue;
                for (int j = 0; j < k; ++j) {
                    const int xx = x + j - a;
                    if (!el[i * k + j] || xx < 0 || xx >= W) continue;
                    const int u = s[(size_t)yy * W + xx];
                    v = dilate ? (u > v ? u : v) : (u < v ? u : v);
                }
            }
            d[(size_t)y * W + x] = (uint8_t)v;
        }
}

/* of:89-90: morphologyEx(MORPH_CLOSE) then morphologyEx(MORPH_OPEN) with
 * getStructuringElement(MORPH_ELLIPSE, (k, k)): dilate, erode, erode, dilate. */
void oc_morph_close_open_k(const uint8_t* src, int W, int H, int k, uint8_t* dst)
{
    uint8_t* el = (uint8_t*)malloc((size_t)k * k);
    uint8_t* a = (uint8_t*)malloc((size_t)W * H);
    uint8_t* b = (uint8_t*)malloc((size_t)W * H);
    oc_ellipse_element(k, el);
    morph_el(src, W, H, el, k, 1, a);   /* close = dilate, erode */
    morph_el(a, W, H, el, k, 0, b);
    morph_el(b, W, H, el, k, 0, a);     /* open = erode, dilate */
    morph_el(a, W, H, el, k, 1, dst);
    free(el); free(a); free(b);
}

/* the reference's default element, [[0,1],[1,1]] (k = 2, of:62) */
void oc_morph_close_open(const uint8_t* src, int W, int H, uint8_t* dst) { oc_morph_close_open_k(src, W, H, 2, dst); }

/* of:93-97: union of (bounding rectangle grown by one px right/down) of every
 * 8-connected component (nested ones lie inside their parent's rectangle, so
 * RETR_EXTERNAL changes nothing). Returns the number of components. */
int64_t oc_rect_mask(const uint8_t* m, int W, int H, uint8_t* out)
{
    size_t N = (size_t)W * H;
    int32_t* lab = (int32_t*)malloc(sizeof(int32_t) * N);
    int32_t* st = (int32_t*)malloc(sizeof(int32_t) * N);
    for (size_t i = 0; i < N; ++i) lab[i] = -1;
    memset(out, 0, N);
    int64_t nl = 0;
    for (size_t s = 0; s < N; ++s) {
        if (!m[s] || lab[s] >= 0) continue;
        int x0 = W, x1 = -1, y0 = H, y1 = -1;
        size_t sp = 0;
        st[sp++] = (int32_t)s;
        lab[s] = (int32_t)nl;
        while (sp) {
            int32_t i = st[--sp];
            int x = i % W, y = i / W;
            if (x < x0) x0 = x;
            if (x > x1) x1 = x;
            if (y < y0) y0 = y;
            if (y > y1) y1 = y;
            for (int dy = -1; dy <= 1; ++dy)
                for (int dx = -1; dx <= 1; ++dx) {
                    int nx = x + dx, ny = y + dy;
                    if (nx < 0 || ny < 0 || nx >= W || ny >= H) continue;
                    size_t j = (size_t)ny * W + nx;
                    if (m[j] && lab[j] < 0) { lab[j] = (int32_t)nl; st[sp++] = (int32_t)j; }
                }
        }
        for (int y = y0; y <= y1 + 1 && y < H; ++y)
            for (int x = x0; x <= x1 + 1 && x < W; ++x) out[(size_t)y * W + x] = 255;
        ++nl;
    }
    free(lab); free(st);
    return nl;
}

/* of:151-183 for one frame: static 8x8 blocks (mask all zero, full blocks only)
 * get Y, Cr, Cb DCT-quantised, everything goes YCrCb->BGR, then static blocks
 * BGR->gray->BGR. */
void oc_of_compress(const uint8_t* bgr, size_t pitch, const uint8_t* mask, int W, int H, float q, uint8_t* out)
{
    uint8_t* ycc = (uint8_t*)malloc(3 * (size_t)W * H);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) oc_bgr2ycrcb_px(bgr + (size_t)y * pitch + 3 * x, ycc + 3 * ((size_t)y * W + x));
    float M[64];
    oc_dct_matrix(8, M);
    uint8_t blk[64], res[64];
    uint8_t* stat = (uint8_t*)calloc((size_t)(W / 8 + 1) * (H / 8 + 1), 1);
    for (int by = 0; by + 8 <= H; by += 8)
        for (int bx = 0; bx + 8 <= W; bx += 8) {
            int zero = 1;
            for (int i = 0; i < 8 && zero; ++i)
                for (int j = 0; j < 8; ++j)
                    if (mask[(size_t)(by + i) * W + bx + j]) { zero = 0; break; }
            if (!zero) continue;
            stat[(by / 8) * (W / 8 + 1) + bx / 8] = 1;
            for (int c = 0; c < 3; ++c) {
                for (int i = 0; i < 8; ++i)
                    for (int j = 0; j < 8; ++j) blk[i * 8 + j] = ycc[3 * ((size_t)(by + i) * W + bx + j) + c];
                oc_block_quant(blk, 8, 8, M, q, res, 8);
                for (int i = 0; i < 8; ++i)
                    for (int j = 0; j < 8; ++j) ycc[3 * ((size_t)(by + i) * W + bx + j) + c] = res[i * 8 + j];
            }
        }
    for (size_t i = 0; i < (size_t)W * H; ++i) oc_ycrcb2bgr_px(ycc + 3 * i, out + 3 * i);
    for (int by = 0; by + 8 <= H; by += 8)
        for (int bx = 0; bx + 8 <= W; bx += 8) {
            if (!stat[(by / 8) * (W / 8 + 1) + bx / 8]) continue;
            for (int i = 0; i < 8; ++i)
                for (int j = 0; j < 8; ++j) {
                    uint8_t* p = out + 3 * ((size_t)(by + i) * W + bx + j);
                    uint8_t g;
                    oc_bgr2gray(p, 3, 1, 1, &g);
                    p[0] = p[1] = p[2] = g;
                }
        }
    free(ycc);
    free(stat);
}

/* ------------------------------------------------------------------------- */
struct oc_of {
    dvc_of_params p;
    int primed, L;      /* frames in the vote window so far */
    uint8_t *prev, *gray, **ring, *cnt, *raw, *smooth, *morph, *rect;
    float* flow;
    int head;
};

oc_of* oc_of_create(const dvc_of_params* p)
{
    if (p->width < 1 || p->height < 1 || p->window < 1 || p->morph_kernel < 1) return NULL;
    oc_of* h = (oc_of*)calloc(1, sizeof(oc_of));
    h->p = *p;
    size_t N = (size_t)p->width * p->height;
    h->prev = (uint8_t*)calloc(N, 1); h->gray = (uint8_t*)calloc(N, 1);
    h->cnt = (uint8_t*)calloc(N, 1); h->raw = (uint8_t*)calloc(N, 1);
    h->smooth = (uint8_t*)calloc(N, 1); h->morph = (uint8_t*)calloc(N, 1); h->rect = (uint8_t*)calloc(N, 1);
    h->flow = (float*)calloc(2 * N, sizeof(float));
    h->ring = (uint8_t**)calloc((size_t)p->window, sizeof(uint8_t*));
    for (int i = 0; i < p->window; ++i) h->ring[i] = (uint8_t*)calloc(N, 1);
    return h;
}

void oc_of_destroy(oc_of* h)
{
    if (!h) return;
    for (int i = 0; i < h->p.window; ++i) free(h->ring[i]);
    free(h->ring); free(h->prev); free(h->gray); free(h->cnt); free(h->raw); free(h->smooth);
    free(h->morph); free(h->rect); free(h->flow); free(h);
}

int oc_of_prime(oc_of* h, const uint8_t* bgr, size_t pitch)
{
    oc_bgr2gray(bgr, pitch, h->p.width, h->p.height, h->prev);   /* of:60 */
    size_t N = (size_t)h->p.width * h->p.height;
    for (int i = 0; i < h->p.window; ++i) memset(h->ring[i], 0, N);
    memset(h->cnt, 0, N);
    h->L = 0;
    h->head = 0;
    h->primed = 1;
    return 0;
}

/* smallest c with c*255 >= alpha*L*255 in float64 (of:86) */
int oc_vote_threshold(double alpha, int L)
{
    double thr = alpha * L * 255;
    int c = 0;
    while (c <= L && !((double)(c * 255) >= thr)) ++c;
    return c;
}

int oc_of_step(oc_of* h, const uint8_t* bgr, size_t pitch, uint8_t* mask, uint8_t* compressed, float* flow)
{
    if (!h->primed) return DVC_E_STATE;
    const dvc_of_params* p = &h->p;
    int W = p->width, H = p->height;
    size_t N = (size_t)W * H;
    oc_bgr2gray(bgr, pitch, W, H, h->gray);                                         /* of:71 */
    const int saved = oc_sliding;                 /* the handle's box-sum order (DVC_FLAG_OF_DIRECT_SUMS) */
    oc_sliding = !(p->flags & DVC_FLAG_OF_DIRECT_SUMS);
    oc_farneback(h->prev, h->gray, W, H, p->pyr_scale, p->levels, p->winsize, p->iterations, p->poly_n,
                 p->poly_sigma, h->flow);                                           /* of:72-81 */
    oc_sliding = saved;
    uint8_t* slot = h->ring[h->head];                                               /* of:84, deque */
    for (size_t i = 0; i < N; ++i) {
        float fx = h->flow[2 * i], fy = h->flow[2 * i + 1];
        float mag = sqrtf(fx * fx + fy * fy);                                       /* of:82 */
        uint8_t v = mag > p->flow_threshold ? 1 : 0;                                /* of:83 */
        h->cnt[i] = (uint8_t)(h->cnt[i] - slot[i] + v);
        slot[i] = v;
        h->raw[i] = v ? 255 : 0;
    }
    h->head = (h->head + 1) % p->window;
    if (h->L < p->window) h->L++;
    int thr = oc_vote_threshold(p->alpha_fraction, h->L);                          /* of:85-86 */
    for (size_t i = 0; i < N; ++i) h->smooth[i] = h->cnt[i] >= thr ? 255 : 0;
    oc_morph_close_open_k(h->smooth, W, H, p->morph_kernel, h->morph);             /* of:89-90 */
    oc_rect_mask(h->morph, W, H, h->rect);                                          /* of:93-97 */
    if (mask) memcpy(mask, h->rect, N);
    if (compressed) oc_of_compress(bgr, pitch, h->rect, W, H, p->quant, compressed); /* of:141-183 */
    if (flow) memcpy(flow, h->flow, sizeof(float) * 2 * N);
    uint8_t* t = h->prev; h->prev = h->gray; h->gray = t;                          /* of:101 */
    return 0;
}

/* Test hook: load a feed state taken mid-sequence — the previous gray (of:101)
 * and the raw |flow| masks of the last n frames, oldest first (the deque,
 * of:84; nonzero = motion) — so the next oc_of_step checks one transition of a
 * long run without replaying it. */
void oc_of_set_state(oc_of* h, const uint8_t* prev_gray, const uint8_t* raw_masks, int n)
{
    size_t N = (size_t)h->p.width * h->p.height;
    int W = h->p.window;
    if (n > W) { raw_masks += (size_t)(n - W) * N; n = W; }
    memcpy(h->prev, prev_gray, N);
    for (int i = 0; i < W; ++i) memset(h->ring[i], 0, N);
    memset(h->cnt, 0, N);
    for (int k = 0; k < n; ++k)
        for (size_t i = 0; i < N; ++i) {
            uint8_t v = raw_masks[(size_t)k * N + i] ? 1 : 0;
            h->ring[k][i] = v;
            h->cnt[i] = (uint8_t)(h->cnt[i] + v);
        }
    h->L = n;
    h->head = n % W;
    h->primed = 1;
}

int oc_of_read_plane(oc_of* h, int which, uint8_t* dst)
{
    size_t N = (size_t)h->p.width * h->p.height;
    const uint8_t* s = which == 0 ? h->raw : which == 1 ? h->smooth : which == 2 ? h->morph : which == 3 ? h->rect : NULL;
    if (!s) return DVC_E_INVALID;
    memcpy(dst, s, N);
    return 0;
}
