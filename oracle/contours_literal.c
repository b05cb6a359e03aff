/*
 * contours_literal.c — CPU ORACLE. TEST INFRASTRUCTURE ONLY.
 *
 * A literal restatement of the three OpenCV 4.11 calls of the reference's
 * contour-area filter, frame_differencing.py:100-104 (and the boundingRect
 * variant of motion_compression_opt.py:93-97):
 *
 *   findContours(mask, RETR_EXTERNAL, CHAIN_APPROX_SIMPLE)
 *       Suzuki & Abe (1985) border following on the image padded by a 1-px zero
 *       frame (foreground 8-connected, background 4-connected); RETR_EXTERNAL
 *       keeps the outer borders whose parent is the frame. Points are returned
 *       uncompressed (CHAIN_APPROX_NONE): CHAIN_APPROX_SIMPLE only drops points
 *       interior to straight horizontal/vertical/diagonal runs, which changes
 *       neither the shoelace area nor the filled pixel set.
 *   contourArea(contour)
 *       |shoelace| / 2 over the pixel-centre vertices (returned here as 2*area,
 *       an exact integer).
 *   drawContours(img, [contour], -1, 255, FILLED)
 *       edges drawn as 8-connected lines + even-odd scanline fill over the
 *       half-open edge spans [ymin, ymax) (OpenCV's CollectPolyEdges +
 *       FillEdgeCollection for integer vertices).
 *
 * This is the independent "literal" formulation that pins the pixel
 * formulation in dvc_oracle.c (tests/test_oracle_contours.py) and backs the cv2
 * shim used to capture golden vectors from the reference's own orchestration
 * (tests/golden/make_golden.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "dvc_oracle.h"

/* clockwise neighbour order in image coordinates (y down): E SE S SW W NW N NE */
static const int DX[8] = {1, 1, 0, -1, -1, -1, 0, 1};
static const int DY[8] = {0, 1, 1, 1, 0, -1, -1, -1};

static int dir_of(int dx, int dy)
{
    for (int d = 0; d < 8; ++d)
        if (DX[d] == dx && DY[d] == dy) return d;
    return -1;
}

typedef struct {
    int32_t* xy;     /* 2 ints per point */
    int64_t npts, cap;
    int32_t* off;    /* start offset (in points) of each contour; count+1 entries */
    int64_t ncont, ccap;
} contour_list;

static void cl_push_pt(contour_list* cl, int x, int y)
{
    if (cl->npts == cl->cap) {
        cl->cap = cl->cap ? cl->cap * 2 : 4096;
        cl->xy = (int32_t*)realloc(cl->xy, sizeof(int32_t) * 2 * (size_t)cl->cap);
    }
    cl->xy[2 * cl->npts] = x;
    cl->xy[2 * cl->npts + 1] = y;
    cl->npts++;
}

static void cl_begin(contour_list* cl)
{
    if (cl->ncont + 2 > cl->ccap) {
        cl->ccap = cl->ccap ? cl->ccap * 2 : 256;
        cl->off = (int32_t*)realloc(cl->off, sizeof(int32_t) * (size_t)cl->ccap);
    }
    cl->off[cl->ncont] = (int32_t)cl->npts;
}

static void cl_end(contour_list* cl)
{
    cl->ncont++;
    cl->off[cl->ncont] = (int32_t)cl->npts;
}

/*
 * Suzuki-Abe over the padded image f (Wp = W+2, Hp = H+2), f in {0,1} initially.
 * Fills `cl` with the outer borders whose parent is the frame (RETR_EXTERNAL),
 * points in original-image coordinates.
 */
static void suzuki_external(const uint8_t* mask, int W, int H, contour_list* cl)
{
    int Wp = W + 2, Hp = H + 2;
    int32_t* f = (int32_t*)calloc((size_t)Wp * Hp, sizeof(int32_t));
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) f[(size_t)(y + 1) * Wp + x + 1] = mask[(size_t)y * W + x] ? 1 : 0;
    int64_t cap = 1024;
    uint8_t* is_hole = (uint8_t*)malloc((size_t)cap);
    int64_t* parent = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap);
    int64_t nbd = 1;
    is_hole[1] = 1; /* the frame behaves as a hole border */
    parent[1] = 0;
#define F(yy, xx) f[(size_t)(yy) * Wp + (xx)]
    for (int i = 1; i < Hp - 1; ++i) {
        int64_t lnbd = 1;
        for (int j = 1; j < Wp - 1; ++j) {
            int32_t fij = F(i, j);
            if (fij == 0) continue;
            int outer = (fij == 1 && F(i, j - 1) == 0);
            int hole = !outer && (fij >= 1 && F(i, j + 1) == 0);
            if (outer || hole) {
                int i2, j2;
                nbd++;
                if (nbd >= cap) {
                    cap *= 2;
                    is_hole = (uint8_t*)realloc(is_hole, (size_t)cap);
                    parent = (int64_t*)realloc(parent, sizeof(int64_t) * (size_t)cap);
                }
                if (outer) { i2 = i; j2 = j - 1; }
                else { i2 = i; j2 = j + 1; if (fij > 1) lnbd = fij; }
                is_hole[nbd] = (uint8_t)hole;
                parent[nbd] = (is_hole[nbd] == is_hole[lnbd]) ? parent[lnbd] : lnbd;
                int record = outer && parent[nbd] == 1;
                if (record) cl_begin(cl);
                /* (3.1) clockwise from (i2,j2) around (i,j) */
                int d0 = dir_of(j2 - j, i2 - i), found = -1;
                for (int k = 0; k < 8; ++k) {
                    int d = (d0 + k) & 7;
                    if (F(i + DY[d], j + DX[d]) != 0) { found = d; break; }
                }
                if (found < 0) {
                    F(i, j) = (int32_t)-nbd;
                    if (record) { cl_push_pt(cl, j - 1, i - 1); cl_end(cl); }
                } else {
                    int i1 = i + DY[found], j1 = j + DX[found];
                    i2 = i1; j2 = j1;
                    int i3 = i, j3 = j;
                    for (;;) {
                        /* (3.3) counter-clockwise from the element after (i2,j2) */
                        int d2 = dir_of(j2 - j3, i2 - i3), i4 = 0, j4 = 0, east0 = 0;
                        for (int k = 1; k <= 8; ++k) {
                            int d = (d2 - k) & 7;
                            int yy = i3 + DY[d], xx = j3 + DX[d];
                            if (F(yy, xx) != 0) { i4 = yy; j4 = xx; break; }
                            if (d == 0) east0 = 1;
                        }
                        /* (3.4) */
                        if (east0) F(i3, j3) = (int32_t)-nbd;
                        else if (F(i3, j3) == 1) F(i3, j3) = (int32_t)nbd;
                        if (record) cl_push_pt(cl, j3 - 1, i3 - 1);
                        /* (3.5) */
                        if (i4 == i && j4 == j && i3 == i1 && j3 == j1) break;
                        i2 = i3; j2 = j3; i3 = i4; j3 = j4;
                    }
                    if (record) cl_end(cl);
                }
            }
            /* (4) */
            int32_t v = F(i, j);
            if (v != 1) lnbd = v < 0 ? -v : v;
        }
    }
#undef F
    free(is_hole); free(parent); free(f);
}

/* 2*contourArea: |sum (x_i y_{i+1} - x_{i+1} y_i)| */
int64_t oc_contour_area2(const int32_t* xy, int64_t n)
{
    if (n < 3) return 0;
    int64_t s = 0;
    for (int64_t k = 0; k < n; ++k) {
        int64_t k1 = (k + 1) % n;
        s += (int64_t)xy[2 * k] * xy[2 * k1 + 1] - (int64_t)xy[2 * k1] * xy[2 * k + 1];
    }
    return s < 0 ? -s : s;
}

typedef struct { int64_t y0, y1; int64_t x0, dx_num, dx_den; } edge_t;

static int cmp_i64(const void* a, const void* b)
{
    int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return x < y ? -1 : x > y;
}

/* 8-connected Bresenham-style line between integer points (both ends drawn). */
static void draw_line8(uint8_t* img, int W, int H, int x0, int y0, int x1, int y1, uint8_t c)
{
    int dx = abs(x1 - x0), dy = abs(y1 - y0);
    int sx = x0 < x1 ? 1 : -1, sy = y0 < y1 ? 1 : -1;
    int n = dx > dy ? dx : dy;
    /* contour edges are unit steps or straight 8-direction runs: exact lattice points */
    for (int k = 0; k <= n; ++k) {
        int x = x0 + (dx ? sx * (int)((int64_t)k * dx / n) : 0);
        int y = y0 + (dy ? sy * (int)((int64_t)k * dy / n) : 0);
        if (x >= 0 && y >= 0 && x < W && y < H) img[(size_t)y * W + x] = c;
    }
}

/* drawContours(img, [c], -1, color, FILLED) for an integer polygon. */
void oc_fill_contour(uint8_t* img, int W, int H, const int32_t* xy, int64_t n, uint8_t color)
{
    if (n <= 0) return;
    edge_t* e = (edge_t*)malloc(sizeof(edge_t) * (size_t)n);
    int64_t ne = 0, ymin = INT64_MAX, ymax = INT64_MIN;
    for (int64_t k = 0; k < n; ++k) {
        int64_t k0 = (k + n - 1) % n;
        int x0 = xy[2 * k0], y0 = xy[2 * k0 + 1], x1 = xy[2 * k], y1 = xy[2 * k + 1];
        draw_line8(img, W, H, x0, y0, x1, y1, color);
        if (y0 == y1) continue;
        if (y0 > y1) { int t = y0; y0 = y1; y1 = t; t = x0; x0 = x1; x1 = t; }
        e[ne].y0 = y0; e[ne].y1 = y1; e[ne].x0 = x0;
        e[ne].dx_num = x1 - x0; e[ne].dx_den = y1 - y0;
        if (y0 < ymin) ymin = y0;
        if (y1 > ymax) ymax = y1;
        ++ne;
    }
    int64_t* xs = (int64_t*)malloc(sizeof(int64_t) * (size_t)(ne + 1));
    for (int64_t y = ymin; y < ymax; ++y) {
        if (y < 0 || y >= H) continue;
        int64_t m = 0;
        /* x scaled by 2*den-free exactness: edges of contours have |dx/dy| in {0,1}
           or straight runs, so x is integral at integral y. */
        for (int64_t k = 0; k < ne; ++k)
            if (e[k].y0 <= y && y < e[k].y1)
                xs[m++] = e[k].x0 + (y - e[k].y0) * e[k].dx_num / e[k].dx_den;
        qsort(xs, (size_t)m, sizeof(int64_t), cmp_i64);
        for (int64_t k = 0; k + 1 < m; k += 2) {
            int64_t a = xs[k] < 0 ? 0 : xs[k], b = xs[k + 1] >= W ? W - 1 : xs[k + 1];
            for (int64_t x = a; x <= b; ++x) img[(size_t)y * W + x] = color;
        }
    }
    free(xs); free(e);
}

/* fd:100-104 literally: external contours, keep 2*area > min_area2, fill. */
int64_t oc_contour_filter_literal(const uint8_t* mask, int W, int H, int64_t min_area2, uint8_t* filtered)
{
    contour_list cl;
    memset(&cl, 0, sizeof(cl));
    cl_begin(&cl);
    suzuki_external(mask, W, H, &cl);
    memset(filtered, 0, (size_t)W * H);
    for (int64_t c = 0; c < cl.ncont; ++c) {
        const int32_t* p = cl.xy + 2 * (size_t)cl.off[c];
        int64_t n = cl.off[c + 1] - cl.off[c];
        if (oc_contour_area2(p, n) > min_area2) oc_fill_contour(filtered, W, H, p, n, 255);
    }
    int64_t nc = cl.ncont;
    free(cl.xy); free(cl.off);
    return nc;
}

/*
 * Raw access for the cv2 shim: find the external contours of `mask`.
 * Returns the number of contours; *xy_out (2 ints/point) and *off_out
 * (ncont+1 offsets) are malloc'd and must be released with oc_free().
 */
int64_t oc_find_external_contours(const uint8_t* mask, int W, int H, int32_t** xy_out, int32_t** off_out)
{
    contour_list cl;
    memset(&cl, 0, sizeof(cl));
    cl_begin(&cl);
    suzuki_external(mask, W, H, &cl);
    if (!cl.off) { cl.off = (int32_t*)malloc(sizeof(int32_t)); cl.off[0] = 0; }
    *xy_out = cl.xy;
    *off_out = cl.off;
    return cl.ncont;
}

void oc_free(void* p) { free(p); }
