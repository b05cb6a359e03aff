/*
 * sanitize_main.c — TEST INFRASTRUCTURE ONLY: drives the oracle's FD and OF
 * workers (and the primitives the golden shim calls) on small synthetic clips
 * of awkward geometry, built with -fsanitize=address,undefined by
 * `make sanitize` (tests/test_sanitizers.py runs it): out-of-bounds accesses,
 * leaks, signed overflow or misaligned loads in the restatement fail the run.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dvc_oracle.h"

static void frame(uint8_t* f, int W, int H, int t, unsigned seed)
{
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            for (int c = 0; c < 3; ++c)
                f[((size_t)y * W + x) * 3 + c] = (uint8_t)(28 + (37 * x + 11 * (c + 1) * y + 29 * c) % 200);
    int s = W / 6 + 2, px = (3 * t + (int)seed) % (W - s), py = (2 * t + (int)seed) % (H - s);   /* a moving block */
    for (int y = py; y < py + s; ++y)
        for (int x = px; x < px + s; ++x) f[((size_t)y * W + x) * 3] = (uint8_t)(200 + seed);
    for (int i = 0; i < W * H / 50; ++i) {                                                         /* noise */
        unsigned r = (unsigned)(i * 2654435761u + (unsigned)t * 40503u + seed);
        f[(r % (unsigned)(W * H)) * 3 + 1] ^= 3;
    }
}

static int run_fd(int sw, int sh, int W, int H, int block, int k, float r, int nf)
{
    dvc_fd_params p;
    memset(&p, 0, sizeof(p));
    p.width = W; p.height = H; p.block = block; p.ithresh = 0; p.min_area2 = 40; p.ksize = k; p.anchor = k / 2;
    p.alpha = r; p.beta = 1.f - r; p.gamma = 0.f; p.quant = 100.f; p.prime_ksize = 25; p.prime_sigma = 30.0;
    p.src_width = sw; p.src_height = sh;
    oc_fd* h = oc_fd_create(&p, 0);
    oc_fd* hl = oc_fd_create(&p, 1);          /* literal Suzuki path too */
    if (!h || !hl) return 1;
    uint8_t* f = malloc((size_t)sw * sh * 3);
    uint8_t *ov = malloc((size_t)W * H * 3), *cp = malloc((size_t)W * H * 3), *acc = malloc((size_t)W * H);
    frame(f, sw, sh, 0, 1);
    oc_fd_prime(h, f, (size_t)3 * sw);
    oc_fd_prime(hl, f, (size_t)3 * sw);
    int rc = 0;
    for (int t = 1; t < nf && rc == 0; ++t) {
        frame(f, sw, sh, t, 1);
        rc = oc_fd_step(h, f, (size_t)3 * sw, ov, cp, acc);
        int rl = oc_fd_step(hl, f, (size_t)3 * sw, ov, cp, acc);
        if (rc != rl) return 2;
    }
    dvc_fd_stats st;
    oc_fd_get_stats(h, &st);
    printf("fd %dx%d->%dx%d b%d k%d: rc %d frames %llu\n", sw, sh, W, H, block, k, rc, (unsigned long long)st.frames);
    oc_fd_destroy(h); oc_fd_destroy(hl);
    free(f); free(ov); free(cp); free(acc);
    return rc == 0 || rc == DVC_E_ODD_DCT ? 0 : 3;
}

static int run_of(int W, int H, int nf)
{
    dvc_of_params p;
    memset(&p, 0, sizeof(p));
    p.width = W; p.height = H; p.flow_threshold = 0.5f; p.quant = 100.f; p.alpha_fraction = 0.2; p.window = 4;
    p.morph_kernel = 2; p.pyr_scale = 0.3; p.levels = 2; p.winsize = 9; p.iterations = 2; p.poly_n = 5;
    p.poly_sigma = 1.1;
    oc_of* h = oc_of_create(&p);
    if (!h) return 1;
    uint8_t* f = malloc((size_t)W * H * 3);
    uint8_t *mk = malloc((size_t)W * H), *cp = malloc((size_t)W * H * 3);
    float* flow = malloc(sizeof(float) * 2 * (size_t)W * H);
    frame(f, W, H, 0, 2);
    oc_of_prime(h, f, (size_t)3 * W);
    for (int s = 0; s < 2; ++s) {
        oc_of_set_sliding(s);
        for (int t = 1; t < nf; ++t) {
            frame(f, W, H, t, 2);
            if (oc_of_step(h, f, (size_t)3 * W, mk, cp, flow)) return 4;
        }
    }
    oc_of_set_sliding(0);
    printf("of %dx%d: ok\n", W, H);
    oc_of_destroy(h);
    free(f); free(mk); free(cp); free(flow);
    return 0;
}

int main(void)
{
    int rc = 0;
    rc |= run_fd(64, 48, 64, 48, 4, 7, 0.5f, 6);
    rc |= run_fd(67, 45, 67, 45, 4, 7, 0.5f, 12);       /* odd partial blocks: stops */
    rc |= run_fd(90, 60, 45, 30, 8, 10, 0.3f, 6);        /* exact 2x area resize, even k */
    rc |= run_fd(70, 50, 91, 65, 6, 3, 0.5f, 6);         /* linear upscale, b = 6 */
    rc |= run_fd(40, 36, 40, 36, 1, 5, 0.5f, 5);
    rc |= run_fd(40, 36, 40, 36, 16, 7, 0.5f, 12);
    rc |= run_of(96, 64, 5);
    rc |= run_of(104, 72, 4);
    printf(rc ? "FAILED\n" : "sanitized run ok\n");
    return rc;
}
