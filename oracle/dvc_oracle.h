/* dvc_oracle.h — CPU ORACLE (test infrastructure only; see dvc_oracle.c). */
#ifndef DVC_ORACLE_H
#define DVC_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include "../include/dvc.h"

int oc_reflect101(int x, int n);
void oc_bgr2gray(const uint8_t* bgr, size_t pitch, int W, int H, uint8_t* gray);
int oc_gauss_kernel_q8(int n, double sigma, uint16_t* taps);
void oc_gauss_kernel_f64(int n, double sigma, double* k);
void oc_gaussian_q8(const uint8_t* src, int W, int H, const uint16_t* k, int n, uint8_t* dst);
void oc_absdiff_threshold(const uint8_t* a, const uint8_t* b, size_t n, int ithresh, uint8_t* m);
int64_t oc_contour_filter(const uint8_t* mask, int W, int H, int64_t min_area2, uint8_t* filtered, uint8_t* filled);
int64_t oc_contour_filter_literal(const uint8_t* mask, int W, int H, int64_t min_area2, uint8_t* filtered);
int64_t oc_find_external_contours(const uint8_t* mask, int W, int H, int32_t** xy_out, int32_t** off_out);
int64_t oc_contour_area2(const int32_t* xy, int64_t n);
void oc_fill_contour(uint8_t* img, int W, int H, const int32_t* xy, int64_t n, uint8_t color);
void oc_free(void* p);
void oc_dilate_rect(const uint8_t* src, int W, int H, int k, int anchor, uint8_t* dst);
uint8_t oc_add_weighted_px(uint8_t a, float alpha, uint8_t b, float beta, float gamma);
void oc_bgr2ycrcb_px(const uint8_t* p, uint8_t* ycc);
void oc_ycrcb2bgr_px(const uint8_t* ycc, uint8_t* p);
void oc_dct_matrix(int B, float* M);
void oc_dct2d(const float* X, int B, const float* M, float* Y);
void oc_idct2d(const float* Y, int B, const float* M, float* X);
void oc_block_quant(const uint8_t* in, int stride, int B, const float* M, float q, uint8_t* out, int ostride);
int oc_dct_size_ok(int bh, int bw);
void oc_dct2d_rect(const float* X, int bh, int bw, const float* Mh, const float* Mw, float* Y);
void oc_idct2d_rect(const float* Y, int bh, int bw, const float* Mh, const float* Mw, float* X);
void oc_block_quant_rect(const uint8_t* in, int stride, int bh, int bw, const float* Mh, const float* Mw, float q,
                         uint8_t* out, int ostride);
int oc_resize_simd_end(int width);
void oc_resize_bgr(const uint8_t* src, size_t spitch, int sw, int sh, uint8_t* dst, size_t dpitch, int dw, int dh);

typedef struct oc_fd oc_fd;
oc_fd* oc_fd_create(const dvc_fd_params* p, int use_literal);
void oc_fd_destroy(oc_fd* h);
int oc_fd_prime(oc_fd* h, const uint8_t* bgr, size_t pitch);
int oc_fd_step(oc_fd* h, const uint8_t* bgr, size_t pitch, uint8_t* overlay, uint8_t* compressed, uint8_t* acc_out);
int oc_fd_read_plane(oc_fd* h, int plane, uint8_t* dst);
void oc_fd_get_stats(oc_fd* h, dvc_fd_stats* out);
void oc_fd_set_state(oc_fd* h, const uint8_t* prev_gray, const uint8_t* acc);

/* optical-flow path (of_oracle.c) */
void oc_blur_f32(const float* src, int W, int H, const float* k, int n, float* dst);
void oc_resize_linear_f32(const float* src, int sw, int sh, int cn, float* dst, int dw, int dh);
void oc_poly_gauss(int n, double sigma, float* g, float* xg, float* xxg, double* ig);
void oc_poly_exp(const float* src, int W, int H, int n, double sigma, float* dst);
void oc_update_matrices(const float* R0, const float* R1, const float* flow, int W, int H, float* M, int y0, int y1);
void oc_update_flow_box(const float* M, int W, int H, int bs, float* flow);
void oc_update_flow_box_sliding(const float* M, int W, int H, int bs, float* flow);
void oc_of_set_sliding(int on);
int oc_fb_levels(int W, int H, double pyr_scale, int levels);
void oc_fb_level_poly(const uint8_t* gray, int W, int H, double pyr_scale, int k, int poly_n, double poly_sigma,
                      float* R, int* lw, int* lh);
void oc_farneback(const uint8_t* prev, const uint8_t* next, int W, int H, double pyr_scale, int levels,
                  int winsize, int iterations, int poly_n, double poly_sigma, float* flow_out);
void oc_morph_close_open(const uint8_t* src, int W, int H, uint8_t* dst);
void oc_morph_close_open_k(const uint8_t* src, int W, int H, int k, uint8_t* dst);
void oc_ellipse_element(int k, uint8_t* el);
int64_t oc_rect_mask(const uint8_t* m, int W, int H, uint8_t* out);
void oc_of_compress(const uint8_t* bgr, size_t pitch, const uint8_t* mask, int W, int H, float q, uint8_t* out);
int oc_vote_threshold(double alpha, int L);
typedef struct oc_of oc_of;
oc_of* oc_of_create(const dvc_of_params* p);
void oc_of_destroy(oc_of* h);
int oc_of_prime(oc_of* h, const uint8_t* bgr, size_t pitch);
int oc_of_step(oc_of* h, const uint8_t* bgr, size_t pitch, uint8_t* mask, uint8_t* compressed, float* flow);
int oc_of_read_plane(oc_of* h, int which, uint8_t* dst);
void oc_of_set_state(oc_of* h, const uint8_t* prev_gray, const uint8_t* raw_masks, int n);

/* yuv_oracle.c: 4:2:0 YUV <-> packed BGR (cvtColor YUV2BGR_I420/NV12, BGR2YUV_I420) */
void oc_yuv420_to_bgr(const uint8_t* y, size_t ypitch, const uint8_t* u, const uint8_t* v, size_t cpitch, int cstep,
                      int W, int H, uint8_t* bgr, size_t bpitch);
void oc_bgr_to_i420(const uint8_t* bgr, size_t bpitch, int W, int H, uint8_t* y, size_t ypitch, uint8_t* u,
                    uint8_t* v, size_t cpitch);
#endif
