/* dvc_oracle.h — CPU ORACLE (test infrastructure only; see dvc_oracle.c). */
#ifndef DVC_ORACLE_H
#define DVC_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include "../include/dvc.h"

int oc_reflect101(int x, int n);
void oc_bgr2gray(const uint8_t* bgr, size_t pitch, int W, int H, uint8_t* gray);
int oc_gauss_kernel_q8(int n, double sigma, uint16_t* taps);
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

typedef struct oc_fd oc_fd;
oc_fd* oc_fd_create(const dvc_fd_params* p, int use_literal);
void oc_fd_destroy(oc_fd* h);
int oc_fd_prime(oc_fd* h, const uint8_t* bgr, size_t pitch);
int oc_fd_step(oc_fd* h, const uint8_t* bgr, size_t pitch, uint8_t* overlay, uint8_t* compressed, uint8_t* acc_out);
int oc_fd_read_plane(oc_fd* h, int plane, uint8_t* dst);
void oc_fd_get_stats(oc_fd* h, dvc_fd_stats* out);
#endif
