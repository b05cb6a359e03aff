/*
 * yuv_oracle.c — CPU oracle (TEST INFRASTRUCTURE ONLY) for the video-I/O
 * colour conversions between 4:2:0 YUV decoder/encoder surfaces and the packed
 * BGR frames the reference's loop works on.
 *
 * The reference gets BGR from cv2.VideoCapture.read() (frame_differencing.py:87,
 * motion_compression_opt.py:66,145) and hands BGR to cv2.VideoWriter.write()
 * (fd:112,131; of:99-100,185). A decoder (VCN/rocDecode, or a Y4M file) yields
 * 4:2:0 YUV and an encoder takes it; the conversions restated here are
 * OpenCV 4.11's cvtColor COLOR_YUV2BGR_I420 / COLOR_YUV2BGR_NV12 and
 * COLOR_BGR2YUV_I420 (modules/imgproc/src/color_yuv.simd.hpp: the ITU-R BT.601
 * fixed-point coefficients with a 20-bit shift, limited range; chroma of the
 * 4:2:0 encode sampled from the top-left pixel of each 2x2 quad). cv2 is not
 * importable here, so these restatements are parity-UNPINNED against OpenCV
 * itself: the GPU kernels are bit-exact against them.
 */
#include <stddef.h>
#include <stdint.h>

#include "dvc_oracle.h"

enum {
    BT601_CY = 1220542, BT601_CUB = 2116026, BT601_CUG = -409993, BT601_CVG = -852492, BT601_CVR = 1673527,
    BT601_CRY = 269484, BT601_CGY = 528482, BT601_CBY = 102760,
    BT601_CRU = -155188, BT601_CGU = -305135, BT601_CBU = 460324,
    BT601_CGV = -385875, BT601_CBV = -74448,
    BT601_SHIFT = 20,
};

static uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

/* One 4:2:0 frame -> packed BGR. Chroma sample (i, j) serves luma (2i..2i+1,
 * 2j..2j+1); u and v point at the U and V samples of chroma row 0 with `cstep`
 * bytes between horizontally adjacent samples (1: I420 planes, 2: NV12's
 * interleaved plane) and `cpitch` bytes between chroma rows. W, H even. */
void oc_yuv420_to_bgr(const uint8_t* y, size_t ypitch, const uint8_t* u, const uint8_t* v, size_t cpitch, int cstep,
                      int W, int H, uint8_t* bgr, size_t bpitch)
{
    for (int r = 0; r < H; ++r) {
        const uint8_t* yr = y + (size_t)r * ypitch;
        const uint8_t* ur = u + (size_t)(r / 2) * cpitch;
        const uint8_t* vr = v + (size_t)(r / 2) * cpitch;
        uint8_t* o = bgr + (size_t)r * bpitch;
        for (int x = 0; x < W; ++x) {
            const int cu = (int)ur[(x / 2) * cstep] - 128, cv = (int)vr[(x / 2) * cstep] - 128;
            const int ruv = (1 << (BT601_SHIFT - 1)) + BT601_CVR * cv;
            const int guv = (1 << (BT601_SHIFT - 1)) + BT601_CVG * cv + BT601_CUG * cu;
            const int buv = (1 << (BT601_SHIFT - 1)) + BT601_CUB * cu;
            const int yy = (yr[x] > 16 ? (int)yr[x] - 16 : 0) * BT601_CY;
            o[3 * x + 0] = sat_u8((yy + buv) >> BT601_SHIFT);
            o[3 * x + 1] = sat_u8((yy + guv) >> BT601_SHIFT);
            o[3 * x + 2] = sat_u8((yy + ruv) >> BT601_SHIFT);
        }
    }
}

/* Packed BGR -> I420 planes (Y: H rows of ypitch; U, V: H/2 rows of cpitch).
 * W, H even. */
void oc_bgr_to_i420(const uint8_t* bgr, size_t bpitch, int W, int H, uint8_t* y, size_t ypitch, uint8_t* u,
                    uint8_t* v, size_t cpitch)
{
    const int half = 1 << (BT601_SHIFT - 1);
    for (int r = 0; r < H; ++r) {
        const uint8_t* s = bgr + (size_t)r * bpitch;
        uint8_t* yr = y + (size_t)r * ypitch;
        for (int x = 0; x < W; ++x) {
            const int b = s[3 * x], g = s[3 * x + 1], rr = s[3 * x + 2];
            yr[x] = sat_u8((BT601_CRY * rr + BT601_CGY * g + BT601_CBY * b + half + (16 << BT601_SHIFT)) >> BT601_SHIFT);
            if (!(r & 1) && !(x & 1)) {
                const int uu = BT601_CRU * rr + BT601_CGU * g + BT601_CBU * b + half + (128 << BT601_SHIFT);
                const int vv = BT601_CBU * rr + BT601_CGV * g + BT601_CBV * b + half + (128 << BT601_SHIFT);
                u[(size_t)(r / 2) * cpitch + x / 2] = sat_u8(uu >> BT601_SHIFT);
                v[(size_t)(r / 2) * cpitch + x / 2] = sat_u8(vv >> BT601_SHIFT);
            }
        }
    }
}
