// yuv_kernels.h — 4:2:0 YUV <-> packed BGR conversion kernels (video I/O,
// SURVEY.md §8f #1). Internal launch interface; the C-ABI is in include/dvc.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dvc {

// A batch of 4:2:0 frames: frame t's luma rows at base + t*fstride (ypitch
// bytes each), its chroma row r's U / V samples at base + t*fstride + uoff /
// voff + r*cpitch, cstep bytes apart (1: I420 planes, 2: NV12's UV plane).
struct YuvLayout {
    const uint8_t* base;
    size_t ypitch, uoff, voff, cpitch, fstride;
    int cstep;
};

// cvtColor COLOR_YUV2BGR_I420 / _NV12 of n W x H frames (W, H even) into
// packed BGR rows of dpitch bytes, frames dstride apart.
hipError_t launch_yuv420_to_bgr(const YuvLayout& s, int W, int H, int n, uint8_t* dst, size_t dpitch, size_t dstride,
                                hipStream_t st);

// cvtColor COLOR_BGR2YUV_I420 of n W x H packed BGR frames (rows of spitch,
// frames sstride apart) into I420 frames laid out as `d` (cstep 1).
hipError_t launch_bgr_to_i420(const uint8_t* src, size_t spitch, size_t sstride, int W, int H, int n,
                              const YuvLayout& d, hipStream_t st);

// The YuvLayout of a DVC_FMT_I420 / DVC_FMT_NV12 frame (include/dvc.h): luma
// rows of `pitch` bytes, the chroma plane(s) after `crows` luma rows.
YuvLayout yuv_layout(const uint8_t* base, size_t pitch, int fmt, int crows, size_t fstride);
// Bytes one such frame spans: pitch * crows * 3 / 2.
size_t yuv_frame_bytes(size_t pitch, int crows);

}  // namespace dvc
