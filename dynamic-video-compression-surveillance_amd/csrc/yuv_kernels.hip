// yuv_kernels.hip — video I/O colour conversions on the GPU.
//
// A decoder (VCN through rocDecode, or a Y4M reader) hands over 4:2:0 YUV
// surfaces; the reference's loop works on the packed BGR frames
// cv2.VideoCapture.read() returns (frame_differencing.py:87,
// motion_compression_opt.py:66,145), and an encoder takes 4:2:0 again
// (cv2.VideoWriter.write, fd:112,131). These kernels are OpenCV 4.11's
// cvtColor COLOR_YUV2BGR_I420 / COLOR_YUV2BGR_NV12 and COLOR_BGR2YUV_I420
// (color_yuv.simd.hpp: ITU-R BT.601 limited range, 20-bit fixed point; the
// 4:2:0 encode takes the chroma of each 2x2 quad from its top-left pixel),
// bit-exact against oracle/yuv_oracle.c. Integer work, HBM-bound: one lane per
// 4 px x 2 rows (two chroma samples), dword loads and stores where the layout
// allows (ALIGNED), byte accesses otherwise.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "../../include/dvc.h"
#include "host_common.h"
#include "yuv_kernels.h"
#include "yuv_px.h"

namespace dvc {

namespace {

using namespace yuvpx;

template <bool ALIGNED>
__global__ void __launch_bounds__(256) k_yuv420_to_bgr(YuvLayout s, int W, int H, uint8_t* __restrict__ dst,
                                                       size_t dpitch, size_t dstride)
{
    const int q = blockIdx.x * 256 + threadIdx.x, x = 4 * q;   // px x .. x+3 (W even: x+2 may be the last pair)
    const int r = 2 * blockIdx.y, t = blockIdx.z;
    if (x >= W) return;
    const uint8_t* f = s.base + (size_t)t * s.fstride;
    const uint8_t* cu = f + s.uoff + (size_t)blockIdx.y * s.cpitch + (size_t)(x / 2) * s.cstep;
    const uint8_t* cvp = f + s.voff + (size_t)blockIdx.y * s.cpitch + (size_t)(x / 2) * s.cstep;
    const bool two = x + 4 > W;   // only px x, x+1 exist
    const int u0 = cu[0], v0 = cvp[0];
    const int u1 = two ? u0 : cu[s.cstep], v1 = two ? v0 : cvp[s.cstep];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const uint8_t* yr = f + (size_t)(r + i) * s.ypitch + x;
        uint8_t* o = dst + (size_t)t * dstride + (size_t)(r + i) * dpitch + 3 * (size_t)x;
        uint32_t y4;
        if (ALIGNED && !two) y4 = *reinterpret_cast<const uint32_t*>(yr);
        else y4 = (uint32_t)yr[0] | ((uint32_t)yr[1] << 8) | (two ? 0u : ((uint32_t)yr[2] << 16) | ((uint32_t)yr[3] << 24));
        uint32_t w[3];
        yuv4_bgr(y4, u0, v0, u1, v1, w);
        if (ALIGNED && !two) {
            uint32_t* o4 = reinterpret_cast<uint32_t*>(o);
            o4[0] = w[0];
            o4[1] = w[1];
            o4[2] = w[2];
        } else {
            for (int k = 0; k < (two ? 6 : 12); ++k) o[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
        }
    }
}

__global__ void __launch_bounds__(256) k_bgr_to_i420(const uint8_t* __restrict__ src, size_t spitch, size_t sstride,
                                                     int W, int H, YuvLayout d)
{
    const int q = blockIdx.x * 256 + threadIdx.x, x = 4 * q;
    const int r = 2 * blockIdx.y, t = blockIdx.z;
    if (x >= W) return;
    const int np = min(4, W - x);   // 4 or 2 px
    uint8_t* f = const_cast<uint8_t*>(d.base) + (size_t)t * d.fstride;
    int us[2] = {0, 0}, vs[2] = {0, 0};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const uint8_t* s = src + (size_t)t * sstride + (size_t)(r + i) * spitch + 3 * (size_t)x;
        uint8_t* yr = f + (size_t)(r + i) * d.ypitch + x;
        for (int j = 0; j < np; ++j) {
            const int b = s[3 * j], g = s[3 * j + 1], rr = s[3 * j + 2];
            yr[j] = (uint8_t)luma(b, g, rr);
            if (i == 0 && !(j & 1)) {
                us[j >> 1] = (int)chroma_u(b, g, rr);
                vs[j >> 1] = (int)chroma_v(b, g, rr);
            }
        }
    }
    uint8_t* u = f + d.uoff + (size_t)blockIdx.y * d.cpitch + (size_t)(x / 2) * d.cstep;
    uint8_t* v = f + d.voff + (size_t)blockIdx.y * d.cpitch + (size_t)(x / 2) * d.cstep;
    for (int j = 0; j < np / 2; ++j) {
        u[j * d.cstep] = (uint8_t)us[j];
        v[j * d.cstep] = (uint8_t)vs[j];
    }
}

}  // namespace

hipError_t launch_yuv420_to_bgr(const YuvLayout& s, int W, int H, int n, uint8_t* dst, size_t dpitch, size_t dstride,
                                hipStream_t st)
{
    const dim3 grid((unsigned)((W / 4 + 1 + 255) / 256), (unsigned)(H / 2), (unsigned)n);
    const bool al = ((uintptr_t)s.base % 4) == 0 && s.ypitch % 4 == 0 && (n <= 1 || s.fstride % 4 == 0) &&
                    ((uintptr_t)dst % 4) == 0 && dpitch % 4 == 0 && (n <= 1 || dstride % 4 == 0);
    if (al) hipLaunchKernelGGL(k_yuv420_to_bgr<true>, grid, dim3(256), 0, st, s, W, H, dst, dpitch, dstride);
    else hipLaunchKernelGGL(k_yuv420_to_bgr<false>, grid, dim3(256), 0, st, s, W, H, dst, dpitch, dstride);
    return hipGetLastError();
}

hipError_t launch_bgr_to_i420(const uint8_t* src, size_t spitch, size_t sstride, int W, int H, int n,
                              const YuvLayout& d, hipStream_t st)
{
    const dim3 grid((unsigned)((W / 4 + 1 + 255) / 256), (unsigned)(H / 2), (unsigned)n);
    hipLaunchKernelGGL(k_bgr_to_i420, grid, dim3(256), 0, st, src, spitch, sstride, W, H, d);
    return hipGetLastError();
}

// Layout of a DVC_FMT_I420 / DVC_FMT_NV12 frame (include/dvc.h): luma rows of
// `pitch`, chroma plane(s) after `crows` luma rows.
YuvLayout yuv_layout(const uint8_t* base, size_t pitch, int fmt, int crows, size_t fstride)
{
    YuvLayout L{};
    L.base = base;
    L.ypitch = pitch;
    L.fstride = fstride;
    L.uoff = pitch * (size_t)crows;
    if (fmt == DVC_FMT_NV12) {
        L.voff = L.uoff + 1;
        L.cpitch = pitch;
        L.cstep = 2;
    } else {
        L.cpitch = pitch / 2;
        L.voff = L.uoff + L.cpitch * (size_t)(crows / 2);
        L.cstep = 1;
    }
    return L;
}

size_t yuv_frame_bytes(size_t pitch, int crows) { return pitch * (size_t)crows * 3 / 2; }

}  // namespace dvc

using dvc_host::fail;

namespace {

int check_yuv_args(int fmt, int crows, int W, int H, size_t pitch, int n, size_t fstride)
{
    if (fmt != DVC_FMT_I420 && fmt != DVC_FMT_NV12) return fail(DVC_E_INVALID, "unknown YUV format %d", fmt);
    if (W < 2 || H < 2 || (W & 1) || (H & 1)) return fail(DVC_E_INVALID, "4:2:0 frame %dx%d: sides must be even", W, H);
    const int cr = crows ? crows : H;
    if (cr < H || (cr & 1)) return fail(DVC_E_INVALID, "chroma_rows %d: even and >= height %d", crows, H);
    if (pitch < (size_t)W || (fmt == DVC_FMT_I420 && (pitch & 1))) return fail(DVC_E_INVALID, "pitch %zu invalid", pitch);
    if (n < 0) return fail(DVC_E_INVALID, "negative frame count");
    if (n > 1 && fstride < dvc::yuv_frame_bytes(pitch, cr)) return fail(DVC_E_INVALID, "frame stride %zu invalid", fstride);
    return DVC_OK;
}

// Device scratch of the host-pointer conversions (a Y4M reader / writer thread
// calls them once per frame): kept across calls instead of hipMalloc/hipFree
// per call — hipFree synchronises the whole device, which would stall every
// worker's pipelined streams. A call takes an entry of its device (or makes
// one), grows it when a frame is larger, and gives it back; entries live until
// the process ends. Each entry has its own non-blocking stream for callers
// that pass none (the legacy default stream would serialise with the rest).
struct Scratch {
    int device = 0;
    uint8_t *a = nullptr, *b = nullptr;
    size_t na = 0, nb = 0;
    hipStream_t stream = nullptr;
};

std::mutex g_scratch_mu;
std::vector<Scratch*> g_scratch_free;

Scratch* scratch_take(int device)
{
    {
        std::lock_guard<std::mutex> lk(g_scratch_mu);
        for (size_t i = 0; i < g_scratch_free.size(); ++i)
            if (g_scratch_free[i]->device == device) {
                Scratch* s = g_scratch_free[i];
                g_scratch_free.erase(g_scratch_free.begin() + (long)i);
                return s;
            }
    }
    Scratch* s = new Scratch();
    s->device = device;
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
        delete s;
        return nullptr;
    }
    return s;
}

void scratch_give(Scratch* s)
{
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    g_scratch_free.push_back(s);
}

hipError_t scratch_fit(uint8_t** p, size_t* have, size_t need)
{
    if (*have >= need) return hipSuccess;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    hipError_t e = hipMalloc(p, need);
    if (e == hipSuccess) *have = need;
    return e;
}

}  // namespace

extern "C" {

int dvc_yuv420_to_bgr(const uint8_t* yuv, size_t pitch, int fmt, int chroma_rows, int width, int height, int n,
                      size_t frame_stride, uint8_t* bgr, size_t bgr_pitch, size_t bgr_stride, int device,
                      void* hip_stream, uint32_t flags)
{
    if (!yuv || !bgr) return fail(DVC_E_INVALID, "NULL argument");
    int rc = check_yuv_args(fmt, chroma_rows, width, height, pitch, n, frame_stride);
    if (rc) return rc;
    if (bgr_pitch < 3 * (size_t)width || (n > 1 && bgr_stride < bgr_pitch * (height - 1) + 3 * (size_t)width))
        return fail(DVC_E_INVALID, "BGR pitch %zu / stride %zu invalid", bgr_pitch, bgr_stride);
    if (n == 0) return DVC_OK;
    const int cr = chroma_rows ? chroma_rows : height;
    HIP_OK(hipSetDevice(device));
    hipStream_t st = (hipStream_t)hip_stream;
    if (flags & DVC_FLAG_DEVICE_PTRS) {
        HIP_OK(dvc::launch_yuv420_to_bgr(dvc::yuv_layout(yuv, pitch, fmt, cr, frame_stride), width, height, n, bgr,
                                         bgr_pitch, bgr_stride, st));
        return DVC_OK;
    }
    // host pointers: one frame at a time through the device scratch, synchronous
    const size_t fb = dvc::yuv_frame_bytes(pitch, cr), ob = 3 * (size_t)width * height;
    Scratch* sc = scratch_take(device);
    if (!sc) return fail(DVC_E_HIP, "yuv420 -> bgr: no stream");
    if (!st) st = sc->stream;
    hipError_t e = scratch_fit(&sc->a, &sc->na, fb);
    if (e == hipSuccess) e = scratch_fit(&sc->b, &sc->nb, ob);
    uint8_t *din = sc->a, *dout = sc->b;
    for (int t = 0; t < n && e == hipSuccess; ++t) {
        e = hipMemcpyAsync(din, yuv + (size_t)t * frame_stride, fb, hipMemcpyHostToDevice, st);
        if (e == hipSuccess)
            e = dvc::launch_yuv420_to_bgr(dvc::yuv_layout(din, pitch, fmt, cr, fb), width, height, 1, dout, 3 * width,
                                          ob, st);
        if (e == hipSuccess)
            e = hipMemcpy2DAsync(bgr + (size_t)t * bgr_stride, bgr_pitch, dout, 3 * (size_t)width, 3 * (size_t)width,
                                 height, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
    }
    scratch_give(sc);
    if (e != hipSuccess) return fail(DVC_E_HIP, "yuv420 -> bgr: %s", hipGetErrorString(e));
    return DVC_OK;
}

int dvc_bgr_to_i420(const uint8_t* bgr, size_t bgr_pitch, size_t bgr_stride, int width, int height, int n,
                    uint8_t* yuv, size_t pitch, int chroma_rows, size_t frame_stride, int device, void* hip_stream,
                    uint32_t flags)
{
    if (!yuv || !bgr) return fail(DVC_E_INVALID, "NULL argument");
    int rc = check_yuv_args(DVC_FMT_I420, chroma_rows, width, height, pitch, n, frame_stride);
    if (rc) return rc;
    if (bgr_pitch < 3 * (size_t)width || (n > 1 && bgr_stride < bgr_pitch * (height - 1) + 3 * (size_t)width))
        return fail(DVC_E_INVALID, "BGR pitch %zu / stride %zu invalid", bgr_pitch, bgr_stride);
    if (n == 0) return DVC_OK;
    const int cr = chroma_rows ? chroma_rows : height;
    HIP_OK(hipSetDevice(device));
    hipStream_t st = (hipStream_t)hip_stream;
    if (flags & DVC_FLAG_DEVICE_PTRS) {
        HIP_OK(dvc::launch_bgr_to_i420(bgr, bgr_pitch, bgr_stride, width, height, n,
                                       dvc::yuv_layout(yuv, pitch, DVC_FMT_I420, cr, frame_stride), st));
        return DVC_OK;
    }
    const size_t fb = dvc::yuv_frame_bytes(pitch, cr), ib = 3 * (size_t)width * height;
    Scratch* sc = scratch_take(device);
    if (!sc) return fail(DVC_E_HIP, "bgr -> i420: no stream");
    if (!st) st = sc->stream;
    hipError_t e = scratch_fit(&sc->a, &sc->na, ib);
    if (e == hipSuccess) e = scratch_fit(&sc->b, &sc->nb, fb);
    uint8_t *din = sc->a, *dout = sc->b;
    for (int t = 0; t < n && e == hipSuccess; ++t) {
        e = hipMemcpy2DAsync(din, 3 * (size_t)width, bgr + (size_t)t * bgr_stride, bgr_pitch, 3 * (size_t)width,
                             height, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(dout, yuv + (size_t)t * frame_stride, fb, hipMemcpyHostToDevice, st);
        if (e == hipSuccess)
            e = dvc::launch_bgr_to_i420(din, 3 * (size_t)width, ib, width, height, 1,
                                        dvc::yuv_layout(dout, pitch, DVC_FMT_I420, cr, fb), st);
        if (e == hipSuccess) e = hipMemcpyAsync(yuv + (size_t)t * frame_stride, dout, fb, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
    }
    scratch_give(sc);
    if (e != hipSuccess) return fail(DVC_E_HIP, "bgr -> i420: %s", hipGetErrorString(e));
    return DVC_OK;
}

}  // extern "C"
