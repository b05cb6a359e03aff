// diag.hip — measurement helpers of the C-ABI (include/dvc.h, "diagnostics").
//
// dvc_copy_rate: this device's practical streaming ceiling, the denominator
// SURVEY.md §8d asks the FD roofline to be quoted against beside the 8 TB/s
// spec. A hand-written copy in the form MI355X_MICROARCH.md measures its
// 6.29 TB/s with (16 B per lane, coalesced, 4 vectors per lane in flight, one
// workgroup per 16 KiB: tools/copy_sweep.hip measured it the fastest of the
// unroll x grid x cache-policy forms on this pool's MI355X, 5.5-5.7 TB/s),
// optionally with nontemporal loads and stores (what FD's streaming stages
// use), over a buffer far beyond the 256 MB Infinity Cache; bytes read +
// written / event time.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/dvc.h"
#include "host_common.h"

using dvc_host::fail;

namespace {

constexpr int COPY_U = 4;   // 16-B vectors per lane per iteration (all loads before the stores)
typedef float f4v __attribute__((ext_vector_type(4)));

// one pass over the buffer (a workgroup per 256 x COPY_U 16-B vectors, no
// grid stride): the fastest form of tools/copy_sweep.hip on MI355X
template <bool NT>
__global__ void __launch_bounds__(256) k_copy(const f4v* __restrict__ src, f4v* __restrict__ dst, size_t n4)
{
    const size_t stride = (size_t)gridDim.x * 256 * COPY_U;
    for (size_t base = (size_t)blockIdx.x * 256 * COPY_U + threadIdx.x; base < n4; base += stride) {
        f4v v[COPY_U];
#pragma unroll
        for (int u = 0; u < COPY_U; ++u) {
            const size_t i = base + (size_t)u * 256;
            if (i < n4) v[u] = NT ? __builtin_nontemporal_load(src + i) : src[i];
        }
#pragma unroll
        for (int u = 0; u < COPY_U; ++u) {
            const size_t i = base + (size_t)u * 256;
            if (i < n4) {
                if (NT) __builtin_nontemporal_store(v[u], dst + i);
                else dst[i] = v[u];
            }
        }
    }
}

}  // namespace

extern "C" {

int dvc_copy_rate(int device, size_t bytes, int reps, int nontemporal, double* gbps)
{
    if (!gbps || reps < 1 || bytes < 4096) return fail(DVC_E_INVALID, "bytes >= 4096, reps >= 1, gbps non-NULL");
    HIP_OK(hipSetDevice(device));
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    const size_t n4 = bytes / 16;
    f4v *a = nullptr, *b = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipError_t e = hipMalloc(&a, n4 * 16);
    if (e == hipSuccess) e = hipMalloc(&b, n4 * 16);
    if (e == hipSuccess) e = hipMemset(a, 1, n4 * 16);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    float ms = 0.f;
    if (e == hipSuccess) {
        const size_t per_wg = (size_t)256 * COPY_U;
        const unsigned grid = (unsigned)((n4 + per_wg - 1) / per_wg);
        (void)cus;
        auto launch = [&]() {
            if (nontemporal) hipLaunchKernelGGL(k_copy<true>, dim3(grid), dim3(256), 0, s, a, b, n4);
            else hipLaunchKernelGGL(k_copy<false>, dim3(grid), dim3(256), 0, s, a, b, n4);
        };
        launch();   // warm-up
        e = hipEventRecord(e0, s);
        for (int r = 0; r < reps && e == hipSuccess; ++r) {
            launch();
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipEventRecord(e1, s);
        if (e == hipSuccess) e = hipEventSynchronize(e1);
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    }
    for (hipEvent_t ev : {e0, e1})
        if (ev) (void)hipEventDestroy(ev);
    if (s) (void)hipStreamDestroy(s);
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    if (e != hipSuccess) return fail(e == hipErrorOutOfMemory ? DVC_E_NOMEM : DVC_E_HIP, "copy rate: %s",
                                     hipGetErrorString(e));
    *gbps = 2.0 * (double)n4 * 16 * reps / (ms * 1e-3) / 1e9;
    return DVC_OK;
}

}  // extern "C"
