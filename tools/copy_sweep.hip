// copy_sweep.hip — which streaming-copy form reaches this MI355X's HBM ceiling
// (the denominator of the FD roofline, dvc_copy_rate). Variants: 16-B vectors
// per lane per iteration (U), workgroups per CU (grid), nontemporal loads /
// stores. Prints GB/s (bytes read + written) per variant.
//   hipcc --offload-arch=gfx950 -O3 -o gpurun_ab/copy_sweep tools/copy_sweep.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f4v __attribute__((ext_vector_type(4)));

template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) k_copy(const f4v* __restrict__ src, f4v* __restrict__ dst, size_t n4)
{
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += stride) {
        f4v v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * 256;
            if (i < n4) v[u] = NTL ? __builtin_nontemporal_load(src + i) : src[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * 256;
            if (i < n4) {
                if (NTS) __builtin_nontemporal_store(v[u], dst + i);
                else dst[i] = v[u];
            }
        }
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <int U, bool NTL, bool NTS>
static void run(const f4v* a, f4v* b, size_t n4, int grid, int reps, const char* name)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_copy<U, NTL, NTS>), dim3(grid), dim3(256), 0, 0, a, b, n4);
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_copy<U, NTL, NTS>), dim3(grid), dim3(256), 0, 0, a, b, n4);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-28s grid %6d  %8.1f GB/s\n", name, grid, 2.0 * n4 * 16 * reps / (ms * 1e-3) / 1e9);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main()
{
    const size_t bytes = (size_t)2 << 30, n4 = bytes / 16;
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    f4v *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 0, bytes));
    const int grids[] = {cus * 2, cus * 4, cus * 8, cus * 16, (int)((n4 + 1023) / 1024)};
    for (int g : grids) {
        run<4, false, false>(a, b, n4, g, 10, "U4 plain/plain");
        run<4, false, true>(a, b, n4, g, 10, "U4 plain/nt");
        run<4, true, true>(a, b, n4, g, 10, "U4 nt/nt");
        run<8, false, true>(a, b, n4, g, 10, "U8 plain/nt");
        run<8, false, false>(a, b, n4, g, 10, "U8 plain/plain");
        run<2, false, true>(a, b, n4, g, 10, "U2 plain/nt");
        run<1, false, false>(a, b, n4, g, 10, "U1 plain/plain");
    }
    return 0;
}
