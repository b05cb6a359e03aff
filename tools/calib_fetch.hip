// calib_fetch.hip — profiling harness (not part of the product): streams a
// buffer far larger than the Infinity Cache with 2-, 4-, 8-, 12- and 16-byte loads per
// lane, so rocprofv3's FETCH_SIZE can be calibrated per access width on gfx950
// (MI355X_MICROARCH.md § HBM calibrates 16-B loads only).
//   calib_fetch [MiB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

template <int WORDS>
__global__ void __launch_bounds__(256) k_read(const uint32_t* __restrict__ src, size_t nvec, uint32_t* __restrict__ out)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < nvec; i += (size_t)gridDim.x * 256) {
        const uint32_t* p = src + i * WORDS;
        if constexpr (WORDS == 0) acc += reinterpret_cast<const uint16_t*>(src)[i];
        if constexpr (WORDS == 1) acc += p[0];
        if constexpr (WORDS == 2) { const uint2 v = *reinterpret_cast<const uint2*>(p); acc += v.x ^ v.y; }
        if constexpr (WORDS == 3) { const uint3 v = *reinterpret_cast<const uint3*>(p); acc += v.x ^ v.y ^ v.z; }
        if constexpr (WORDS == 4) { const uint4 v = *reinterpret_cast<const uint4*>(p); acc += v.x ^ v.y ^ v.z ^ v.w; }
    }
    if (acc == 0x12345678u) out[0] = acc;   // keeps the loads alive; practically never stores
}

int main(int argc, char** argv)
{
    const size_t mib = argc > 1 ? std::atoll(argv[1]) : 1536;
    const size_t bytes = mib << 20;
    uint32_t *buf, *out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_read<0>, dim3(8192), dim3(256), 0, nullptr, buf, bytes / 2, out);
        hipLaunchKernelGGL(k_read<1>, dim3(8192), dim3(256), 0, nullptr, buf, bytes / 4, out);
        hipLaunchKernelGGL(k_read<2>, dim3(8192), dim3(256), 0, nullptr, buf, bytes / 8, out);
        hipLaunchKernelGGL(k_read<3>, dim3(8192), dim3(256), 0, nullptr, buf, bytes / 12, out);
        hipLaunchKernelGGL(k_read<4>, dim3(8192), dim3(256), 0, nullptr, buf, bytes / 16, out);
    }
    (void)hipDeviceSynchronize();
    std::printf("streamed %zu MiB per kernel (2/4/8/12/16-B loads); expected FETCH bytes per launch: %zu\n", mib, bytes);
    return 0;
}
