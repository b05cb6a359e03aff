// host_common.h — host-side helpers shared by the FD and OF C-ABI sources
// (fd_api.hip, of_api.hip). Internal.
#pragma once
#include <hip/hip_runtime.h>

#include "fd_kernels.h"

namespace dvc_host {

// Set the calling thread's dvc_last_error() text; returns `code`.
int fail(int code, const char* fmt, ...);
const char* last_error();
// getGaussianKernelBitExact values in double (n odd <= 63).
void gauss_f64(int n, double sigma, double* k);
// BxB orthonormal DCT-II basis M[k][n], float32.
void dct_matrix(int B, dvc::DctMat& M);   // M and its transpose

}  // namespace dvc_host

#define HIP_OK(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return dvc_host::fail(DVC_E_HIP, "%s failed: %s (%s:%d)", #expr,                  \
                                  hipGetErrorString(e_), __FILE__, __LINE__);                 \
    } while (0)
