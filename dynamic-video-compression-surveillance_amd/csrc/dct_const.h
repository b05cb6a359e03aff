// dct_const.h — the DCT bases of the fast block sizes as compile-time
// constants (internal; not part of include/dvc.h). Kernels that take their
// factors from these instead of kernel arguments keep 32 (4x4) or 128 (8x8)
// SGPRs free; each launcher checks the host-built basis against the table
// first and refuses a mismatch, so the constants can never silently differ.
#pragma once
#include <hip/hip_runtime.h>
#include <cstring>

#include "fd_kernels.h"

namespace dvc {

// The 4x4 DCT basis as dct_matrix(4) builds it on the host (fd_api.hip:
// (float)(c * cos(pi (2n+1) k / 8))), as compile-time constants: the fused
// front's DCT then takes its factors as literals / inline constants instead
// of 32 kernel-argument SGPRs. launch_front checks FrontOut::M against it
// bit for bit and refuses the fused form otherwise (dct4_is_const).
#define DVC_A4 0x1.4e7aeap-1f
#define DVC_B4 0x1.1517a8p-2f
__device__ constexpr DctMat kDct4 = {
    {0.5f, 0.5f, 0.5f, 0.5f, DVC_A4, DVC_B4, -DVC_B4, -DVC_A4, 0.5f, -0.5f, -0.5f, 0.5f, DVC_B4, -DVC_A4, DVC_A4, -DVC_B4},
    {0.5f, DVC_A4, 0.5f, DVC_B4, 0.5f, DVC_B4, -0.5f, -DVC_A4, 0.5f, -DVC_B4, -0.5f, DVC_A4, 0.5f, -DVC_A4, 0.5f, -DVC_B4}};
constexpr float kDct4Host[32] = {
    0.5f, 0.5f, 0.5f, 0.5f, DVC_A4, DVC_B4, -DVC_B4, -DVC_A4, 0.5f, -0.5f, -0.5f, 0.5f, DVC_B4, -DVC_A4, DVC_A4, -DVC_B4,
    0.5f, DVC_A4, 0.5f, DVC_B4, 0.5f, DVC_B4, -0.5f, -DVC_A4, 0.5f, -DVC_B4, -0.5f, DVC_A4, 0.5f, -DVC_A4, 0.5f, -DVC_B4};
#undef DVC_A4
#undef DVC_B4

inline bool dct4_is_const(const DctMat& M)
{
    return std::memcmp(M.m, kDct4Host, 16 * sizeof(float)) == 0 &&
           std::memcmp(M.mt, kDct4Host + 16, 16 * sizeof(float)) == 0;
}


// The 8x8 DCT basis as dct_matrix(8) builds it on the host (fd_api.hip:
// (float)(c * cos(pi (2n+1) k / 16))), as compile-time constants: k_of_out's and
// k_out<8>'s DCT passes take their factors as literals instead of 128 kernel-argument
// SGPRs (which spilled). of_launch_out / launch_out check the basis they are given bit for bit.
__device__ constexpr DctMat kDct8 = {
    {0x1.6a09e6p-2f, 0x1.6a09e6p-2f, 0x1.6a09e6p-2f, 0x1.6a09e6p-2f, 0x1.6a09e6p-2f, 0x1.6a09e6p-2f, 0x1.6a09e6p-2f, 0x1.6a09e6p-2f,
    0x1.f6297cp-2f, 0x1.a9b662p-2f, 0x1.1c73b4p-2f, 0x1.8f8b84p-4f, -0x1.8f8b84p-4f, -0x1.1c73b4p-2f, -0x1.a9b662p-2f, -0x1.f6297cp-2f,
    0x1.d906bcp-2f, 0x1.87de2ap-3f, -0x1.87de2ap-3f, -0x1.d906bcp-2f, -0x1.d906bcp-2f, -0x1.87de2ap-3f, 0x1.87de2ap-3f, 0x1.d906bcp-2f,
    0x1.a9b662p-2f, -0x1.8f8b84p-4f, -0x1.f6297cp-2f, -0x1.1c73b4p-2f, 0x1.1c73b4p-2f, 0x1.f6297cp-2f, 0x1.8f8b84p-4f, -0x1.a9b662p-2f,
    0x1.6a09e6p-2f, -0x1.6a09e6p-2f, -0x1.6a09e6p-2f, 0x1.6a09e6p-2f, 0x1.6a09e6p-2f, -0x1.6a09e6p-2f, -0x1.6a09e6p-2f, 0x1.6a09e6p-2f,
    0x1.1c73b4p-2f, -0x1.f6297cp-2f, 0x1.8f8b84p-4f, 0x1.a9b662p-2f, -0x1.a9b662p-2f, -0x1.8f8b84p-4f, 0x1.f6297cp-2f, -0x1.1c73b4p-2f,
    0x1.87de2ap-3f, -0x1.d906bcp-2f, 0x1.d906bcp-2f, -0x1.87de2ap-3f, -0x1.87de2ap-3f, 0x1.d906bcp-2f, -0x1.d906bcp-2f, 0x1.87de2ap-3f,
    0x1.8f8b84p-4f, -0x1.1c73b4p-2f, 0x1.a9b662p-2f, -0x1.f6297cp-2f, 0x1.f6297cp-2f, -0x1.a9b662p-2f, 0x1.1c73b4p-2f, -0x1.8f8b84p-4f},
    {0x1.6a09e6p-2f, 0x1.f6297cp-2f, 0x1.d906bcp-2f, 0x1.a9b662p-2f, 0x1.6a09e6p-2f, 0x1.1c73b4p-2f, 0x1.87de2ap-3f, 0x1.8f8b84p-4f,
    0x1.6a09e6p-2f, 0x1.a9b662p-2f, 0x1.87de2ap-3f, -0x1.8f8b84p-4f, -0x1.6a09e6p-2f, -0x1.f6297cp-2f, -0x1.d906bcp-2f, -0x1.1c73b4p-2f,
    0x1.6a09e6p-2f, 0x1.1c73b4p-2f, -0x1.87de2ap-3f, -0x1.f6297cp-2f, -0x1.6a09e6p-2f, 0x1.8f8b84p-4f, 0x1.d906bcp-2f, 0x1.a9b662p-2f,
    0x1.6a09e6p-2f, 0x1.8f8b84p-4f, -0x1.d906bcp-2f, -0x1.1c73b4p-2f, 0x1.6a09e6p-2f, 0x1.a9b662p-2f, -0x1.87de2ap-3f, -0x1.f6297cp-2f,
    0x1.6a09e6p-2f, -0x1.8f8b84p-4f, -0x1.d906bcp-2f, 0x1.1c73b4p-2f, 0x1.6a09e6p-2f, -0x1.a9b662p-2f, -0x1.87de2ap-3f, 0x1.f6297cp-2f,
    0x1.6a09e6p-2f, -0x1.1c73b4p-2f, -0x1.87de2ap-3f, 0x1.f6297cp-2f, -0x1.6a09e6p-2f, -0x1.8f8b84p-4f, 0x1.d906bcp-2f, -0x1.a9b662p-2f,
    0x1.6a09e6p-2f, -0x1.a9b662p-2f, 0x1.87de2ap-3f, 0x1.8f8b84p-4f, -0x1.6a09e6p-2f, 0x1.f6297cp-2f, -0x1.d906bcp-2f, 0x1.1c73b4p-2f,
    0x1.6a09e6p-2f, -0x1.f6297cp-2f, 0x1.d906bcp-2f, -0x1.a9b662p-2f, 0x1.6a09e6p-2f, -0x1.1c73b4p-2f, 0x1.87de2ap-3f, -0x1.8f8b84p-4f}};
constexpr float kDct8Host[128] = {
    0x1.6a09e6p-2f, 0x1.6a09e6p-2f, 0x1.6a09e6p-2f, 0x1.6a09e6p-2f, 0x1.6a09e6p-2f, 0x1.6a09e6p-2f, 0x1.6a09e6p-2f, 0x1.6a09e6p-2f,
    0x1.f6297cp-2f, 0x1.a9b662p-2f, 0x1.1c73b4p-2f, 0x1.8f8b84p-4f, -0x1.8f8b84p-4f, -0x1.1c73b4p-2f, -0x1.a9b662p-2f, -0x1.f6297cp-2f,
    0x1.d906bcp-2f, 0x1.87de2ap-3f, -0x1.87de2ap-3f, -0x1.d906bcp-2f, -0x1.d906bcp-2f, -0x1.87de2ap-3f, 0x1.87de2ap-3f, 0x1.d906bcp-2f,
    0x1.a9b662p-2f, -0x1.8f8b84p-4f, -0x1.f6297cp-2f, -0x1.1c73b4p-2f, 0x1.1c73b4p-2f, 0x1.f6297cp-2f, 0x1.8f8b84p-4f, -0x1.a9b662p-2f,
    0x1.6a09e6p-2f, -0x1.6a09e6p-2f, -0x1.6a09e6p-2f, 0x1.6a09e6p-2f, 0x1.6a09e6p-2f, -0x1.6a09e6p-2f, -0x1.6a09e6p-2f, 0x1.6a09e6p-2f,
    0x1.1c73b4p-2f, -0x1.f6297cp-2f, 0x1.8f8b84p-4f, 0x1.a9b662p-2f, -0x1.a9b662p-2f, -0x1.8f8b84p-4f, 0x1.f6297cp-2f, -0x1.1c73b4p-2f,
    0x1.87de2ap-3f, -0x1.d906bcp-2f, 0x1.d906bcp-2f, -0x1.87de2ap-3f, -0x1.87de2ap-3f, 0x1.d906bcp-2f, -0x1.d906bcp-2f, 0x1.87de2ap-3f,
    0x1.8f8b84p-4f, -0x1.1c73b4p-2f, 0x1.a9b662p-2f, -0x1.f6297cp-2f, 0x1.f6297cp-2f, -0x1.a9b662p-2f, 0x1.1c73b4p-2f, -0x1.8f8b84p-4f,
    0x1.6a09e6p-2f, 0x1.f6297cp-2f, 0x1.d906bcp-2f, 0x1.a9b662p-2f, 0x1.6a09e6p-2f, 0x1.1c73b4p-2f, 0x1.87de2ap-3f, 0x1.8f8b84p-4f,
    0x1.6a09e6p-2f, 0x1.a9b662p-2f, 0x1.87de2ap-3f, -0x1.8f8b84p-4f, -0x1.6a09e6p-2f, -0x1.f6297cp-2f, -0x1.d906bcp-2f, -0x1.1c73b4p-2f,
    0x1.6a09e6p-2f, 0x1.1c73b4p-2f, -0x1.87de2ap-3f, -0x1.f6297cp-2f, -0x1.6a09e6p-2f, 0x1.8f8b84p-4f, 0x1.d906bcp-2f, 0x1.a9b662p-2f,
    0x1.6a09e6p-2f, 0x1.8f8b84p-4f, -0x1.d906bcp-2f, -0x1.1c73b4p-2f, 0x1.6a09e6p-2f, 0x1.a9b662p-2f, -0x1.87de2ap-3f, -0x1.f6297cp-2f,
    0x1.6a09e6p-2f, -0x1.8f8b84p-4f, -0x1.d906bcp-2f, 0x1.1c73b4p-2f, 0x1.6a09e6p-2f, -0x1.a9b662p-2f, -0x1.87de2ap-3f, 0x1.f6297cp-2f,
    0x1.6a09e6p-2f, -0x1.1c73b4p-2f, -0x1.87de2ap-3f, 0x1.f6297cp-2f, -0x1.6a09e6p-2f, -0x1.8f8b84p-4f, 0x1.d906bcp-2f, -0x1.a9b662p-2f,
    0x1.6a09e6p-2f, -0x1.a9b662p-2f, 0x1.87de2ap-3f, 0x1.8f8b84p-4f, -0x1.6a09e6p-2f, 0x1.f6297cp-2f, -0x1.d906bcp-2f, 0x1.1c73b4p-2f,
    0x1.6a09e6p-2f, -0x1.f6297cp-2f, 0x1.d906bcp-2f, -0x1.a9b662p-2f, 0x1.6a09e6p-2f, -0x1.1c73b4p-2f, 0x1.87de2ap-3f, -0x1.8f8b84p-4f};
inline bool dct8_is_const(const DctMat& M)
{
    return std::memcmp(M.m, kDct8Host, 64 * sizeof(float)) == 0 && std::memcmp(M.mt, kDct8Host + 64, 64 * sizeof(float)) == 0;
}


}  // namespace dvc
