// fd_kernels.h — launch interface between the C-ABI host code (fd_api.hip) and
// the gfx950 kernels (fd_kernels.hip). Internal; not part of include/dvc.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dvc {

// Row geometry of the run-length (CCL) stage.
struct RowGeom {
    int W, H;
    int WW;   // 64-px words per mask row = ceil(W/64)
    int CAP;  // max foreground runs per row = W/2 + 1 (gaps per row <= CAP+1)
};

struct GaussTaps {
    int n;
    uint16_t t[64];
};

struct DctMat {
    float m[64];  // BxB row-major orthonormal DCT-II basis M[k][n], float32
};

// Device buffers of the contour-filter stage of one feed.
struct CclBufs {
    const uint64_t* mbits;  // H x WW motion mask
    uint64_t* fbits;        // H x WW filled mask (not-E)
    uint16_t *rs, *re;      // H x CAP run starts / ends
    uint32_t* nfg;          // H runs per row
    uint32_t* fpar;         // H x CAP run union-find parents (root after k_area)
    uint32_t* gpar;         // 1 + H x (CAP+1) gap parents, node 0 = outside
    uint8_t* gE;            // H x (CAP+1) gap is outside (1) / hole (0)
    uint32_t* area2;        // H x CAP 2*area per root
    uint64_t* kbits;        // H x WW kept (filtered) mask
    unsigned long long* stats;  // 64 slots x 4 counters
};

struct BackArgs {
    RowGeom g;
    const uint8_t* bgr;
    int pitch;
    uint8_t* acc;
    uint8_t* overlay;     // nullable
    uint8_t* compressed;  // nullable
    int opitch;
    const uint64_t* kbits;  // kept (filtered) mask from k_paint
    int ksize, anchor;
    float alpha, beta, gamma, quant;
    DctMat M;
    unsigned long long* stats;
    uint64_t* dbg_dil;   // nullable: dilated mask bits
};

hipError_t launch_prime(const uint8_t* bgr, int pitch, uint8_t* gray_tmp, uint32_t* tmp32, uint8_t* out,
                        int W, int H, const GaussTaps& k, hipStream_t s);
hipError_t launch_front(const uint8_t* bgr, int pitch, const uint8_t* prev, uint8_t* cur, uint64_t* mbits,
                        const RowGeom& g, int ithresh, hipStream_t s);
int band_rows(const RowGeom& g);
hipError_t launch_ccl(const CclBufs& c, const RowGeom& g, int64_t min_area2, hipStream_t s);
hipError_t launch_back(const BackArgs& a, int block, hipStream_t s);

}  // namespace dvc
