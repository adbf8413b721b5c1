// Instantiations of the beam-search kernel for vocabularies with V+1 <= 8
// columns (ctc_beam_kernel.inc).  Split per vocabulary class so that the
// template variants compile in parallel.  The .cu-semantics variants
// (CU = true, asr_ctc_set_semantics) exist for the automatic wave count only.
#include "ctc_beam_kernel.inc"

namespace asr {

#define ASR_VARIANTS(X) \
    X(1, 8, 1) \
    X(1, 8, 2) \
    X(2, 4, 1) \
    X(2, 4, 2) \
    X(4, 2, 1) \
    X(4, 2, 2) \
    X(4, 2, 4) \

#define ASR_CU_VARIANTS(X) \
    X(4, 2, 1) \
    X(4, 2, 2) \
    X(4, 2, 4) \

int ctc_launch_decode_v8(const CtcArgs& a, int waves, int rpt, hipStream_t s) {
    const size_t lds = ctc_lds_bytes(a.g);
    const dim3 grid(a.B);
#define X(nw, cw, rp)                                                                     \
    if (waves == nw && rpt == rp) {                                                       \
        if (a.cu_mode) return ASR_ERR_UNSUPPORTED;                                        \
        hipLaunchKernelGGL((ctc_beam_kernel<nw, cw, rp, false>), grid, dim3(64 * nw), lds, s, a); \
        ASR_LAUNCH_TRY();                                                                 \
        return ASR_OK;                                                                    \
    }
#define XC(nw, cw, rp)                                                                    \
    if (a.cu_mode && waves == nw && rpt == rp) {                                          \
        hipLaunchKernelGGL((ctc_beam_kernel<nw, cw, rp, true>), grid, dim3(64 * nw), lds, s, a); \
        ASR_LAUNCH_TRY();                                                                 \
        return ASR_OK;                                                                    \
    }
    ASR_CU_VARIANTS(XC)
    ASR_VARIANTS(X)
#undef X
#undef XC
    return ASR_ERR_UNSUPPORTED;
}

int ctc_set_max_lds_v8() {
    const int lim = 160 * 1024;
#define X(nw, cw, rp)                                                                        \
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_beam_kernel<nw, cw, rp, false>,          \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lim));
#define XC(nw, cw, rp)                                                                       \
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_beam_kernel<nw, cw, rp, true>,           \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ASR_VARIANTS(X)
    ASR_CU_VARIANTS(XC)
#undef X
#undef XC
    return ASR_OK;
}

// Workgroups of the (waves, rpt) variant that fit on one CU at this layout's
// LDS size (registers, LDS and wave slots; the runtime's occupancy query), for
// the automatic schedule choice (runtime.hip auto_waves).  0 if not built.
int ctc_occupancy_v8(const CtcGeom& g, int waves, int rpt) {
    const size_t lds = ctc_lds_bytes(g);
    int n = 0;
#define X(nw, cw, rp)                                                                        \
    if (waves == nw && rpt == rp) {                                                          \
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(                                    \
                &n, ctc_beam_kernel<nw, cw, rp, false>, 64 * nw, lds) != hipSuccess)         \
            return 0;                                                                        \
        return n;                                                                            \
    }
    ASR_VARIANTS(X)
#undef X
    return 0;
}

}  // namespace asr
