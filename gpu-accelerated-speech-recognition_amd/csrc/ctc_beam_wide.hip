// Instantiations of the large-vocabulary beam-search kernel (V+1 > 64
// columns, ctc_wide_kernel.inc): 8 waves, 1/2/4 rows per thread, CPU or
// .cu semantics.
#include "ctc_wide_kernel.inc"

namespace asr {

size_t ctc_tile0_bytes(int B, int T) { return sizeof(uint32_t) * WREC * (size_t)B * T; }

int ctc_launch_tile0(const CtcArgs& a, hipStream_t s) {
    if (!a.tile0 || a.g.V - 1 <= WTILE || a.g.V > WVMAX || a.t1 <= a.t0) return ASR_ERR_ARG;
    // the launch's frames [t0, t1) (a segment of a segmented decode)
    hipLaunchKernelGGL(ctc_tile0_kernel, dim3((unsigned)(a.B * (a.t1 - a.t0))), dim3(64), sizeof(uint32_t) * a.g.V,
                       s, a, a.tile0);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

int ctc_launch_decode_wide(const CtcArgs& a, int rpt, hipStream_t s) {
    if (a.tile0 && !a.tile0_ext) {   // every frame's first tile (ctc_tile0_kernel), then the decode
        if (int rc = ctc_launch_tile0(a, s)) return rc;
    }
    const size_t lds = ctc_lds_bytes(a.g);
    const dim3 grid(a.B), block(WNT);
#define ASR_W_LAUNCH(R)                                                                        \
    if (rpt == R) {                                                                            \
        if (a.cu_mode) hipLaunchKernelGGL((ctc_wide_kernel<R, true>), grid, block, lds, s, a); \
        else hipLaunchKernelGGL((ctc_wide_kernel<R, false>), grid, block, lds, s, a);          \
        ASR_LAUNCH_TRY();                                                                      \
        return ASR_OK;                                                                         \
    }
    ASR_W_LAUNCH(1)
    ASR_W_LAUNCH(2)
    ASR_W_LAUNCH(4)
#undef ASR_W_LAUNCH
    return ASR_ERR_UNSUPPORTED;
}

size_t ctc_seg_bytes_wide(int kc) {
    switch (kc) {
    case 64: return LdsW<64>::SEG;
    case 128: return LdsW<128>::SEG;
    default: return LdsW<256>::SEG;
    }
}

size_t ctc_lds_bytes_wide(int kc, int V) {
    switch (kc) {
    case 64: return LdsW<64>::total(V);
    case 128: return LdsW<128>::total(V);
    default: return LdsW<256>::total(V);
    }
}

int ctc_set_max_lds_wide() {
    const int lim = 160 * 1024;
#define ASR_W_ATTR(R, C) \
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_wide_kernel<R, C>, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ASR_W_ATTR(1, false) ASR_W_ATTR(2, false) ASR_W_ATTR(4, false)
    ASR_W_ATTR(1, true) ASR_W_ATTR(2, true) ASR_W_ATTR(4, true)
#undef ASR_W_ATTR
    return ASR_OK;
}

}  // namespace asr
