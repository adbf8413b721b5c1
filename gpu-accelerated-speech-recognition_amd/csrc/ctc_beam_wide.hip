// Instantiations of the large-vocabulary beam-search kernel (V+1 > 64
// columns, ctc_wide_kernel.inc): 8 waves, 1/2/4 rows per thread.
#include "ctc_wide_kernel.inc"

namespace asr {

int ctc_launch_decode_wide(const CtcArgs& a, int rpt, hipStream_t s) {
    const size_t lds = ctc_lds_bytes(a.g);
    const dim3 grid(a.B), block(WNT);
    if (rpt == 1) { hipLaunchKernelGGL((ctc_wide_kernel<1>), grid, block, lds, s, a); ASR_LAUNCH_TRY(); return ASR_OK; }
    if (rpt == 2) { hipLaunchKernelGGL((ctc_wide_kernel<2>), grid, block, lds, s, a); ASR_LAUNCH_TRY(); return ASR_OK; }
    if (rpt == 4) { hipLaunchKernelGGL((ctc_wide_kernel<4>), grid, block, lds, s, a); ASR_LAUNCH_TRY(); return ASR_OK; }
    return ASR_ERR_UNSUPPORTED;
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
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_wide_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_wide_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_wide_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    return ASR_OK;
}

}  // namespace asr
