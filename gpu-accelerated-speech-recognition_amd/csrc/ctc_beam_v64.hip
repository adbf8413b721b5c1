// Instantiations of the beam-search kernel for vocabularies with V+1 <= 64
// columns (ctc_beam_kernel.inc).  Split per vocabulary class so that the
// template variants compile in parallel.
#include "ctc_beam_kernel.inc"

namespace asr {

int ctc_launch_decode_v64(const CtcArgs& a, int waves, int rpt, hipStream_t s) {
    const size_t lds = ctc_lds_bytes(a.g);
    const dim3 grid(a.B);
    if (waves == 2 && rpt == 1) { hipLaunchKernelGGL((ctc_beam_kernel<2, 32, 1>), grid, dim3(128), lds, s, a); ASR_LAUNCH_TRY(); return ASR_OK; }
    if (waves == 2 && rpt == 2) { hipLaunchKernelGGL((ctc_beam_kernel<2, 32, 2>), grid, dim3(128), lds, s, a); ASR_LAUNCH_TRY(); return ASR_OK; }
    if (waves == 4 && rpt == 1) { hipLaunchKernelGGL((ctc_beam_kernel<4, 16, 1>), grid, dim3(256), lds, s, a); ASR_LAUNCH_TRY(); return ASR_OK; }
    if (waves == 4 && rpt == 2) { hipLaunchKernelGGL((ctc_beam_kernel<4, 16, 2>), grid, dim3(256), lds, s, a); ASR_LAUNCH_TRY(); return ASR_OK; }
    if (waves == 4 && rpt == 4) { hipLaunchKernelGGL((ctc_beam_kernel<4, 16, 4>), grid, dim3(256), lds, s, a); ASR_LAUNCH_TRY(); return ASR_OK; }
    if (waves == 8 && rpt == 1) { hipLaunchKernelGGL((ctc_beam_kernel<8, 8, 1>), grid, dim3(512), lds, s, a); ASR_LAUNCH_TRY(); return ASR_OK; }
    if (waves == 8 && rpt == 2) { hipLaunchKernelGGL((ctc_beam_kernel<8, 8, 2>), grid, dim3(512), lds, s, a); ASR_LAUNCH_TRY(); return ASR_OK; }
    if (waves == 8 && rpt == 4) { hipLaunchKernelGGL((ctc_beam_kernel<8, 8, 4>), grid, dim3(512), lds, s, a); ASR_LAUNCH_TRY(); return ASR_OK; }
    return ASR_ERR_UNSUPPORTED;
}

int ctc_set_max_lds_v64() {
    const int lim = 160 * 1024;
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_beam_kernel<2, 32, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_beam_kernel<2, 32, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_beam_kernel<4, 16, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_beam_kernel<4, 16, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_beam_kernel<4, 16, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_beam_kernel<8, 8, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_beam_kernel<8, 8, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_beam_kernel<8, 8, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    return ASR_OK;
}

}  // namespace asr
