// Instantiations of the one-wave-per-utterance beam-search kernel
// (ctc_wave_kernel.inc): rows per lane 1, 2, 4 (max_states <= 64, 128, 256).
#include "ctc_wave_kernel.inc"

namespace asr {

size_t ctc_lds_bytes_wave(const CtcGeom& g) {
    switch (ctc_row_capacity(g.kcap)) {
    case 64: return WLds<64>::total(g.V);
    case 128: return WLds<128>::total(g.V);
    default: return WLds<256>::total(g.V);
    }
}

bool ctc_wave_supported(const CtcGeom& g, int cu_mode) {
    return !cu_mode && g.V + 1 <= 64 && g.kcap <= 256 && ctc_lds_bytes_wave(g) <= 160u * 1024u;
}

int ctc_launch_decode_wave(const CtcArgs& a, hipStream_t s) {
    const size_t lds = ctc_lds_bytes_wave(a.g);
    const dim3 grid(a.B), block(64);
    switch (ctc_row_capacity(a.g.kcap)) {
    case 64: hipLaunchKernelGGL(ctc_wave_kernel<1>, grid, block, lds, s, a); break;
    case 128: hipLaunchKernelGGL(ctc_wave_kernel<2>, grid, block, lds, s, a); break;
    default: hipLaunchKernelGGL(ctc_wave_kernel<4>, grid, block, lds, s, a); break;
    }
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

// Utterances (one-wave workgroups) that fit on one CU at this layout's LDS
// size (registers, LDS, wave slots: the runtime's occupancy query); 0 on failure.
int ctc_occupancy_wave(const CtcGeom& g) {
    const size_t lds = ctc_lds_bytes_wave(g);
    int n = 0;
    hipError_t e;
    switch (ctc_row_capacity(g.kcap)) {
    case 64: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, ctc_wave_kernel<1>, 64, lds); break;
    case 128: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, ctc_wave_kernel<2>, 64, lds); break;
    default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, ctc_wave_kernel<4>, 64, lds); break;
    }
    return e == hipSuccess ? n : 0;
}

int ctc_set_max_lds_wave() {
    const int lim = 160 * 1024;
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_wave_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_wave_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_wave_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    return ASR_OK;
}

}  // namespace asr
