// Instantiations of the one-wave-per-utterance beam-search kernel
// (ctc_wave_kernel.inc): rows per lane 1, 2, 4 (max_states <= 64, 128, 256).
#include "ctc_wave_kernel.inc"

namespace asr {

size_t ctc_lds_bytes_wave(const CtcGeom& g) {
    const bool c64 = g.V > 32;
    switch (ctc_row_capacity(g.kcap)) {
    case 64: return c64 ? WLds<64, true>::total(g.V) : WLds<64, false>::total(g.V);
    case 128: return c64 ? WLds<128, true>::total(g.V) : WLds<128, false>::total(g.V);
    default: return c64 ? WLds<256, true>::total(g.V) : WLds<256, false>::total(g.V);
    }
}

size_t ctc_seg_bytes_wave(const CtcGeom& g) {
    const bool c64 = g.V > 32;
    switch (ctc_row_capacity(g.kcap)) {
    case 64: return c64 ? WLds<64, true>::SEG : WLds<64, false>::SEG;
    case 128: return c64 ? WLds<128, true>::SEG : WLds<128, false>::SEG;
    default: return c64 ? WLds<256, true>::SEG : WLds<256, false>::SEG;
    }
}

bool ctc_wave_supported(const CtcGeom& g, int cu_mode) {
    return !cu_mode && g.V + 1 <= 64 && g.kcap <= 256 && ctc_lds_bytes_wave(g) <= 160u * 1024u;
}

int ctc_launch_decode_wave(const CtcArgs& a, hipStream_t s) {
    // the emission prefetch addresses a chunk's elements by 32-bit offsets
    if (((long)(wave_ch(a.g.V) - 1) * a.tstride + a.g.V) * 4 >= 0x7fffffffL) return ASR_ERR_UNSUPPORTED;
    const size_t lds = ctc_lds_bytes_wave(a.g);
    const dim3 grid(a.B), block(64);
    const bool c64 = a.g.V > 32;
    switch (ctc_row_capacity(a.g.kcap)) {
    case 64:
        if (c64) hipLaunchKernelGGL((ctc_wave_kernel<1, true>), grid, block, lds, s, a);
        else hipLaunchKernelGGL((ctc_wave_kernel<1, false>), grid, block, lds, s, a);
        break;
    case 128:
        if (c64) hipLaunchKernelGGL((ctc_wave_kernel<2, true>), grid, block, lds, s, a);
        else hipLaunchKernelGGL((ctc_wave_kernel<2, false>), grid, block, lds, s, a);
        break;
    default:
        if (c64) hipLaunchKernelGGL((ctc_wave_kernel<4, true>), grid, block, lds, s, a);
        else hipLaunchKernelGGL((ctc_wave_kernel<4, false>), grid, block, lds, s, a);
        break;
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
    const bool c64 = g.V > 32;
#define ASR_WOCC(r) c64 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, ctc_wave_kernel<r, true>, 64, lds) \
                        : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, ctc_wave_kernel<r, false>, 64, lds)
    switch (ctc_row_capacity(g.kcap)) {
    case 64: e = ASR_WOCC(1); break;
    case 128: e = ASR_WOCC(2); break;
    default: e = ASR_WOCC(4); break;
    }
#undef ASR_WOCC
    return e == hipSuccess ? n : 0;
}

int ctc_set_max_lds_wave() {
    const int lim = 160 * 1024;
#define ASR_WLIM(r, c) ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_wave_kernel<r, c>, \
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ASR_WLIM(1, false) ASR_WLIM(2, false) ASR_WLIM(4, false)
    ASR_WLIM(1, true) ASR_WLIM(2, true) ASR_WLIM(4, true)
#undef ASR_WLIM
    return ASR_OK;
}

}  // namespace asr
