// Traceback kernels and launch dispatch of the CTC beam search
// (the per-frame kernel is in ctc_beam_kernel.inc).
#include "ctc_beam_kernel.inc"

namespace asr {

size_t ctc_lds_bytes(const CtcGeom& g) { return lds_plan(g).total; }

// Best-path traceback: per utterance, the maximum final score; among ties the
// smallest code string (std::map order, cpp:76-84).  Labels are written in
// forward order to best_lab[b][T].
__global__ __launch_bounds__(64) void ctc_best_kernel(CtcArgs a, const int* codes) {
    const int b = blockIdx.x, lane = threadIdx.x;
    const int kcap = a.g.kcap;
    const int n = a.fin_n[b];
    const double* sc = a.fin_score + (size_t)b * kcap;
    const int* fn = a.fin_node + (size_t)b * kcap;
    const int2* nodes = a.nodes + (size_t)b * a.T * kcap;
    const int nmax = a.T * kcap;
    int* out = a.best_lab + (size_t)b * a.T;

    uint64_t best = 0ull;
    for (int i = lane; i < n; i += 64) {
        const uint64_t k = asr_d2key(sc[i]);
        best = k > best ? k : best;
    }
    for (int o = 32; o > 0; o >>= 1) { uint64_t x = __shfl_xor(best, o); best = x > best ? x : best; }
    if (lane != 0) return;
    // Among ties (almost always one), keep the smallest code string.
    int bi = -1;
    for (int i = 0; i < n; i++) {
        if (asr_d2key(sc[i]) != best) continue;
        if (bi < 0) { bi = i; continue; }
        // Compare strings of slots i and bi from the front: materialise both
        // (reversed) then compare; ties are rare, this path is cold.
        int li = 0, lb = 0;
        for (int x = fn[i]; x >= 0 && x < nmax && li < a.T; x = nodes[x].x) li++;
        for (int x = fn[bi]; x >= 0 && x < nmax && lb < a.T; x = nodes[x].x) lb++;
        // k-th symbol from the front of slot s: walk (len-1-k) parents.
        bool less = false, decided = false;
        const int lmin = li < lb ? li : lb;
        for (int k = 0; k < lmin && !decided; k++) {
            int xi = fn[i], xb = fn[bi];
            for (int s = 0; s < li - 1 - k && xi >= 0; s++) xi = nodes[xi].x;
            for (int s = 0; s < lb - 1 - k && xb >= 0; s++) xb = nodes[xb].x;
            if (xi < 0 || xb < 0) break;
            const unsigned yi = (unsigned)nodes[xi].y, yb = (unsigned)nodes[xb].y;
            const int ci = yi < (unsigned)a.g.V ? codes[yi] : 0;
            const int cb = yb < (unsigned)a.g.V ? codes[yb] : 0;
            if (ci != cb) { less = ci < cb; decided = true; }
        }
        if (!decided) less = li < lb;
        if (less) bi = i;
    }
    if (bi < 0) {   // no final hypothesis (never expected: n >= 1)
        a.best_len[b] = 0;
        a.best_score[b] = -INFINITY;
        return;
    }
    int len = 0;
    // Links always point to earlier frames, so a chain has at most T nodes;
    // the bounds only guard against a corrupted table (never expected).
    for (int x = fn[bi]; x >= 0 && x < nmax && len < a.T; x = nodes[x].x) {
        const int2 e = nodes[x];
        out[len++] = e.y;
    }
    for (int i = 0, j = len - 1; i < j; i++, j--) {   // chased last-first: reverse
        const int tmp = out[i];
        out[i] = out[j];
        out[j] = tmp;
    }
    a.best_len[b] = len;
    a.best_score[b] = sc[bi];
}

// Full-beam traceback: every final hypothesis of every utterance, labels in
// forward order into all_lab[b][slot][T].
__global__ __launch_bounds__(64) void ctc_all_kernel(CtcArgs a, int* all_lab, int* all_len) {
    const int b = blockIdx.x;
    const int kcap = a.g.kcap;
    const int n = a.fin_n[b];
    const int* fn = a.fin_node + (size_t)b * kcap;
    const int2* nodes = a.nodes + (size_t)b * a.T * kcap;
    const int nmax = a.T * kcap;
    for (int i = threadIdx.x; i < n; i += 64) {
        int* out = all_lab + ((size_t)b * kcap + i) * a.T;
        int len = 0;
        for (int x = fn[i]; x >= 0 && x < nmax && len < a.T; x = nodes[x].x) out[len++] = nodes[x].y;
        for (int p = 0, q = len - 1; p < q; p++, q--) {
            const int tmp = out[p];
            out[p] = out[q];
            out[q] = tmp;
        }
        all_len[(size_t)b * kcap + i] = len;
    }
}

int ctc_launch_decode(const CtcArgs& a, int waves, hipStream_t s) {
    const int R = a.g.V + 1;
    const int rpt = a.g.kcap <= 64 ? 1 : (a.g.kcap <= 128 ? 2 : 4);
    if (R <= 8) return ctc_launch_decode_v8(a, waves, rpt, s);
    if (R <= 32) return ctc_launch_decode_v32(a, waves, rpt, s);
    if (R <= 64) return ctc_launch_decode_v64(a, waves, rpt, s);
    return ASR_ERR_UNSUPPORTED;
}

int ctc_launch_best(const CtcArgs& a, const int* d_codes, hipStream_t s) {
    hipLaunchKernelGGL(ctc_best_kernel, dim3(a.B), dim3(64), 0, s, a, d_codes);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

int ctc_launch_all(const CtcArgs& a, int* d_all_lab, int* d_all_len, hipStream_t s) {
    hipLaunchKernelGGL(ctc_all_kernel, dim3(a.B), dim3(64), 0, s, a, d_all_lab, d_all_len);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

int ctc_set_max_lds() {
    int rc = ctc_set_max_lds_v8();
    if (!rc) rc = ctc_set_max_lds_v32();
    if (!rc) rc = ctc_set_max_lds_v64();
    return rc;
}

}  // namespace asr
