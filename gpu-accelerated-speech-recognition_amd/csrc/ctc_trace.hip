// Traceback kernels and launch dispatch of the CTC beam search
// (the per-frame kernel is in ctc_beam_kernel.inc).
#include "ctc_beam_kernel.inc"

namespace asr {

int ctc_row_capacity(int kcap) { return kcap <= 64 ? 64 : (kcap <= 128 ? 128 : 256); }

size_t ctc_lds_bytes(const CtcGeom& g) {
    if (g.V + 1 > 64) return ctc_lds_bytes_wide(ctc_row_capacity(g.kcap), g.V);
    switch (ctc_row_capacity(g.kcap)) {
    case 64: return g.ts ? Lds<64>::total_ts(g.ch, g.V) : Lds<64>::total(g.ch, g.V);
    case 128: return g.ts ? Lds<128>::total_ts(g.ch, g.V) : Lds<128>::total(g.ch, g.V);
    default: return g.ts ? Lds<256>::total_ts(g.ch, g.V) : Lds<256>::total(g.ch, g.V);
    }
}

// A hypothesis is (node, tail): the chain of 8-label blocks ending at node
// (each record: parent node, 8 labels packed 8 bits each, first label lowest)
// followed by the tail's labels.  Links always point to earlier frames, so a
// chain has at most T/8 blocks; the bounds only guard a corrupted table.

// Labels are lbits wide: 8 (8 per record, up to 7 in a tail) or 16 (4 per
// record, up to 3 in a tail, wide-vocabulary kernel).
__device__ __forceinline__ uint32_t block_label(const int4 r, int k, int lbits) {
    const uint64_t pk = ((uint64_t)(uint32_t)r.w << 32) | (uint32_t)r.z;
    return (uint32_t)(pk >> (lbits * k)) & ((1u << lbits) - 1u);
}
__device__ __forceinline__ uint32_t tail_label(uint64_t tail, int k, int lbits) {
    return (uint32_t)(tail >> (lbits * k)) & ((1u << lbits) - 1u);
}

// Append frame k (16-bit field k) of a 128-bit frame record: a node's
// nodes_ts entry, or a final tail's two fin_ts words.
__device__ __forceinline__ int frame_field(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, int k) {
    const uint32_t wd = k < 2 ? w0 : (k < 4 ? w1 : (k < 6 ? w2 : w3));
    return (int)((wd >> (16 * (k & 1))) & 0xFFFFu);
}

// Chase the block chain of `x` into ids[] (last block first); returns the
// number of blocks.
__device__ int chase_blocks(const int4* nodes, int nmax, int x, int* ids, int maxb) {
    int nb = 0;
    for (; x >= 0 && x < nmax && nb < maxb; x = nodes[x].x) ids[nb++] = x;
    return nb;
}

// Label k (from the front) of a hypothesis whose blocks are ids[0..nb)
// (last first) followed by tail.
__device__ uint32_t label_at(const int4* nodes, const int* ids, int nb, uint64_t tail, int k,
                             int lbits) {
    const int per = 64 / lbits;
    if (k < per * nb) return block_label(nodes[ids[nb - 1 - k / per]], k % per, lbits);
    return tail_label(tail, k - per * nb, lbits);
}

// Best-path traceback: per utterance, the maximum final score; among ties the
// smallest code string (std::map order, cpp:76-84).  Labels are written in
// forward order to best_lab[b][T].  chain: [B][2][T/4+1] scratch.
__global__ __launch_bounds__(64) void ctc_best_kernel(CtcArgs a, const int* codes, int* chain) {
    const int b = blockIdx.x, lane = threadIdx.x;
    const int kcap = a.g.kcap;
    const int n = a.fin_n[b];
    const double* sc = a.fin_score + (size_t)b * kcap;
    const int* fn = a.fin_node + (size_t)b * kcap;
    const uint64_t* ft = a.fin_tail + (size_t)b * kcap;
    const int4* nodes = a.nodes + (size_t)b * a.T * kcap;
    const int nmax = a.T * kcap;
    const int lbits = a.g.lbits, per = 64 / lbits;
    const int maxb = a.T / 4 + 1;
    int* ids = chain + (size_t)b * 2 * maxb;   // best candidate's blocks
    int* ids2 = ids + maxb;                    // challenger's (ties only)
    int* out = a.best_lab + (size_t)b * a.T;
    __shared__ int s_nb, s_bi;

    uint64_t best = 0ull;
    for (int i = lane; i < n; i += 64) {
        const uint64_t k = asr_d2key(sc[i]);
        best = k > best ? k : best;
    }
    for (int o = 32; o > 0; o >>= 1) { uint64_t x = __shfl_xor(best, o); best = x > best ? x : best; }
    if (lane == 0) {
        // Among ties (almost always one), keep the smallest code string.
        int bi = -1, nb = 0;
        for (int i = 0; i < n; i++) {
            if (asr_d2key(sc[i]) != best) continue;
            if (bi < 0) {
                bi = i;
                nb = chase_blocks(nodes, nmax, fn[i], ids, maxb);
                continue;
            }
            const int nb2 = chase_blocks(nodes, nmax, fn[i], ids2, maxb);
            const int li = per * nb2 + (int)(ft[i] >> 56), lb = per * nb + (int)(ft[bi] >> 56);
            const int lmin = li < lb ? li : lb;
            bool less = li < lb, decided = false;
            for (int k = 0; k < lmin && !decided; k++) {
                const uint32_t yi = label_at(nodes, ids2, nb2, ft[i], k, lbits);
                const uint32_t yb = label_at(nodes, ids, nb, ft[bi], k, lbits);
                const int ci = yi < (unsigned)a.g.V ? codes[yi] : 0;
                const int cb = yb < (unsigned)a.g.V ? codes[yb] : 0;
                if (ci != cb) { less = ci < cb; decided = true; }
            }
            if (less) {   // the challenger becomes the best: keep its blocks
                bi = i;
                nb = nb2;
                for (int j = 0; j < nb2; j++) ids[j] = ids2[j];
            }
        }
        s_nb = nb;
        s_bi = bi;
    }
    __syncthreads();
    const int bi = s_bi, nb = s_nb;
    if (bi < 0) {   // no final hypothesis (never expected: n >= 1)
        if (lane == 0) {
            a.best_len[b] = 0;
            a.best_score[b] = -INFINITY;
        }
        return;
    }
    const uint64_t tail = ft[bi];
    const int nt = (int)(tail >> 56) < per ? (int)(tail >> 56) : per - 1;
    const int len = per * nb + nt <= a.T ? per * nb + nt : a.T;
    for (int j = lane; j < nb; j += 64) {   // block j from the front
        const int4 r = nodes[ids[nb - 1 - j]];
        for (int k = 0; k < per; k++)
            if (per * j + k < len) out[per * j + k] = (int)block_label(r, k, lbits);
    }
    if (lane < nt && per * nb + lane < len) out[per * nb + lane] = (int)tail_label(tail, lane, lbits);
    if (lane == 0) {
        a.best_len[b] = len;
        a.best_score[b] = sc[bi];
    }
}

// Full-beam traceback: every final hypothesis of every utterance, labels in
// forward order into all_lab[b][slot][T] (and, in timesteps mode, each
// label's append frame into all_ts[b][slot][T]).  One lane per hypothesis:
// count the blocks, then chase again writing each block at its final position.
__global__ __launch_bounds__(64) void ctc_all_kernel(CtcArgs a, int* all_lab, int* all_len, int* all_ts) {
    const int b = blockIdx.x;
    const int kcap = a.g.kcap;
    const int n = a.fin_n[b];
    const int* fn = a.fin_node + (size_t)b * kcap;
    const uint64_t* ft = a.fin_tail + (size_t)b * kcap;
    const int4* nodes = a.nodes + (size_t)b * a.T * kcap;
    const int nmax = a.T * kcap;
    const int lbits = a.g.lbits, per = 64 / lbits;
    const int maxb = a.T / 4 + 1;
    for (int i = threadIdx.x; i < n; i += 64) {
        int* out = all_lab + ((size_t)b * kcap + i) * a.T;
        int nb = 0;
        for (int x = fn[i]; x >= 0 && x < nmax && nb < maxb; x = nodes[x].x) nb++;
        const uint64_t tail = ft[i];
        const int nt = (int)(tail >> 56) < per ? (int)(tail >> 56) : per - 1;
        const int len = per * nb + nt <= a.T ? per * nb + nt : a.T;
        const bool ts = all_ts && a.nodes_ts;
        int* ots = ts ? all_ts + ((size_t)b * kcap + i) * a.T : nullptr;
        const int4* nts = ts ? a.nodes_ts + (size_t)b * a.T * kcap : nullptr;
        int j = nb - 1;
        for (int x = fn[i]; x >= 0 && x < nmax && j >= 0; x = nodes[x].x, j--) {
            const int4 r = nodes[x];
            for (int k = 0; k < per; k++)
                if (per * j + k < len) out[per * j + k] = (int)block_label(r, k, lbits);
            if (ts) {
                const int4 f = nts[x];
                for (int k = 0; k < per; k++)
                    if (per * j + k < len)
                        ots[per * j + k] = frame_field((uint32_t)f.x, (uint32_t)f.y, (uint32_t)f.z, (uint32_t)f.w, k);
            }
        }
        for (int k = 0; k < nt; k++)
            if (per * nb + k < len) out[per * nb + k] = (int)tail_label(tail, k, lbits);
        if (ts) {
            const uint64_t f0 = a.fin_ts[((size_t)b * kcap + i) * 2], f1 = a.fin_ts[((size_t)b * kcap + i) * 2 + 1];
            for (int k = 0; k < nt; k++)
                if (per * nb + k < len)
                    ots[per * nb + k] = frame_field((uint32_t)f0, (uint32_t)(f0 >> 32), (uint32_t)f1,
                                                    (uint32_t)(f1 >> 32), k);
        }
        all_len[(size_t)b * kcap + i] = len;
    }
}

int ctc_launch_decode(const CtcArgs& a, int waves, hipStream_t s) {
    if (waves < 0) return ctc_launch_decode_wave(a, s);
    const int R = a.g.V + 1;
    const int rpt = ctc_row_capacity(a.g.kcap) / 64;   // rows per thread: the layout's KC
    if (R <= 8) return ctc_launch_decode_v8(a, waves, rpt, s);
    if (R <= 32) return ctc_launch_decode_v32(a, waves, rpt, s);
    if (R <= 64) return ctc_launch_decode_v64(a, waves, rpt, s);
    return ctc_launch_decode_wide(a, rpt, s);
}

int ctc_occupancy(const CtcGeom& g, int waves) {
    const int R = g.V + 1;
    const int rpt = ctc_row_capacity(g.kcap) / 64;
    if (R <= 8) return ctc_occupancy_v8(g, waves, rpt);
    if (R <= 32) return ctc_occupancy_v32(g, waves, rpt);
    if (R <= 64) return ctc_occupancy_v64(g, waves, rpt);
    return 0;
}

int ctc_launch_best(const CtcArgs& a, const int* d_codes, int* d_chain, hipStream_t s) {
    hipLaunchKernelGGL(ctc_best_kernel, dim3(a.B), dim3(64), 0, s, a, d_codes, d_chain);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

int ctc_launch_all(const CtcArgs& a, int* d_all_lab, int* d_all_len, int* d_all_ts, hipStream_t s) {
    hipLaunchKernelGGL(ctc_all_kernel, dim3(a.B), dim3(64), 0, s, a, d_all_lab, d_all_len, d_all_ts);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

int ctc_set_max_lds() {
    int rc = ctc_set_max_lds_v8();
    if (!rc) rc = ctc_set_max_lds_v32();
    if (!rc) rc = ctc_set_max_lds_v64();
    if (!rc) rc = ctc_set_max_lds_wide();
    if (!rc) rc = ctc_set_max_lds_wave();
    return rc;
}

}  // namespace asr
