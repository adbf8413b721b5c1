// ============================================================================
// Native throughput pipeline (asr_pipeline_*, include/asr_amd.h): the hot
// path RNN (input projection + recurrence) -> Linear + log_softmax -> CTC
// beam search over a stream of equal-shape batches, with the production of
// later batches overlapped with the decodes of earlier ones on library-owned
// HIP streams.  The reference runs one batch at a time on the default stream
// with host syncs between every call (main.cpp:40-72, RNN.cu:9-30,
// CTCBeamSearch.cu:262-312); a decode is sequential in T and one batch
// leaves most CUs idle or starves its own production, so throughput needs
// several batches in flight and a placement of the kernels on the CUs.
//
// Schedules (chosen from the shapes):
//   GROUPS  small batches (<= 1/4 of the CUs at one decode workgroup per
//           utterance, H <= 256; C2): D = 3 decode streams, each restricted
//           to its own group of CUs (one workgroup per utterance), the
//           recurrence on the remaining CUs, the input / emission GEMMs on a
//           stream over every CU, the input projection issued one batch
//           ahead so that it overlaps the previous batch's recurrence.
//   SHARED  batches that fill the chip (H <= 256, beam capacity <= 64; C4's
//           shards): the decodes get half of the CUs and D batches decode
//           there at once, 16 utterances per decode CU (the one-wave
//           kernel's occupancy; the decoders learn the load through
//           asr_ctc_set_concurrency), the production the other half on 3-4
//           streams with the MFMA recurrence — from round 3 the recurrence
//           with the emission projection fused (asr_rnn_emit_fwd, V <= 32),
//           part of the input projection optionally on the decode CUs.
//   GROUPS2 H > 256 (C5: 2000 per-frame recurrence launches, replayed from
//           the library's HIP graph): D = 2 decode groups, 2 production
//           streams on the remaining CUs; optionally the recurrences of G
//           consecutive batches as one (production groups, measured slower
//           at C5, off by default).
// Results come back in submission order (asr_pipeline_collect).  A batch's
// buffers are reused only after its results were fetched (the decoder's
// overflow retry re-reads its emissions): submit collects internally when
// the caller is nbuf batches behind.
// ============================================================================
#include <hip/hip_ext.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <vector>

#include "asr_internal.h"
#include "dense.h"

namespace {

enum Mode { GROUPS = 0, SHARED = 1, GROUPS2 = 2 };

struct Result {
    std::vector<int32_t> lab, len;
    std::vector<double> lp;
    float ms = 0.f;
    int rc = ASR_OK;
    long batch = -1;
};

}  // namespace

struct asr_pipeline {
    asr_pipeline_config cfg{};
    const float *W_ih = nullptr, *W_hh = nullptr, *b_ih = nullptr, *b_hh = nullptr;
    const float *W_out = nullptr, *b_out = nullptr;
    int ncu = 0, mode = SHARED, D = 1, P = 1, nbuf = 2, gcu = 0, dcus = 0, rnn_kind = -1;
    int arith = -1;       // the dense arithmetic latched at creation (asr_internal_dense_arith)
    int ngroups = 1;      // CU groups of the decodes (GROUPS / GROUPS2): decode d on group d % ngroups
    bool split = false;   // GROUPS: input GEMM / recurrence / emission GEMM on two streams
    bool fuse = false;    // SHARED: recurrence + emission projection in one kernel (asr_rnn_emit_fwd)
    // fused split-bf16 production: the input projection is stored in the
    // recurrence's fragment-major layout (asr::gemm_x3_frag_launch: two
    // 16-byte stores / loads per lane instead of eight 4-byte ones; the same
    // values, so the same emission bits as asr_linear_fwd + asr_rnn_emit_fwd)
    bool pfrag = false;
    long grows = 0;       // SHARED + fuse: input-projection rows run on the decode CUs
    int gtiled = 0;       // ... with the tiled GEMM kernel, row tiles per workgroup (0: persistent)
    int S = 1;            // T-segments per batch (fused production only)
    double seg0 = 0.0;    // first segment's share of T when S = 2 (0: T / 2)
    // Dynamic batching (asr_pipeline_create_coalesced): cg consecutive
    // submits of Bo utterances each are one pipeline batch of cfg.B = cg * Bo
    // utterances (one production and one decode launch for all of them).
    int cg = 1, Bo = 0;
    std::vector<float*> stage;   // inputs [T][cfg.B][in] of the batches being assembled / in flight
    int cfill = 0;               // columns of pipeline batch `submitted` filled so far
    std::deque<std::pair<long, int>> opend;   // caller's uncollected batches: (pipeline batch, column)
    Result ocache;               // the pipeline batch whose rows collects are returning
    long ocache_q = -1;
    int ocol = 0;                // column of the caller's batch collected last
    bool tile0_prod = false;   // the wide decoder's first tiles computed by the production (produce_full_segments)
    // Drain (S > 1): the last decode segment of the newest `hold` batches is
    // held back.  A newer batch releases the oldest onto its decode stream
    // (the steady state); when the caller drains (collects a batch within D
    // of a held one), every held segment is queued on its batch's production
    // stream instead, behind that stream's last production: the drain's
    // decodes then also use the production CUs, which are idle by then.
    int hold = 0;
    std::deque<long> held;
    std::vector<hipEvent_t> ev_dpre;  // [nbuf] decode of segments [0, S - 1) of buffer k done
    int pcus = 0;         // CUs one production stream's recurrence may count on (one-launch H > 256 recurrence)
    int G = 1;            // GROUPS2: batches whose recurrences run as one (a production group)
    std::vector<long> group;          // batches whose input projection is queued, recurrence not yet
    std::vector<float*> hst;          // [nbuf][B][H] the recurrence's h at a segment end
    std::vector<hipEvent_t> ev_seg;   // [nbuf][S] segment s of buffer k's emissions ready
    hipStream_t s_gdec = nullptr;   // the decode CUs' share of the input projections
    std::vector<float*> hid, emis;
    std::vector<asr_ctc_t*> dec;
    std::vector<hipStream_t> s_dec, s_prod;
    hipStream_t s_gemm = nullptr;
    // split production: the emission GEMMs on a stream of their own, so that
    // the next batch's input GEMM does not queue behind the previous batch's
    // emission GEMM, which waits for that batch's whole recurrence (C2: the
    // recurrence stalled 65-150 us per batch for its input); s_gemm itself
    // when the hardware queues are short
    hipStream_t s_tail = nullptr;
    bool tail_own = false;
    std::vector<hipEvent_t> ev_ready, ev_free, ev_proj, ev_rec;
    long submitted = 0, decoded = 0, collected = 0;
    long pending_tail = -1;   // split production: batch whose emission GEMM and decode are not queued yet
    std::deque<Result> stash;
    long returned = -1;   // the batch the last asr_pipeline_collect returned
    // A batch accepted by submit whose remaining work (emission GEMM, decode)
    // then failed to queue can never return results: from it on the pipeline
    // is failed, and every later submit / collect returns fail_rc.
    long fail_from = -1;
    int fail_rc = ASR_OK;
    int hw_queues = 4, streams = 0;   // HIP hardware queues of the process, streams created
    int shared_queue_streams = 0;     // ... of which unmasked (they share the hw_queues)
    // every stream created: role (ASR_PIPE_ROLE_*) and CU range [lo, hi) of its mask
    struct Placed { int role, lo, hi; hipStream_t s; };
    std::vector<Placed> placed;
    // Timeline (asr_pipeline_set_timing): per buffer, timing events at
    // production start / end and decode start / end, read back per batch at
    // its fetch as ms after the reference event ev_t0ref.
    bool timing = false;
    long timing_from = 0;
    hipEvent_t ev_t0ref = nullptr;
    std::vector<hipEvent_t> ev_t[4];
    struct Stamp { long batch; float t[4]; };
    std::vector<Stamp> timeline;
    // test hook (ASR_PIPELINE_FAULT=<batch>:<stage>, stage head|tail|produce|decode):
    // the named stage of that batch returns ASR_ERR_INTERNAL instead of queueing
    long fault_batch = -1;
    char fault_stage[8] = {0};
};

namespace {

bool fault(asr_pipeline* p, long i, const char* stage) {   // fires once
    if (i != p->fault_batch || std::strcmp(p->fault_stage, stage) != 0) return false;
    p->fault_batch = -1;
    return true;
}

// One-wave decoder utterances per CU for this configuration's beam (0: the
// one-wave kernel does not apply).
int wave_occupancy(const asr_pipeline_config& c) {
    asr_ctc_t* h = nullptr;
    if (asr_ctc_create(nullptr, c.V, c.beam, c.blank, 0, &h) != ASR_OK) return 0;
    const int n = asr_internal_ctc_wave_occupancy(h);
    asr_ctc_destroy(h);
    return n;
}

// The automatic T-segment count of a fused chip-filling production (the
// measurements are at asr_pipeline_create's use of it).
int auto_segments(const asr_pipeline_config& c, int kcap) {
    const bool x3s = asr::dense_x3_on() && kcap <= 64;
    return x3s && c.B >= 512 && c.B < 1024 ? 4 : (c.B < 512 || x3s) ? 2 : 1;
}

// Timeline stamp `which` (0 production start, 1 production end, 2 decode
// start, 3 decode end) of buffer k on stream s, when timing is on.
int mark(asr_pipeline* p, int which, int k, hipStream_t s) {
    if (p->timing) ASR_HIP_TRY(hipEventRecord(p->ev_t[which][k], s));
    return ASR_OK;
}

// First frame of T-segment s (s = S: T).
int seg_bound(const asr_pipeline* p, int s) {
    const int T = p->cfg.T;
    if (s <= 0) return 0;
    if (s >= p->S) return T;
    if (p->S == 2 && p->seg0 > 0.0) return std::max(1, std::min(T - 1, (int)(p->seg0 * T + 0.5)));
    return (int)((long)T * s / p->S);
}

void set_failed(asr_pipeline* p, long from, int rc) {
    if (p->fail_from < 0 || from < p->fail_from) p->fail_from = from;
    if (p->fail_rc == ASR_OK) p->fail_rc = rc;
}

int cu_stream(hipStream_t* s, int ncu, int lo, int hi) {
    if (lo <= 0 && hi >= ncu) {
        ASR_HIP_TRY(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
        return ASR_OK;
    }
    const int words = (ncu + 31) / 32;
    std::vector<uint32_t> m(words, 0u);
    for (int c = std::max(0, lo); c < std::min(ncu, hi); c++) m[c / 32] |= 1u << (c % 32);
    ASR_HIP_TRY(hipExtStreamCreateWithCUMask(s, (uint32_t)words, m.data()));
    return ASR_OK;
}

// Sets this thread's dense arithmetic to a pipeline's latched one for the
// scope of a pipeline call (restores the previous value).
struct ArithGuard {
    int prev;
    explicit ArithGuard(int a) : prev(asr_internal_dense_arith) { asr_internal_dense_arith = a; }
    ~ArithGuard() { asr_internal_dense_arith = prev; }
};

// The fused production's input projection of `rows` rows (x rows -> P rows):
// fragment-major when the pipeline reads it so, else asr_linear_fwd.
int input_projection(asr_pipeline* p, const float* x, float* P, long rows, int tiled, hipStream_t st) {
    const auto& c = p->cfg;
    if (p->pfrag) return asr::gemm_x3_frag_launch(x, p->W_ih, P, (int)rows, c.in, c.H, tiled, st);
    asr_internal_gemm_tiled = tiled;
    const int rc = asr_linear_fwd(x, p->W_ih, nullptr, P, (int)rows, c.in, c.H, ASR_EPI_NONE, st);
    asr_internal_gemm_tiled = 0;
    return rc;
}

// The unfused production in S T-segments (H > 256 with the wide decoder:
// C5): segment s is its rows of the input projection, the recurrence over
// its frames from h_{t0-1} (the previous segment's last hidden rows), and its
// rows of the emission projection + log_softmax; event ev_seg[k][s] releases
// the decode of those frames.  Rows and frames are independent and the
// kernels are chosen by shape, not M: the unsegmented production's bits.
int produce_full_segments(asr_pipeline* p, long i, const float* x, hipStream_t sp) {
    const auto& c = p->cfg;
    const int k = (int)(i % p->nbuf);
    int rc = ASR_OK;
    for (int s = 0; s < p->S && !rc; s++) {
        const int t0 = seg_bound(p, s), t1 = seg_bound(p, s + 1);
        const long r0 = (long)t0 * c.B, rows = (long)(t1 - t0) * c.B;
        float* hs = p->hid[k] + r0 * c.H;
        rc = asr_linear_fwd(x + r0 * c.in, p->W_ih, nullptr, hs, (int)rows, c.in, c.H, ASR_EPI_NONE, sp);
        if (rc) return rc;
        asr_internal_rnn_kind = p->rnn_kind;
        asr_internal_graph_now = 1;
        asr_internal_persist_cus = p->pcus;
        rc = asr_rnn_recur_fwd(s > 0 ? hs - (long)c.B * c.H : nullptr, p->W_hh, p->b_ih, p->b_hh, hs, t1 - t0, c.B,
                               c.H, sp);
        asr_internal_persist_cus = 0;
        asr_internal_graph_now = 0;
        asr_internal_rnn_kind = -1;
        if (!rc) rc = asr_linear_fwd(hs, p->W_out, p->b_out, p->emis[k] + r0 * c.V, (int)rows, c.H, c.V,
                                     ASR_EPI_BIAS_LOGSOFTMAX, sp);
        // the wide decoder's first-tile records of these frames, here on the
        // production CUs instead of ahead of the decode on its CU group
        if (!rc && p->tile0_prod)
            rc = asr_internal_ctc_tile0(p->dec[k], p->emis[k] + r0 * c.V, c.T, t0, t1, c.B, (long)c.B * c.V, c.V, sp);
        if (rc) return rc;
        ASR_HIP_TRY(hipEventRecord(p->ev_seg[(size_t)k * p->S + s], sp));
    }
    if (int r = mark(p, 1, k, sp)) return r;
    ASR_HIP_TRY(hipEventRecord(p->ev_ready[k], sp));
    return ASR_OK;
}

// Production of batch i into buffer k (unsplit): RNN forward + emission projection.
int produce_full(asr_pipeline* p, long i, const float* x) {
    const auto& c = p->cfg;
    const int k = (int)(i % p->nbuf);
    hipStream_t sp = p->s_prod[i % p->P];
    if (fault(p, i, "produce")) return ASR_ERR_INTERNAL;
    ASR_HIP_TRY(hipStreamWaitEvent(sp, p->ev_free[k], 0));   // the decode reading this buffer is done
    if (int r = mark(p, 0, k, sp)) return r;
    if (p->S > 1) return produce_full_segments(p, i, x, sp);
    asr_internal_rnn_kind = p->rnn_kind;
    asr_internal_graph_now = 1;
    asr_internal_persist_cus = p->pcus;
    int rc = asr_rnn_fwd(x, nullptr, p->W_ih, p->W_hh, p->b_ih, p->b_hh, p->hid[k], c.T, c.B, c.in, c.H, sp);
    asr_internal_persist_cus = 0;
    asr_internal_graph_now = 0;
    asr_internal_rnn_kind = -1;
    if (!rc) rc = asr_linear_fwd(p->hid[k], p->W_out, p->b_out, p->emis[k], c.T * c.B, c.H, c.V,
                                 ASR_EPI_BIAS_LOGSOFTMAX, sp);
    if (rc) return rc;
    if (int r = mark(p, 1, k, sp)) return r;
    ASR_HIP_TRY(hipEventRecord(p->ev_ready[k], sp));
    return ASR_OK;
}

// The fused production in S T-segments: segment s (frames [t0, t1)) is its
// rows of the input projection (the decode CUs' share first, as below), then
// the fused recurrence over those frames from h_{t0-1} (hst[k], written by
// segment s-1), its last h to hst[k]; event ev_seg[k][s] releases the
// decode of those frames.  The same kernels over the same rows in the same
// order: the emissions are the unsegmented production's bits.
int produce_fused_segments(asr_pipeline* p, long i, const float* x, hipStream_t sp) {
    const auto& c = p->cfg;
    const int k = (int)(i % p->nbuf);
    const long frac128 = p->grows;   // decode-CU rows of the whole batch
    int rc = ASR_OK;
    if (frac128 > 0) ASR_HIP_TRY(hipStreamWaitEvent(p->s_gdec, p->ev_free[k], 0));
    for (int s = 0; s < p->S && !rc; s++) {
        const int t0 = seg_bound(p, s), t1 = seg_bound(p, s + 1);
        const long r0 = (long)t0 * c.B, rows = (long)(t1 - t0) * c.B;
        const long ga = frac128 > 0 ? std::min(rows, frac128 * rows / ((long)c.T * c.B) / 128 * 128) : 0;
        if (ga > 0) {
            rc = input_projection(p, x + r0 * c.in, p->hid[k] + r0 * c.H, ga, p->gtiled, p->s_gdec);
            if (rc) return rc;
            ASR_HIP_TRY(hipEventRecord(p->ev_proj[k], p->s_gdec));
        }
        if (ga < rows)
            rc = input_projection(p, x + (r0 + ga) * c.in, p->hid[k] + (r0 + ga) * c.H, rows - ga, 0, sp);
        if (rc) return rc;
        if (ga > 0) ASR_HIP_TRY(hipStreamWaitEvent(sp, p->ev_proj[k], 0));
        rc = asr::rnn_emit_mfma_launch(s > 0 ? p->hst[k] : nullptr, p->W_hh, p->b_ih, p->b_hh,
                                       p->hid[k] + r0 * c.H, nullptr, p->W_out, p->b_out,
                                       p->emis[k] + (long)t0 * c.B * c.V, t1 - t0, c.B, c.H, c.V, sp,
                                       s + 1 < p->S ? p->hst[k] : nullptr, p->pfrag);
        if (rc) return rc;
        ASR_HIP_TRY(hipEventRecord(p->ev_seg[(size_t)k * p->S + s], sp));
    }
    if (int r = mark(p, 1, k, sp)) return r;
    ASR_HIP_TRY(hipEventRecord(p->ev_ready[k], sp));
    return ASR_OK;
}

// Fused production of batch i into buffer k (chip-filling batches, H <= 256,
// V <= 32): the input projection P = x.W_ih into hid[k] — its first grows rows
// on the decode CUs (s_gdec, which runs them whenever the decodes leave those
// CUs free, so the decode and production halves of the chip carry equal
// work), the rest on the production stream — then the recurrence with the
// emission projection + log_softmax fused (asr_rnn_emit_fwd: the hidden
// states never go to HBM).  Rows are independent, so the split never changes
// a bit (the wide and tiled GEMM kernels accumulate in the same k order).
int produce_fused(asr_pipeline* p, long i, const float* x) {
    const auto& c = p->cfg;
    const int k = (int)(i % p->nbuf);
    hipStream_t sp = p->s_prod[i % p->P];
    const long M = (long)c.T * c.B;
    const long ga = std::min(p->grows, M);
    if (fault(p, i, "produce")) return ASR_ERR_INTERNAL;
    ASR_HIP_TRY(hipStreamWaitEvent(sp, p->ev_free[k], 0));   // the decode reading this buffer is done
    if (int r = mark(p, 0, k, sp)) return r;
    if (p->S > 1) return produce_fused_segments(p, i, x, sp);
    int rc = ASR_OK;
    if (ga > 0) {
        ASR_HIP_TRY(hipStreamWaitEvent(p->s_gdec, p->ev_free[k], 0));
        // with several decodes in flight the decode-side rows use the tiled
        // kernel: a decode launched meanwhile then waits at most one tile's
        // workgroups for its CUs, not a persistent workgroup's whole share
        rc = input_projection(p, x, p->hid[k], ga, p->gtiled, p->s_gdec);
        if (rc) return rc;
        ASR_HIP_TRY(hipEventRecord(p->ev_proj[k], p->s_gdec));
    }
    if (ga < M) rc = input_projection(p, x + ga * c.in, p->hid[k] + ga * c.H, M - ga, 0, sp);
    if (rc) return rc;
    if (ga > 0) ASR_HIP_TRY(hipStreamWaitEvent(sp, p->ev_proj[k], 0));
    rc = p->pfrag ? asr::rnn_emit_mfma_launch(nullptr, p->W_hh, p->b_ih, p->b_hh, p->hid[k], nullptr, p->W_out,
                                              p->b_out, p->emis[k], c.T, c.B, c.H, c.V, sp, nullptr, true)
                  : asr_rnn_emit_fwd(nullptr, p->W_hh, p->b_ih, p->b_hh, p->W_out, p->b_out, p->hid[k], nullptr,
                                     p->emis[k], c.T, c.B, c.H, c.V, sp);
    if (rc) return rc;
    if (int r = mark(p, 1, k, sp)) return r;
    ASR_HIP_TRY(hipEventRecord(p->ev_ready[k], sp));
    return ASR_OK;
}

// Split production, part 1: input projection on the GEMM stream, recurrence
// on the recurrence stream.
int produce_head(asr_pipeline* p, long i, const float* x) {
    const auto& c = p->cfg;
    const int k = (int)(i % p->nbuf);
    if (fault(p, i, "head")) return ASR_ERR_INTERNAL;
    // hid[k]'s previous batch: its emission GEMM has read it (stream order
    // when both GEMMs share s_gemm)
    if (p->tail_own) ASR_HIP_TRY(hipStreamWaitEvent(p->s_gemm, p->ev_ready[k], 0));
    if (int r = mark(p, 0, k, p->s_gemm)) return r;
    asr_internal_gemm_tiled = p->gtiled;
    int rc = asr_linear_fwd(x, p->W_ih, nullptr, p->hid[k], c.T * c.B, c.in, c.H, ASR_EPI_NONE, p->s_gemm);
    asr_internal_gemm_tiled = 0;
    if (rc) return rc;
    ASR_HIP_TRY(hipEventRecord(p->ev_proj[k], p->s_gemm));
    ASR_HIP_TRY(hipStreamWaitEvent(p->s_prod[0], p->ev_proj[k], 0));
    asr_internal_rnn_kind = p->rnn_kind;
    rc = asr_rnn_recur_fwd(nullptr, p->W_hh, p->b_ih, p->b_hh, p->hid[k], c.T, c.B, c.H, p->s_prod[0]);
    asr_internal_rnn_kind = -1;
    if (rc) return rc;
    ASR_HIP_TRY(hipEventRecord(p->ev_rec[k], p->s_prod[0]));
    return ASR_OK;
}

// Split production, part 2: emission projection once the recurrence is done
// and the previous decode of this buffer has finished.
int produce_tail(asr_pipeline* p, long i) {
    const auto& c = p->cfg;
    const int k = (int)(i % p->nbuf);
    if (fault(p, i, "tail")) return ASR_ERR_INTERNAL;
    ASR_HIP_TRY(hipStreamWaitEvent(p->s_tail, p->ev_rec[k], 0));
    ASR_HIP_TRY(hipStreamWaitEvent(p->s_tail, p->ev_free[k], 0));
    int rc = asr_linear_fwd(p->hid[k], p->W_out, p->b_out, p->emis[k], c.T * c.B, c.H, c.V,
                            ASR_EPI_BIAS_LOGSOFTMAX, p->s_tail);
    if (rc) return rc;
    if (int r = mark(p, 1, k, p->s_tail)) return r;
    ASR_HIP_TRY(hipEventRecord(p->ev_ready[k], p->s_tail));
    return ASR_OK;
}

// Queue the held last decode segment of batch i: on its decode stream, or
// (drain) on its production stream behind that stream's productions, after
// the decode of its earlier segments.
int release_held(asr_pipeline* p, long i, bool drain) {
    const auto& c = p->cfg;
    const int k = (int)(i % p->nbuf);
    const int s = p->S - 1;
    const int t0 = seg_bound(p, s);
    hipStream_t st = drain ? p->s_prod[i % p->P] : p->s_dec[i % p->D];
    if (drain) ASR_HIP_TRY(hipStreamWaitEvent(st, p->ev_dpre[k], 0));
    ASR_HIP_TRY(hipStreamWaitEvent(st, p->ev_seg[(size_t)k * p->S + s], 0));
    int rc = asr_ctc_decode_segment(p->dec[k], p->emis[k] + (long)t0 * c.B * c.V, c.T, t0, c.T, c.B,
                                    (long)c.B * c.V, c.V, nullptr, 1, st);
    if (rc) return rc;
    if (int r = mark(p, 3, k, st)) return r;
    ASR_HIP_TRY(hipEventRecord(p->ev_free[k], st));
    return ASR_OK;
}

// Every held segment onto the production streams (the caller drains).
int release_all_held(asr_pipeline* p) {
    int rc = ASR_OK;
    while (!p->held.empty() && !rc) {
        const long h = p->held.front();
        p->held.pop_front();
        rc = release_held(p, h, true);
        if (rc) set_failed(p, h, rc);   // batch h was accepted: its results can never come
    }
    return rc;
}

int enqueue_decode(asr_pipeline* p, long i) {
    const auto& c = p->cfg;
    const int k = (int)(i % p->nbuf);
    hipStream_t sd = p->s_dec[i % p->D];
    if (fault(p, i, "decode")) return ASR_ERR_INTERNAL;
    int rc = ASR_OK;
    if (p->S > 1) {   // segment by segment, each behind its production
        const int ns = p->hold > 0 ? p->S - 1 : p->S;   // held: the last one is queued later
        for (int s = 0; s < ns && !rc; s++) {
            const int t0 = seg_bound(p, s), t1 = seg_bound(p, s + 1);
            ASR_HIP_TRY(hipStreamWaitEvent(sd, p->ev_seg[(size_t)k * p->S + s], 0));
            if (s == 0) if (int r = mark(p, 2, k, sd)) return r;
            rc = asr_ctc_decode_segment(p->dec[k], p->emis[k] + (long)t0 * c.B * c.V, c.T, t0, t1, c.B,
                                        (long)c.B * c.V, c.V, nullptr, 1, sd);
        }
        if (rc) return rc;
        if (ns < p->S) {
            ASR_HIP_TRY(hipEventRecord(p->ev_dpre[k], sd));
            p->held.push_back(i);
            p->decoded = i + 1;
            while ((int)p->held.size() > p->hold) {   // the steady state: on its own decode stream
                const long h = p->held.front();
                p->held.pop_front();
                if (int r = release_held(p, h, false)) return r;
            }
            return ASR_OK;
        }
    } else {
        ASR_HIP_TRY(hipStreamWaitEvent(sd, p->ev_ready[k], 0));
        if (int r = mark(p, 2, k, sd)) return r;
        rc = asr_ctc_decode(p->dec[k], p->emis[k], c.T, c.B, 1, sd);
    }
    if (rc) return rc;
    if (int r = mark(p, 3, k, sd)) return r;
    ASR_HIP_TRY(hipEventRecord(p->ev_free[k], sd));
    p->decoded = i + 1;
    return ASR_OK;
}

// Production groups (GROUPS2, H > 256: C5): the recurrence is T dependent
// step launches whose time hardly depends on B (latency-bound), so the
// recurrences of G consecutive batches run as one (asr_internal_rnn_recur_multi:
// one step launch for all of them per frame).  Part 1 at each submit: the
// batch's input projection, on its group's production stream.
int produce_group_head(asr_pipeline* p, long i, const float* x) {
    const auto& c = p->cfg;
    const int k = (int)(i % p->nbuf);
    if (fault(p, i, "produce")) return ASR_ERR_INTERNAL;
    hipStream_t sp = p->s_prod[(i / p->G) % p->P];
    ASR_HIP_TRY(hipStreamWaitEvent(sp, p->ev_free[k], 0));   // the decode reading this buffer is done
    if (int r = mark(p, 0, k, sp)) return r;
    return asr_linear_fwd(x, p->W_ih, nullptr, p->hid[k], c.T * c.B, c.in, c.H, ASR_EPI_NONE, sp);
}

// Part 2, once the group is complete (or a fetch needs a member): one
// recurrence over the group, each member's emission projection, its decode.
int flush_group(asr_pipeline* p) {
    if (p->group.empty()) return ASR_OK;
    const auto& c = p->cfg;
    std::vector<long> g;
    g.swap(p->group);
    hipStream_t sp = p->s_prod[(g[0] / p->G) % p->P];
    float* hids[4];
    for (size_t j = 0; j < g.size(); j++) hids[j] = p->hid[g[j] % p->nbuf];
    asr_internal_graph_now = 1;
    int rc = asr_internal_rnn_recur_multi(p->W_hh, p->b_ih, p->b_hh, hids, (int)g.size(), c.T, c.B, c.H, sp);
    asr_internal_graph_now = 0;
    for (size_t j = 0; j < g.size() && !rc; j++) {
        const int k = (int)(g[j] % p->nbuf);
        rc = asr_linear_fwd(p->hid[k], p->W_out, p->b_out, p->emis[k], c.T * c.B, c.H, c.V,
                            ASR_EPI_BIAS_LOGSOFTMAX, sp);
        if (!rc) rc = mark(p, 1, k, sp);
        if (!rc && hipEventRecord(p->ev_ready[k], sp) != hipSuccess) rc = ASR_ERR_HIP;
        if (!rc) rc = enqueue_decode(p, g[j]);
    }
    if (rc) set_failed(p, g[0], rc);   // the group's batches were accepted: no results can come
    return rc;
}

// Queue the emission GEMM and decode of the batch whose production was split.
int flush_tail(asr_pipeline* p) {
    if (p->pending_tail < 0) return ASR_OK;
    const long j = p->pending_tail;
    p->pending_tail = -1;
    static const bool trace = [] { const char* e = getenv("ASR_PIPELINE_TRACE"); return e && atoi(e); }();
    const auto t0 = std::chrono::steady_clock::now();
    int rc = produce_tail(p, j);
    const auto t1 = std::chrono::steady_clock::now();
    if (!rc) rc = enqueue_decode(p, j);
    if (rc) set_failed(p, j, rc);   // batch j was accepted: its results can never come
    if (trace) {
        const auto t2 = std::chrono::steady_clock::now();
        const double a = std::chrono::duration<double, std::milli>(t1 - t0).count();
        const double b = std::chrono::duration<double, std::milli>(t2 - t1).count();
        if (a + b > 0.5) fprintf(stderr, "asr_pipeline: batch %ld emission GEMM %.3f ms, decode enqueue %.3f ms\n", j, a, b);
    }
    return rc;
}

// Fetch the results of the oldest uncollected batch (blocking).
// ... straight into the caller's arrays (asr_ctc_get_best's layout): the
// host copies of a batch's results are on the critical path of small
// batches (C2: 0.6 ms per batch), so nothing is staged in between.
int fetch_to(asr_pipeline* p, int32_t* labels, int max_len, int32_t* lengths, double* logp, float* ms, long* batch,
             int* res_rc) {
    const long j = p->collected;
    if (j >= p->submitted) return ASR_ERR_STATE;
    if (p->fail_from >= 0 && j >= p->fail_from) return p->fail_rc;
    // Work held back for overlap (a split production's last emission GEMM +
    // decode, a production group still filling) is queued before the host
    // blocks on a batch within D of it: the caller is draining (no submit
    // comes while it waits), and held back it would start only when the
    // caller reaches it (C2, 20 steps: the last decode started 1.5 ms late,
    // 8 % of the job).  In steady state the caller fetches batches more than
    // D behind the newest, so nothing changes there.
    if (!p->held.empty() && j + p->D >= p->held.front()) {   // draining: held segments on the production CUs
        const int rc = release_all_held(p);
        if (rc && (p->fail_from >= 0 && j >= p->fail_from)) return rc;
    }
    const bool drain_tail = p->pending_tail >= 0 && j + p->D >= p->pending_tail;
    const bool drain_group = !p->group.empty() && j + p->D >= p->group.front();
    if (j >= p->decoded || drain_tail || drain_group) {
        // a failed flush fails the pipeline from the flushed batch on
        // (set_failed); batch j itself is returned normally when it was
        // already decoded (the header's promise for earlier batches)
        int rc = flush_tail(p);
        if (!rc) rc = flush_group(p);
        if (rc && (j >= p->decoded || (p->fail_from >= 0 && j >= p->fail_from))) return rc;
    }
    if (j >= p->decoded) return ASR_ERR_INTERNAL;   // never queued (cannot happen once flushed)
    asr_ctc_t* h = p->dec[j % p->nbuf];
    *res_rc = asr_ctc_get_best(h, labels, max_len, lengths, logp);
    if (*res_rc != ASR_OK && *res_rc != ASR_ERR_BEAM_OVERFLOW) return *res_rc;
    // (a one-launch H > 256 recurrence that gave up waiting for its
    // workgroups was finished by its recovery kernel before the emission
    // projection read it: asr_rnn_persist_stats counts those)
    if (ms) asr_ctc_last_kernel_ms(h, ms);
    if (p->timing && j >= p->timing_from) {   // the batch's stamps, all complete once its decode is
        const int k = (int)(j % p->nbuf);
        ASR_HIP_TRY(hipEventSynchronize(p->ev_t[3][k]));
        asr_pipeline::Stamp st{j, {0.f, 0.f, 0.f, 0.f}};
        for (int w = 0; w < 4; w++) ASR_HIP_TRY(hipEventElapsedTime(&st.t[w], p->ev_t0ref, p->ev_t[w][k]));
        p->timeline.push_back(st);
    }
    *batch = j;
    p->collected = j + 1;
    return ASR_OK;
}

// Fetch the results of the oldest uncollected batch into a stash entry (a
// submit that must reuse its buffer before the caller collected it).
int fetch(asr_pipeline* p, Result& r) {
    const auto& c = p->cfg;
    r.lab.assign((size_t)c.B * c.T, 0);
    r.len.assign(c.B, 0);
    r.lp.assign(c.B, 0.0);
    return fetch_to(p, r.lab.data(), c.T, r.len.data(), r.lp.data(), &r.ms, &r.batch, &r.rc);
}

void release(asr_pipeline* p) {
    for (auto s : p->s_dec) if (s) hipStreamSynchronize(s);
    for (auto s : p->s_prod) if (s) hipStreamSynchronize(s);
    if (p->s_gemm) hipStreamSynchronize(p->s_gemm);
    if (p->tail_own && p->s_tail) hipStreamSynchronize(p->s_tail);
    if (p->s_gdec) hipStreamSynchronize(p->s_gdec);
    for (auto h : p->dec) asr_ctc_destroy(h);
    for (auto b : p->hid) hipFree(b);
    for (auto b : p->emis) hipFree(b);
    for (auto b : p->hst) hipFree(b);
    for (auto b : p->stage) hipFree(b);
    for (auto e : p->ev_seg) if (e) hipEventDestroy(e);
    for (auto e : p->ev_dpre) if (e) hipEventDestroy(e);
    for (auto* v : {&p->ev_ready, &p->ev_free, &p->ev_proj, &p->ev_rec, &p->ev_t[0], &p->ev_t[1], &p->ev_t[2],
                    &p->ev_t[3]})
        for (auto e : *v) if (e) hipEventDestroy(e);
    if (p->ev_t0ref) hipEventDestroy(p->ev_t0ref);
    for (auto s : p->s_dec) if (s) hipStreamDestroy(s);
    for (auto s : p->s_prod) if (s) hipStreamDestroy(s);
    if (p->s_gemm) hipStreamDestroy(p->s_gemm);
    if (p->tail_own && p->s_tail) hipStreamDestroy(p->s_tail);
    if (p->s_gdec) hipStreamDestroy(p->s_gdec);
}

// Placement probe: every workgroup records the XCD (HW_REG_XCC_ID) and the
// shader engine / array / CU (HW_REG_HW_ID bits 15:8) its wave runs on, after
// a short spin so that the grid spreads over every CU the stream's mask
// allows.  Reads two hardware registers; nothing else.
constexpr int PROBE_BLOCKS = 8192;
__global__ __launch_bounds__(64) void placement_probe_kernel(uint32_t* out, long long spin) {
    // s_getreg immediates: id | offset << 6 | (size - 1) << 11
    const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (15 << 11));   // HW_REG_XCC_ID
    const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));     // HW_REG_HW_ID
    const long long t0 = clock64();
    while (clock64() - t0 < spin) __builtin_amdgcn_s_sleep(1);
    if (threadIdx.x == 0) out[blockIdx.x] = ((xcc & 0xFu) << 16) | ((hw >> 8) & 0xFFu);
}

}  // namespace

extern "C" {

int asr_pipeline_get_placement(asr_pipeline_t* p, int cap, int* n, int* role, int* cu_lo, int* cu_hi) {
    if (!p || !n || cap < 0 || (cap > 0 && (!role || !cu_lo || !cu_hi))) return ASR_ERR_ARG;
    *n = (int)p->placed.size();
    for (int i = 0; i < std::min(cap, *n); i++) {
        role[i] = p->placed[i].role;
        cu_lo[i] = p->placed[i].lo;
        cu_hi[i] = p->placed[i].hi;
    }
    return ASR_OK;
}

int asr_pipeline_probe_placement(asr_pipeline_t* p, int role, int* cus_per_xcc, int* n_xcc) {
    if (!p || !cus_per_xcc || !n_xcc) return ASR_ERR_ARG;
    hipStream_t st = nullptr;
    for (const auto& q : p->placed)
        if (q.role == role) { st = q.s; break; }
    if (!st) return ASR_ERR_ARG;
    for (int x = 0; x < ASR_MAX_XCC; x++) cus_per_xcc[x] = 0;
    *n_xcc = 0;
    uint32_t* d = nullptr;
    ASR_HIP_TRY(hipMalloc(&d, sizeof(uint32_t) * PROBE_BLOCKS));
    std::vector<uint32_t> h(PROBE_BLOCKS, 0xFFFFFFFFu);
    int rc = ASR_OK;
    if (hipMemsetAsync(d, 0xFF, sizeof(uint32_t) * PROBE_BLOCKS, st) != hipSuccess) rc = ASR_ERR_HIP;
    if (!rc) {
        hipLaunchKernelGGL(placement_probe_kernel, dim3(PROBE_BLOCKS), dim3(64), 0, st, d, 20000ll);
        if (hipGetLastError() != hipSuccess) rc = ASR_ERR_HIP;
    }
    if (!rc && hipMemcpyAsync(h.data(), d, sizeof(uint32_t) * PROBE_BLOCKS, hipMemcpyDeviceToHost, st) != hipSuccess)
        rc = ASR_ERR_HIP;
    if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = ASR_ERR_HIP;
    hipFree(d);
    if (rc) return rc;
    std::vector<char> seen((size_t)ASR_MAX_XCC * 256, 0);
    for (uint32_t v : h) {
        if (v == 0xFFFFFFFFu) return ASR_ERR_INTERNAL;   // a workgroup never wrote
        const uint32_t x = (v >> 16) & 0xFu, cu = v & 0xFFu;
        if (x >= (uint32_t)ASR_MAX_XCC) return ASR_ERR_INTERNAL;
        char& s = seen[(size_t)x * 256 + cu];
        if (!s) {
            s = 1;
            cus_per_xcc[x]++;
            *n_xcc = std::max(*n_xcc, (int)x + 1);
        }
    }
    return ASR_OK;
}

int asr_pipeline_create(const asr_pipeline_config* cfg, const float* W_ih, const float* W_hh,
                        const float* b_ih, const float* b_hh, const float* W_out, const float* b_out,
                        asr_pipeline_t** out) {
    if (!cfg || !out || !W_ih || !W_hh || !b_ih || !b_hh || !W_out || !b_out) return ASR_ERR_ARG;
    *out = nullptr;
    const auto& c = *cfg;
    if (c.T < 1 || c.B < 1 || c.in < 1 || c.H < 1 || c.V < 2 || c.beam < 1 || c.blank < 0 || c.blank >= c.V ||
        c.inflight < 0 || c.prod_streams < 0 || c.decode_cus < -1 || c.segments < 0)
        return ASR_ERR_ARG;
    asr_pipeline* p = new asr_pipeline();
    p->cfg = c;
    if (const char* f = getenv("ASR_PIPELINE_FAULT")) {   // test hook: "<batch>:<stage>"
        long b = -1;
        char st[8] = {0};
        if (sscanf(f, "%ld:%7s", &b, st) == 2) {
            p->fault_batch = b;
            std::memcpy(p->fault_stage, st, sizeof st);
        }
    }
    p->W_ih = W_ih; p->W_hh = W_hh; p->b_ih = b_ih; p->b_hh = b_hh; p->W_out = W_out; p->b_out = b_out;
    p->arith = asr::dense_arith();
    ArithGuard arith_guard(p->arith);
    int dev = 0;
    int rc = ASR_OK;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&p->ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || p->ncu < 8) {
        delete p;
        return ASR_ERR_HIP;
    }
    const int ncu = p->ncu;
    // the decoder's beam capacity (asr_ctc_create's automatic max_states)
    const int K = c.beam + 1;
    const int kcap = (K + std::max(8, K / 8) + 31) / 32 * 32;
    const int bcu = (c.B + 7) / 8 * 8;   // CUs at one decode workgroup per utterance
    int occw = 0;                          // one-wave decoder workgroups per CU (SHARED)
    // Batches of 64 utterances or more take the chip-filling schedule (many
    // one-wave decodes in flight on half of the CUs) even when one batch
    // would fit a quarter of the CUs at one 8-wave workgroup per utterance:
    // C2 (B = 64, T = 500), 20 steps / warmup 5: CU groups 51.8 M frames/s,
    // chip-filling 67.5 M (10 decodes in flight; 6 / 12 / 16: 45.5 / 68.6 /
    // 63.2 M; 192 decode CUs or 32 hardware queues: 20-48 M; runs sg, sh).
    // ASR_PIPELINE_MODE=0 keeps the CU groups (A/B).
    const char* fm = getenv("ASR_PIPELINE_MODE");
    const bool small_shared = c.B >= 64 && !(fm && atoi(fm) == 0);
    if (c.H <= 256 && c.V + 1 <= 64 && 4 * bcu <= ncu && !small_shared) {
        p->mode = GROUPS;
        p->gcu = bcu;
        p->D = c.inflight ? c.inflight : std::max(1, std::min(3, ncu / bcu - 1));
        p->P = 1;
        p->split = true;
    } else if (c.H <= 256 && c.V + 1 <= 64 && kcap <= 128 && (2 * bcu > ncu || small_shared) &&
               (occw = wave_occupancy(c)) > 0) {
        p->mode = SHARED;
        p->rnn_kind = ASR_RNN_RECUR_MFMA;
        // decodes and production on their own halves of the CUs (the
        // decode workgroups fill a CU's registers, the wide GEMM needs most
        // of its LDS), D batches decoding at once so that the decode CUs
        // hold 16 utterances each: the one-wave kernel's occupancy, where
        // it decodes fastest (measured, profiles/r03: 2048 per GPU 107 ->
        // 167 M frames/s, 1024 per GPU 94 -> 163 M).  Small batches need
        // many in flight (256 per GPU: 8), and as many production streams as
        // the recurrence's latency (T steps, whatever B) needs to keep up.
        const bool part = c.decode_cus != -1;
        // decode CUs: half of them, 3/8 for batches under 512 utterances,
        // whose production costs more CU time per frame (the input GEMM of a
        // short M; measured at 256 per GPU, 60 steps: 128 / 96 / 80 decode
        // CUs 137-142 / 155-162 / 145 M frames/s; at 512: 128 / 96 CUs
        // 183 / 168-182 M; profiles/r03/bench_scan.md).  Beam capacity
        // 65-128 (C3's beam 100: two rows per lane): an utterance-frame costs
        // the decoder more CU time, so half of them decode at any batch size
        // (C3, B = 256, 20 steps: 96 / 112 / 128 / 144 / 160 / 176 / 192
        // decode CUs 59.5 / 72.5 / 88.3 / 79.4 / 77.1 / 57.2 / 61.1 M frames/s,
        // profiles/r04/bench_scan.md).
        // On the split-bf16 arithmetic (dense_x3.hip) production costs ~half
        // the CU time, and half of the CUs decode at every batch size (256
        // per GPU, GSPLIT 0: 96 / 112 / 128 decode CUs 162 / 188 / 186 M
        // frames/s; C4: 120 / 128 / 144 / 160 decode CUs 271 / 325 / 271 /
        // 269 M, a sharp optimum at half; profiles/r04/bench_scan.md).
        const bool x3 = asr::dense_x3_on();
        const int dauto = (kcap > 64 || x3 ? ncu / 2 : (c.B < 512 ? ncu * 3 / 8 : ncu / 2)) / 8 * 8;
        p->dcus = part ? (c.decode_cus > 0 ? std::min(c.decode_cus, ncu - 8) : dauto) : 0;
        const int dc = p->dcus ? p->dcus : ncu;
        // as many batches decoding at once as fill the decode CUs at the
        // one-wave kernel's occupancy (16 per CU at beam <= 56, ~9 at 100)
        const int Dw = std::max(1, std::min(8, (occw * dc + c.B / 2) / c.B));
        // On the split-bf16 production (beam <= 56) two more decodes are
        // queued than the decode CUs hold: their workgroups start in the CUs
        // the oldest decodes' last utterances free, instead of after the host
        // queues them (20 / 5, decodes in flight Dw / Dw + 1 / Dw + 2: C4 as
        // two 1024 batches 293.4 / 320.6 / 330.2 M frames/s, 1024 per GPU
        // 270.0 / 304.4 / 300.3 M, 512 242.4 / 259.5 / 255.9 M, 256 188.3 /
        // 196.6 / 210.3 M; profiles/r04/bench_scan.md)
        // With four T-segments per batch (512-1023 utterances, below) three
        // (512 per GPU, 20 / 5, 6 / 7 / 8 decodes: 267.7-268.0 / 281.5-289.6
        // / 278.1 M; 1024 and C4 at 2 segments: 4 / 5 decodes 310.2 / 305.5
        // and 334.0-334.5 / 329.7-332.8 M; 256: 10 / 11 / 12 decodes 207.3 /
        // 199.2 / 153.3 M; run c4d)
        const int Sw = c.segments ? c.segments : auto_segments(c, kcap);
        p->D = c.inflight ? c.inflight : (x3 && kcap <= 64 ? std::min(10, Dw + (Sw >= 4 ? 3 : 2)) : Dw);
        // production streams: the recurrence of a batch is latency-bound
        // (T steps) on B / 16 CUs, so as many batches produce at once as
        // decode at once (small shards: 256 per GPU, D = 8 -> P = 8)
        p->P = c.prod_streams ? c.prod_streams : (part ? std::max(3, p->D) : 1);
        // the fused recurrence + emission kernel, and the decode CUs' share
        // of the input projection rows (ASR_PIPELINE_GSPLIT: a fraction of
        // the rows, A/B)
        p->fuse = (c.H & 15) == 0 && c.V <= 32;
        if (p->fuse && p->dcus) {
            const char* ge = getenv("ASR_PIPELINE_GSPLIT");
            // default 0.3 (measured, C4 one GPU: 0 / 0.2 / 0.3 / 0.4 / 0.5 ->
            // 176 / 198 / 202 / 196 / 191 M frames/s).  With several decodes
            // in flight the rows run on the tiled GEMM kernel (below): with
            // the persistent one a decode launched meanwhile waited for its
            // CUs (1024 per GPU: 171 vs 180 M at 0.3 / 0), with the tiled one
            // 0 / 0.2 / 0.3 -> 173 / 196 / 198 M, 512 per GPU 167 / 182 / 182 M
            // (profiles/r03/bench_scan.md)
            // two rows per lane: the decode CUs are the busier half, no share (A/B).
            // Split-bf16 arithmetic: none either — its GEMM workgroups take a
            // whole CU (2 waves per SIMD at ~240 VGPRs), so a share on the
            // decode CUs holds decodes back (256 / 512 / 1024 per GPU at 0.3 vs
            // 0: 103 / 181 / 205 vs 162 / 242 / 269 M frames/s; 2048: 233 vs
            // 236 M, 240 M at 0.1)
            const double f = ge ? atof(ge) : (kcap > 64 || x3 ? 0.0 : 0.3);
            p->grows = (long)(std::max(0.0, std::min(1.0, f)) * c.T * c.B) / 128 * 128;
            p->gtiled = p->D > 1 ? 8 : 0;
        }
    } else if (4 * bcu <= ncu) {   // small batches otherwise (C5: H = 1024, V = 1000)
        p->mode = GROUPS2;
        p->gcu = bcu;
        // production groups: G batches' recurrences as one (H > 256, the
        // per-frame step launches; rows in whole 16-row tiles), D = 2G.
        // Default 1 (ASR_PIPELINE_GROUP=n selects n): measured at C5, a
        // 64-row step beside the production GEMMs costs 2.1x a 32-row one
        // (14.9 vs 6.9 us), so groups of 2 / 3 ran 1.77 / 1.45 M frames/s
        // against 3.37 M (profiles/r04/bench_scan.md).
        const char* ge = getenv("ASR_PIPELINE_GROUP");
        const int Gw = ge ? atoi(ge) : 1;
        p->G = (c.H > 256 && (c.H % 128) == 0 && (c.B % 16) == 0) ? std::max(1, std::min(4, Gw)) : 1;
        p->D = c.inflight ? c.inflight : std::max(1, std::min(2 * p->G, ncu / bcu - 1));
        p->P = c.prod_streams ? c.prod_streams : (c.H > 256 ? 2 : 1);
        // With the one-launch recurrence (H > 256, asr::rnn_recur_persist_launch)
        // production holds its CUs for ~5 us a frame instead of ~14 beside
        // the GEMMs, so three decodes run at once where each production
        // stream keeps the recurrence's workgroups (C5, 10 / 3 steps: D = 2 /
        // 3 / 4 3.45 / 4.24 / 4.27 M frames/s; P = 3 leaves too few CUs per
        // stream and falls back to the per-frame steps: 1.7-2.1 M; run sv).
        if (!c.inflight && p->G == 1 && c.H > 256 && (c.H % 128) == 0 && c.H >= 384 && c.H <= 1024 &&
            c.B <= 256) {
            const int nwg = (c.H / 32) * ((c.B + 15) / 16);
            if ((ncu - 3 * bcu) / std::max(1, p->P) >= nwg && 4 * bcu <= ncu) p->D = 3;
        }
    } else {   // chip-filling batches otherwise (C3's beam 100, BL's H = 2048): one decode at a time
        p->mode = SHARED;
        p->dcus = c.decode_cus > 0 ? std::min(c.decode_cus, ncu - 8) : 0;
        p->D = c.inflight ? c.inflight : 1;
        // two productions in flight beside the decode; for H <= 256 the
        // MFMA recurrence (B / 16 CUs, its workgroups fit beside the decode's
        // instead of one 1024-thread workgroup per utterance on every CU)
        // with the emission layer fused when V <= 32
        p->P = c.prod_streams ? c.prod_streams : 2;
        if (c.H <= 256 && (c.H & 15) == 0) {
            p->rnn_kind = ASR_RNN_RECUR_MFMA;
            p->fuse = c.V <= 32;
        }
    }
    // T-segments (fused production only): explicit (config.segments), else 2 for small shards (under 512 utterances: the job's fill
    // and drain are a large part of it; measured at 256 per GPU, 20 steps:
    // 1 / 2 / 4 segments 132.5 / 136.4 / 134.7 M frames/s), 1 otherwise
    // (2048 per GPU: 206.7 vs 201.6 M at 2; profiles/r04/bench_scan.md)
    // On the split-bf16 production, 2 at every batch size (20 / 5, 1 / 2
    // segments: C4 as two 1024 batches 330.8 / 335.0 M frames/s, 1024 per GPU
    // 301.3 / 316.4 M, 512 256.4 / 259.0 M (268.9 at 4), 256 196.8 / 211.3 M
    // (202.8 at 4): with decodes queued behind the resident ones a segment
    // boundary no longer idles the decode CUs, and the last batch's decode
    // starts T/2 recurrence steps earlier); 4 for 512-1023 utterances
    // (run c4s: 512 per GPU 264.2 / 271.6 M at 2 / 4; 1024 312.6 / 315.3 M
    // and C4 332.6 / 323.3 M, within or below the noise; 256 211.3 / 202.8).
    if (p->fuse && p->mode == SHARED) {
        const int S = c.segments ? c.segments : auto_segments(c, kcap);
        p->S = std::max(1, std::min(S, c.T));
    }
    // H > 256 small batches with the wide decoder (C5): the production hands
    // the decode two T-segments (the first decode starts after half of the
    // first production, the last batch's drain is half a decode)
    if (p->mode == GROUPS2 && p->G == 1 && c.V + 1 > 64 && c.V <= 4096) {
        const int S = c.segments ? c.segments : 2;
        p->S = std::max(1, std::min(S, c.T / 2));
    }
    // fragment-major P between the input projection and the split-bf16 fused
    // recurrence (measured against row-major P: production ~2-3 % shorter,
    // the same emission bits; run se)
    p->pfrag = p->fuse && asr::dense_x3_on() && asr::rnn_x3_applies(c.B, c.H) && (c.B % 16) == 0 &&
               c.in <= 256 && (c.in % 4) == 0;
    // HIP maps the process's UNMASKED streams round-robin onto
    // GPU_MAX_HW_QUEUES hardware queues (default 4, read when the runtime
    // starts), and streams that share a queue run one after another (C5, 5
    // streams on 4 queues: 1.03 M vs 3.48 M frames/s).  A CU-masked stream
    // (hipExtStreamCreateWithCUMask) gets a hardware queue of its own — the
    // mask is a property of the queue — so only the unmasked streams count
    // against the variable (measured round 6, run r6b, 20 / 5 steps, at
    // GPU_MAX_HW_QUEUES=4 with the 24-queue schedule kept: C4 365.3 M, 256
    // per GPU 224.6 M, C2 63.9 M frames/s, the same as at 24 queues, where
    // round 5's fit of every stream to 4 queues gave 310.7 / 97.8 / 22.1 M).
    // Fit the automatic schedule so that the unmasked streams fit the
    // queues: no decode-CU share of the input projection first, then fewer
    // production streams and decodes in flight, the larger count first;
    // explicit counts are kept as given.  asr_pipeline_get_streams /
    // asr_pipeline_get_queue_use report the outcome.
    {
        const char* q = getenv("GPU_MAX_HW_QUEUES");
        p->hw_queues = (q && atoi(q) > 0) ? atoi(q) : 4;
        auto nstreams = [&] { return p->D + p->P + (p->grows > 0 ? 1 : 0) + (p->split ? 1 : 0); };
        // streams created without a CU mask (the layout below)
        auto unmasked = [&] {
            if (p->mode == SHARED) return p->dcus > 0 ? 0 : p->D + p->P + (p->grows > 0 ? 1 : 0);
            const bool masked = p->gcu > 0 && !(p->mode == GROUPS2 && p->D == 1);
            return (masked ? 0 : p->D + p->P) + (p->split ? 1 : 0);
        };
        if (unmasked() > p->hw_queues && p->grows > 0) p->grows = 0;
        // then production streams down to half the decodes in flight, then
        // both (small batches need both: C2 at 8 queues as D = 7, P = 1 ran
        // 16.4 M frames/s, at D = P = 4 38.7 M; at 16 queues D = 10, P = 6
        // 61.3 M against D = P = 8 53.9 M; runs sn, sn2)
        while (unmasked() > p->hw_queues) {
            const bool canP = !c.prod_streams && p->P > 1, canD = !c.inflight && p->D > 1;
            if (canP && (!canD || p->P > (p->D + 1) / 2)) p->P--;
            else if (canD) p->D--;
            else break;
        }
        p->tail_own = p->split && unmasked() < p->hw_queues;
        p->streams = nstreams() + (p->tail_own ? 1 : 0);
        p->shared_queue_streams = unmasked() + (p->tail_own ? 1 : 0);
    }
    // drain hold (S > 1; A/B: ASR_PIPELINE_DRAIN=W held batches, -1: P - 1)
    // and the first segment's share of T (ASR_PIPELINE_SEG0, S = 2)
    if (p->S > 1) {
        const char* de = getenv("ASR_PIPELINE_DRAIN");
        const int w = de ? atoi(de) : 0;
        p->hold = std::max(0, w < 0 ? p->P - 1 : std::min(w, p->P - 1));
        if (const char* f0 = getenv("ASR_PIPELINE_SEG0")) p->seg0 = std::max(0.0, std::min(0.95, atof(f0)));
    }
    // CU groups (GROUPS / GROUPS2), from the decode count the queue fit left:
    // decode d runs on group d % ngroups, so an explicit inflight beyond the
    // groups queues decodes behind a group's current one.  Not the default:
    // one or two queued decodes measured slower here (C2 50.8 -> 42.5 / 47.4 M
    // frames/s, C5 3.37 -> 1.54 / 1.39 M; profiles/r04/bench_scan.md), unlike
    // the chip-filling mode.  One decode in flight (GROUPS2) runs on every CU.
    if (p->mode == GROUPS2 && p->D == 1) p->gcu = 0;
    if (p->mode != SHARED && p->gcu) p->ngroups = std::max(1, std::min(p->D, ncu / p->gcu - 1));
    if (p->mode != SHARED && p->D > 1 && (p->ngroups + 1) * p->gcu > ncu) { delete p; return ASR_ERR_UNSUPPORTED; }
    // D decoding + P producing (+1: split production queues the next input
    // projection before the previous batch's emission projection)
    p->nbuf = p->D + p->P + (p->split ? 1 : 0);
    if (p->G > 1) p->nbuf = p->D + (p->P + 1) * p->G;   // P groups producing, one filling, D decoding
    if (p->nbuf < 2) p->nbuf = 2;
    // streams
    auto mkr = [&](int role, hipStream_t* s, int lo, int hi) {
        if (rc) return rc;
        rc = cu_stream(s, ncu, lo, hi);
        if (!rc) p->placed.push_back({role, std::max(0, lo), std::min(ncu, hi), *s});
        return rc;
    };
    p->s_dec.assign(p->D, nullptr);
    p->s_prod.assign(p->P, nullptr);
    if (p->mode == SHARED) {
        // every decode on all of the decode CUs (decode d on its own 1/D of
        // them, several rounds of utterances per CU: 206.7 -> 196.9 M frames/s
        // at C4, D = 2, profiles/r04/bench_scan.md)
        for (int d = 0; d < p->D; d++) mkr(ASR_PIPE_ROLE_DECODE, &p->s_dec[d], 0, p->dcus ? p->dcus : ncu);
        for (int q = 0; q < p->P; q++) mkr(ASR_PIPE_ROLE_PRODUCTION, &p->s_prod[q], p->dcus, ncu);
        p->pcus = (ncu - p->dcus) / std::max(1, p->P);
        if (p->grows > 0) mkr(ASR_PIPE_ROLE_DECODE_CU_GEMM, &p->s_gdec, 0, p->dcus);
    } else {
        for (int d = 0; d < p->D; d++)
            mkr(ASR_PIPE_ROLE_DECODE, &p->s_dec[d], p->gcu ? (d % p->ngroups) * p->gcu : 0,
                p->gcu ? (d % p->ngroups + 1) * p->gcu : ncu);
        for (int q = 0; q < p->P; q++) mkr(ASR_PIPE_ROLE_PRODUCTION, &p->s_prod[q], p->gcu ? p->ngroups * p->gcu : 0, ncu);
        // each production stream's share of its CUs, for a recurrence whose
        // workgroups must all be resident at once (P of them may run together)
        p->pcus = (ncu - (p->gcu ? p->ngroups * p->gcu : 0)) / std::max(1, p->P);
        if (p->split) mkr(ASR_PIPE_ROLE_GEMM, &p->s_gemm, 0, ncu);   // the GEMMs on every CU
        if (p->tail_own) mkr(ASR_PIPE_ROLE_GEMM, &p->s_tail, 0, ncu);
        else p->s_tail = p->s_gemm;
    }
    // buffers, decoders, events
    const size_t nh = (size_t)c.T * c.B * c.H, ne = (size_t)c.T * c.B * c.V;
    for (int k = 0; k < p->nbuf && !rc; k++) {
        float *hb = nullptr, *eb = nullptr;
        if (hipMalloc(&hb, nh * sizeof(float)) != hipSuccess) rc = ASR_ERR_OOM;
        p->hid.push_back(hb);
        if (!rc && hipMalloc(&eb, ne * sizeof(float)) != hipSuccess) rc = ASR_ERR_OOM;
        p->emis.push_back(eb);
        asr_ctc_t* h = nullptr;
        if (!rc) rc = asr_ctc_create(nullptr, c.V, c.beam, c.blank, 0, &h);
        p->dec.push_back(h);
        if (p->S > 1) {
            float* hs = nullptr;
            if (!rc && hipMalloc(&hs, sizeof(float) * (size_t)c.B * c.H) != hipSuccess) rc = ASR_ERR_OOM;
            p->hst.push_back(hs);
            for (int s = 0; s < p->S; s++) {
                hipEvent_t e = nullptr;
                if (!rc && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) rc = ASR_ERR_HIP;
                p->ev_seg.push_back(e);
            }
            hipEvent_t e = nullptr;
            if (!rc && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) rc = ASR_ERR_HIP;
            p->ev_dpre.push_back(e);
        }
        // the decoders' schedule (asr_ctc_set_concurrency): D batches share the
        // decode CUs, which are dcus of the ncu the decoder plans for
        const int conc = p->mode == SHARED ? (p->D * ncu + (p->dcus ? p->dcus : ncu) - 1) / (p->dcus ? p->dcus : ncu) : 1;
        if (!rc && conc > 1) rc = asr_ctc_set_concurrency(h, conc);
        // chip-filling batches: many utterances per decode CU, the one-wave kernel
        if (!rc && p->mode == SHARED && occw > 0) rc = asr_ctc_set_waves(h, ASR_CTC_WAVES_LIST);
        // segmented unfused production with the wide decoder (C5): the
        // first-tile precompute runs on the production stream (A/B:
        // ASR_PIPELINE_TILE0_PROD=0 leaves it ahead of each decode launch)
        if (!rc && k == 0 && p->S > 1 && !p->fuse && c.V + 1 > 64) {
            const char* te = getenv("ASR_PIPELINE_TILE0_PROD");
            p->tile0_prod = !(te && te[0] == '0');
        }
        if (!rc && p->tile0_prod) {
            const int r = asr_internal_ctc_tile0_external(h, c.B, c.T);
            if (r == ASR_ERR_UNSUPPORTED && k == 0) p->tile0_prod = false;   // no precompute for this V
            else if (r) rc = r;
        }
        for (auto* v : {&p->ev_ready, &p->ev_free, &p->ev_proj, &p->ev_rec}) {
            hipEvent_t e = nullptr;
            if (!rc && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) rc = ASR_ERR_HIP;
            v->push_back(e);
        }
    }
    if (rc) {
        release(p);
        delete p;
        return rc;
    }
    *out = p;
    return ASR_OK;
}

}  // extern "C"

namespace {

int submit_batch(asr_pipeline* p, const float* x) {
    if (p->fail_rc) return p->fail_rc;
    const long i = p->submitted;
    // buffer i % nbuf is reused: its previous batch's results must be fetched first
    while (i - p->collected >= p->nbuf) {
        Result r;
        int rc = fetch(p, r);
        if (rc) return rc;
        p->stash.push_back(std::move(r));
    }
    // ASR_PIPELINE_TRACE=1: host time of each submit step over 0.5 ms (diagnostic)
    static const bool trace = [] { const char* e = getenv("ASR_PIPELINE_TRACE"); return e && atoi(e); }();
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    auto lap = [&](const char* what, clk::time_point& last) {
        const auto now = clk::now();
        const double ms = std::chrono::duration<double, std::milli>(now - last).count();
        if (ms > 0.5) fprintf(stderr, "asr_pipeline: batch %ld %s %.3f ms\n", i, what, ms);
        last = now;
    };
    auto last = t0;
    // A batch is accepted (counted as submitted) only once its production is
    // queued; a failure before that returns the error and leaves the
    // pipeline as it was (buffer i % nbuf is free: nothing else reads it).
    // A failure in the rest of an accepted batch's work fails the pipeline
    // from that batch on (set_failed): its results cannot come back.
    int rc;
    if (p->split) {
        rc = produce_head(p, i, x);
        if (trace) lap("head", last);
        if (rc) return rc;
        p->submitted = i + 1;
        rc = flush_tail(p);   // the previous batch: emission GEMM after this batch's input GEMM
        if (trace) lap("tail+decode", last);
        p->pending_tail = i;
    } else if (p->G > 1) {
        rc = produce_group_head(p, i, x);
        if (trace) lap("group head", last);
        if (rc) return rc;
        p->submitted = i + 1;
        p->group.push_back(i);
        if ((int)p->group.size() == p->G) rc = flush_group(p);
        if (trace) lap("group", last);
    } else {
        rc = p->fuse ? produce_fused(p, i, x) : produce_full(p, i, x);
        if (trace) lap("produce", last);
        if (rc) return rc;
        p->submitted = i + 1;
        rc = enqueue_decode(p, i);
        if (rc) set_failed(p, i, rc);
        if (trace) lap("decode", last);
    }
    return rc;
}

// Dynamic batching: the caller's batch goes into columns [j Bo, (j + 1) Bo)
// of the pipeline batch being assembled (a strided copy on the production
// stream that batch will run on); the cg-th submit queues the pipeline batch.
int submit_coalesced(asr_pipeline* p, const float* x) {
    if (p->fail_rc) return p->fail_rc;
    const auto& c = p->cfg;
    const long q = p->submitted;   // the pipeline batch being assembled
    const long ns = (long)p->stage.size();
    if (p->cfill == 0)   // stage q % ns was read by pipeline batch q - ns: fetched (stashed) first
        while (q - ns >= p->collected) {
            Result r;
            if (int rc = fetch(p, r)) return rc;
            p->stash.push_back(std::move(r));
        }
    const int j = p->cfill;
    const size_t row = sizeof(float) * (size_t)p->Bo * c.in;
    ASR_HIP_TRY(hipMemcpy2DAsync(p->stage[q % ns] + (size_t)j * p->Bo * c.in, sizeof(float) * (size_t)c.B * c.in, x,
                                 row, row, c.T, hipMemcpyDeviceToDevice, p->s_prod[q % p->P]));
    p->opend.emplace_back(q, j);
    if (++p->cfill < p->cg) return ASR_OK;
    p->cfill = 0;
    const int rc = submit_batch(p, p->stage[q % ns]);
    if (rc && p->submitted == q) {   // not accepted: this submit may come again
        p->opend.pop_back();
        p->cfill = p->cg - 1;
    }
    return rc;
}

// The results of pipeline batch q: a partial batch (the caller collects
// before cg submits) is completed with zero features, whose rows are decoded
// and dropped.
int coalesced_result(asr_pipeline* p, long q) {
    if (p->ocache_q == q) return ASR_OK;
    const auto& c = p->cfg;
    if (q >= p->submitted) {
        float* st = p->stage[q % (long)p->stage.size()];
        const int have = p->cfill;
        ASR_HIP_TRY(hipMemset2DAsync(st + (size_t)have * p->Bo * c.in, sizeof(float) * (size_t)c.B * c.in, 0,
                                     sizeof(float) * (size_t)(p->cg - have) * p->Bo * c.in, c.T, p->s_prod[q % p->P]));
        p->cfill = 0;
        if (int rc = submit_batch(p, st)) return rc;
    }
    Result r;
    if (!p->stash.empty()) {
        r = std::move(p->stash.front());
        p->stash.pop_front();
    } else if (int rc = fetch(p, r)) {
        return rc;
    }
    p->ocache = std::move(r);
    p->ocache_q = q;
    return ASR_OK;
}

int collect_coalesced(asr_pipeline* p, int32_t* labels, int max_len, int32_t* lengths, double* logp,
                      float* decode_ms) {
    if (p->opend.empty()) return ASR_ERR_STATE;
    const long q = p->opend.front().first;
    const int col = p->opend.front().second;
    if (int rc = coalesced_result(p, q)) return rc;
    const auto& c = p->cfg;
    const Result& r = p->ocache;
    const int b0 = col * p->Bo;
    for (int b = 0; b < p->Bo; b++) {
        const int len = r.len[b0 + b];
        if (lengths) lengths[b] = len;
        if (logp) logp[b] = r.lp[b0 + b];
        if (labels) {
            const int n = std::min(len, max_len);
            std::memcpy(labels + (size_t)b * max_len, r.lab.data() + (size_t)(b0 + b) * c.T, sizeof(int32_t) * n);
        }
    }
    if (decode_ms) *decode_ms = r.ms;
    p->returned = r.batch;
    p->ocol = col;
    p->opend.pop_front();
    return r.rc;
}

}  // namespace

extern "C" {

int asr_pipeline_submit(asr_pipeline_t* p, const float* x) {
    if (!p || !x) return ASR_ERR_ARG;
    ArithGuard arith_guard(p->arith);
    return p->cg > 1 ? submit_coalesced(p, x) : submit_batch(p, x);
}

int asr_pipeline_collect(asr_pipeline_t* p, int32_t* labels, int max_len, int32_t* lengths, double* logp,
                         float* decode_ms) {
    if (!p || (!labels && max_len > 0)) return ASR_ERR_ARG;
    ArithGuard arith_guard(p->arith);   // a drain may queue held-back production
    if (p->cg > 1) return collect_coalesced(p, labels, max_len, lengths, logp, decode_ms);
    if (p->stash.empty()) {   // the common case: straight into the caller's arrays
        long batch = -1;
        int res = ASR_OK;
        const int rc = fetch_to(p, labels, max_len, lengths, logp, decode_ms, &batch, &res);
        if (rc) return rc;
        p->returned = batch;
        return res;
    }
    Result r = std::move(p->stash.front());
    p->stash.pop_front();
    const auto& c = p->cfg;
    for (int b = 0; b < c.B; b++) {
        const int len = r.len[b];
        if (lengths) lengths[b] = len;
        if (logp) logp[b] = r.lp[b];
        if (labels) {
            const int n = std::min(len, max_len);
            std::memcpy(labels + (size_t)b * max_len, r.lab.data() + (size_t)b * c.T, sizeof(int32_t) * n);
        }
    }
    if (decode_ms) *decode_ms = r.ms;
    p->returned = r.batch;
    return r.rc;
}

int asr_pipeline_peek_emissions(asr_pipeline_t* p, const float** d_emis) {
    if (!p || !d_emis) return ASR_ERR_ARG;
    *d_emis = nullptr;
    // its buffer is rewritten by the production of batch returned + nbuf
    if (p->returned < 0 || p->submitted - p->returned > p->nbuf) return ASR_ERR_STATE;
    *d_emis = p->emis[p->returned % p->nbuf];
    return ASR_OK;
}

int asr_pipeline_create_coalesced(const asr_pipeline_config* cfg, int group, const float* W_ih, const float* W_hh,
                                  const float* b_ih, const float* b_hh, const float* W_out, const float* b_out,
                                  asr_pipeline_t** out) {
    if (!cfg || !out || group < 1 || cfg->B < 1 || (long)cfg->B * group > (1L << 20)) return ASR_ERR_ARG;
    if (group == 1) return asr_pipeline_create(cfg, W_ih, W_hh, b_ih, b_hh, W_out, b_out, out);
    asr_pipeline_config c = *cfg;
    c.B = cfg->B * group;
    if (int rc = asr_pipeline_create(&c, W_ih, W_hh, b_ih, b_hh, W_out, b_out, out)) return rc;
    asr_pipeline* p = *out;
    // the caller's features are copied onto the production stream that reads
    // them: schedules whose input projection runs elsewhere are not coalesced;
    // nor are the unfused productions, whose kernels are chosen by the batch
    // shape (the fused one's bits do not depend on it)
    if (p->split || p->G > 1 || p->grows > 0 || !p->fuse || p->mode != SHARED) {
        asr_pipeline_destroy(p);
        *out = nullptr;
        return ASR_ERR_UNSUPPORTED;
    }
    p->cg = group;
    p->Bo = cfg->B;
    for (int k = 0; k <= p->nbuf; k++) {
        float* b = nullptr;
        if (hipMalloc(&b, sizeof(float) * (size_t)c.T * c.B * c.in) != hipSuccess) {
            asr_pipeline_destroy(p);
            *out = nullptr;
            return ASR_ERR_OOM;
        }
        p->stage.push_back(b);
    }
    return ASR_OK;
}

int asr_pipeline_get_coalesce(asr_pipeline_t* p, int* group, int* batch, int* column) {
    if (!p) return ASR_ERR_ARG;
    if (group) *group = p->cg;
    if (batch) *batch = p->cg > 1 ? p->Bo : p->cfg.B;
    if (column) *column = p->cg > 1 ? p->ocol : 0;
    return ASR_OK;
}

int asr_pipeline_pending(asr_pipeline_t* p, int* n) {
    if (!p || !n) return ASR_ERR_ARG;
    *n = p->cg > 1 ? (int)p->opend.size() : (int)(p->submitted - p->collected);
    return ASR_OK;
}

int asr_pipeline_describe(asr_pipeline_t* p, int* mode, int* inflight, int* prod_streams, int* decode_cus,
                          int* decode_waves) {
    if (!p) return ASR_ERR_ARG;
    if (decode_waves) {   // the schedule of the last decode (before any: that of this batch size)
        const asr_ctc_t* last = p->dec[p->decoded > 0 ? (p->decoded - 1) % p->nbuf : 0];
        int w = 0;
        const int rc = asr_ctc_get_config(const_cast<asr_ctc_t*>(last), nullptr, &w, nullptr);
        if (rc) return rc;
        *decode_waves = w;
    }
    if (mode) *mode = p->mode;
    if (inflight) *inflight = p->D;
    if (prod_streams) *prod_streams = p->P;
    if (decode_cus) *decode_cus = p->mode == SHARED ? (p->dcus ? p->dcus : p->ncu) : (p->gcu ? p->gcu : p->ncu);
    return ASR_OK;
}

int asr_pipeline_get_production(asr_pipeline_t* p, int* fused, long long* decode_cu_rows, int* recurrence) {
    if (!p) return ASR_ERR_ARG;
    if (fused) *fused = p->fuse ? 1 : 0;
    if (decode_cu_rows) *decode_cu_rows = p->fuse ? p->grows : 0;
    if (recurrence) *recurrence = p->rnn_kind >= 0 ? p->rnn_kind : ASR_RNN_RECUR_AUTO;
    return ASR_OK;
}

int asr_pipeline_get_groups(asr_pipeline_t* p, int* group) {
    if (!p || !group) return ASR_ERR_ARG;
    *group = p->G;
    return ASR_OK;
}

int asr_pipeline_get_segments(asr_pipeline_t* p, int* segments) {
    if (!p || !segments) return ASR_ERR_ARG;
    *segments = p->S;
    return ASR_OK;
}

int asr_pipeline_get_queue_use(asr_pipeline_t* p, int* shared_queue_streams, int* dedicated_queue_streams) {
    if (!p) return ASR_ERR_ARG;
    if (shared_queue_streams) *shared_queue_streams = p->shared_queue_streams;
    if (dedicated_queue_streams) *dedicated_queue_streams = p->streams - p->shared_queue_streams;
    return ASR_OK;
}

int asr_pipeline_get_drain(asr_pipeline_t* p, int* held_batches, double* first_segment_share) {
    if (!p) return ASR_ERR_ARG;
    if (held_batches) *held_batches = p->hold;
    if (first_segment_share) *first_segment_share = p->S > 1 ? (double)seg_bound(p, 1) / p->cfg.T : 1.0;
    return ASR_OK;
}

int asr_pipeline_get_streams(asr_pipeline_t* p, int* streams, int* hw_queues) {
    if (!p) return ASR_ERR_ARG;
    if (streams) *streams = p->streams;
    if (hw_queues) *hw_queues = p->hw_queues;
    return ASR_OK;
}

int asr_pipeline_set_timing(asr_pipeline_t* p, int on) {
    if (!p) return ASR_ERR_ARG;
    if (on && p->ev_t[0].empty()) {
        for (int w = 0; w < 4; w++) {
            p->ev_t[w].assign(p->nbuf, nullptr);
            for (auto& e : p->ev_t[w]) ASR_HIP_TRY(hipEventCreate(&e));
        }
        ASR_HIP_TRY(hipEventCreate(&p->ev_t0ref));
    }
    p->timeline.clear();
    p->timing = on != 0;
    p->timing_from = p->submitted;
    if (on) {   // the reference: now, on an idle device (the caller drained the pipeline)
        ASR_HIP_TRY(hipDeviceSynchronize());
        ASR_HIP_TRY(hipEventRecord(p->ev_t0ref, p->s_dec[0]));
        ASR_HIP_TRY(hipEventSynchronize(p->ev_t0ref));
    }
    return ASR_OK;
}

int asr_pipeline_get_timeline(asr_pipeline_t* p, int cap, int* n, long long* batch, float* t) {
    if (!p || !n || cap < 0 || (cap > 0 && (!batch || !t))) return ASR_ERR_ARG;
    *n = (int)p->timeline.size();
    for (int i = 0; i < std::min(cap, *n); i++) {
        batch[i] = p->timeline[i].batch;
        for (int w = 0; w < 4; w++) t[4 * i + w] = p->timeline[i].t[w];
    }
    return ASR_OK;
}

int asr_pipeline_destroy(asr_pipeline_t* p) {
    if (!p) return ASR_OK;
    release(p);
    delete p;
    return ASR_OK;
}

}  // extern "C"
