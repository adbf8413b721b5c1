/*
 * asr_amd.h — C ABI of libasr_amd.so, the MI355X (gfx950) RNN + CTC
 * beam-search decode path.
 *
 * This is the drop-in boundary.  The reference (jrxk/GPU-Accelerated-Speech-
 * Recognition, mounted at /root/reference) is C++/CUDA with no FFI of its own;
 * its callers (main.cpp, nn_test.cpp) use the C++ classes cuMatrix / Linear /
 * RNN / RNN_Cell / CTCBeamSearch.  Those classes are re-implemented in
 * gpu-accelerated-speech-recognition_amd/api/ on top of THIS interface, and
 * every entry point below names the reference member it replaces.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Pointers named d_* are device pointers
 *    (from asr_device_malloc or any other HIP allocation on the current
 *    device); h_* are host pointers.
 *  - Matrices are row-major fp32, exactly as cuMatrix stores them
 *    (cuMatrix.h:12 "rows-major"); weights are [in][out] (Linear.cu:13,
 *    RNN_Cell.cu:16-17).
 *  - Emissions are time-major [T][B][V] (CTCBeamSearch.cu:67-69
 *    getBatchAtT; RNN.cu:20 writes hiddens at offset t*B*H).
 *  - asr_stream_t is a hipStream_t; NULL means the default stream.
 *  - Every call returns an asr_status (0 = ASR_OK).  No exception crosses
 *    this boundary.  The reference prints and calls exit(0) instead
 *    (cuMatrix.h:85,103,207,218; cuMatrix.cpp:35-41; CTCBeamSearch.cu:267-270);
 *    the C++ layer in api/ restores that behaviour for drop-in callers.
 *  - All calls are asynchronous on the given stream unless documented.
 */
#ifndef ASR_AMD_H_
#define ASR_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* asr_stream_t;

typedef enum asr_status {
    ASR_OK = 0,
    ASR_ERR_ARG = 1,            /* bad argument / shape mismatch           */
    ASR_ERR_HIP = 2,            /* HIP runtime error                       */
    ASR_ERR_OOM = 3,            /* device or pinned host allocation failed */
    ASR_ERR_BEAM_OVERFLOW = 4,  /* more tied survivors than max_states     */
    ASR_ERR_UNSUPPORTED = 5,    /* shape outside what the kernels support  */
    ASR_ERR_STATE = 6,          /* call out of order (e.g. no decode yet)  */
    ASR_ERR_INTERNAL = 7        /* a decoder self-check failed (a bug)     */
} asr_status;

const char* asr_status_string(int status);
/* Library build identification ("gfx950 ..."). */
const char* asr_version(void);

/* ---- device / memory: replaces MemoryMonitor (MemoryMonitor.cpp:9-51) and
 *      the cudaMemcpy/cudaMemset calls of cuMatrix (cuMatrix.h:72-130). ---- */
int asr_get_device_count(int* count);
int asr_set_device(int device);
int asr_get_device(int* device);
int asr_device_malloc(void** d_ptr, size_t bytes);     /* MemoryMonitor::gpuMalloc, zero-filled */
int asr_device_free(void* d_ptr);                      /* MemoryMonitor::freeGpuMemory */
int asr_host_malloc(void** h_ptr, size_t bytes);       /* MemoryMonitor::cpuMalloc (pinned) */
int asr_host_free(void* h_ptr);                        /* MemoryMonitor::freeCpuMemory */
int asr_memcpy_h2d(void* d_dst, const void* h_src, size_t bytes, asr_stream_t s); /* cuMatrix::toGpu */
int asr_memcpy_d2h(void* h_dst, const void* d_src, size_t bytes, asr_stream_t s); /* cuMatrix::toCpu */
int asr_memcpy_d2d(void* d_dst, const void* d_src, size_t bytes, asr_stream_t s);
int asr_memset(void* d_ptr, int value, size_t bytes, asr_stream_t s);             /* cuMatrix::gpuClear */
int asr_stream_create(asr_stream_t* s);
int asr_stream_destroy(asr_stream_t s);
int asr_stream_sync(asr_stream_t s);
int asr_device_sync(void);

/* ---- dense ops (MFMA fp32) ---------------------------------------------- */

/* z[M,N] = x[M,K] . y[K,N]  — cuMatrix.cpp:33-70 matrixMul (cublasSgemm). */
int asr_matmul(const float* d_x, const float* d_y, float* d_z, int M, int K, int N,
               asr_stream_t s);
/* matrixMulTA (cuMatrix.cpp:73-107): z[K,N] = x[M,K]^T . y[M,N] */
int asr_matmul_ta(const float* d_x, const float* d_y, float* d_z, int M, int K, int N,
                  asr_stream_t s);
/* matrixMulTB (cuMatrix.cpp:110-145): z[M,N] = x[M,K] . y[N,K]^T */
int asr_matmul_tb(const float* d_x, const float* d_y, float* d_z, int M, int K, int N,
                  asr_stream_t s);
/* z = x + lambda*y over M*N elements — cuMatrix.cpp:147-168 matrixAdd (cublasSgeam). */
int asr_matadd(const float* d_x, const float* d_y, float* d_z, int M, int N, float lambda,
               asr_stream_t s);

typedef enum asr_epilogue {
    ASR_EPI_NONE = 0,            /* y = x.W                                         */
    ASR_EPI_BIAS = 1,            /* y = x.W + b                                     */
    ASR_EPI_BIAS_RELU = 2,       /* y = max(x.W + b, 0)  — Linear.cu:3-10 ReLU      */
    ASR_EPI_BIAS_LOGSOFTMAX = 3  /* y = log_softmax(x.W + b) per row (model.py:49)  */
} asr_epilogue;

/* Linear::forward (Linear.cu:42-49): y[M,N] = epi(x[M,K] . W[K,N] + b[N]).
 * ASR_EPI_BIAS_LOGSOFTMAX is fused into the GEMM for N <= 64 and a row pass
 * after it otherwise. */
int asr_linear_fwd(const float* d_x, const float* d_W, const float* d_b, float* d_y, int M,
                   int K, int N, int epilogue, asr_stream_t s);

/* RNN_Cell::forward (RNN_Cell.cu:65-74):
 * h_out[B,H] = tanh((x[B,in].W_ih[in,H] + h_prev[B,H].W_hh[H,H]) + (b_hh + b_ih)). */
int asr_rnn_cell_fwd(const float* d_x, const float* d_h_prev, const float* d_W_ih,
                     const float* d_W_hh, const float* d_b_ih, const float* d_b_hh,
                     float* d_h_out, int B, int in, int H, asr_stream_t s);

/* One RNN layer over a whole sequence — RNN::forward (RNN.cu:9-30) for one
 * layer: x time-major [T*B, in], h0 [B,H] (NULL = zeros, RNN.h:15-16),
 * hiddens [T*B, H].  The input projection for all T is one MFMA GEMM; the
 * recurrence runs in one launch with W_hh resident on chip (H <= 256) or as
 * T fused cell launches otherwise. */
int asr_rnn_fwd(const float* d_x, const float* d_h0, const float* d_W_ih, const float* d_W_hh,
                const float* d_b_ih, const float* d_b_hh, float* d_hiddens, int T, int B,
                int in, int H, asr_stream_t s);

/* The recurrence stage of asr_rnn_fwd alone, for callers that run the input
 * projection themselves (e.g. asr_linear_fwd(x, W_ih, NULL, hiddens, ...,
 * ASR_EPI_NONE) on another stream, so that the next batch's projection
 * overlaps this batch's recurrence): on entry d_hiddens [T*B, H] holds
 * P = x.W_ih, on return the hidden states, in place.  asr_rnn_fwd is exactly
 * this after that GEMM (RNN.cu:9-30 split at its two stages). */
int asr_rnn_recur_fwd(const float* d_h0, const float* d_W_hh, const float* d_b_ih,
                      const float* d_b_hh, float* d_hiddens, int T, int B, int H, asr_stream_t s);

/* For 384 <= H <= 1024 (H % 128 == 0, B <= 256) asr_rnn_fwd / asr_rnn_recur_fwd
 * run the whole recurrence in ONE launch whose workgroups hand h_t to each
 * other (W_hh resident in registers); it is taken only when its H/32 x
 * ceil(B/16) workgroups fit the CUs the stream may use (half of them for a
 * plain call, less other such launches in flight; the pipeline's share for
 * its own), never while the stream is capturing.  Residency is still not
 * guaranteed (other processes, other work on those CUs), so a launch that
 * waits 0.5 s without progress gives up and a one-workgroup recovery kernel
 * queued behind it on the same stream finishes the frames it had not
 * published, with the same arithmetic: the call's result is always the
 * complete recurrence, bit for bit (never a partial h with ASR_OK), only
 * slower.  This reports how many such launches ran and how many completed
 * through the recovery (counted once their stream has passed them).
 * (Replaces nothing in the reference: RNN.cu:9-30 launched T steps.) */
int asr_rnn_persist_stats(long long* launches, long long* recoveries);

/* Recurrence kernel choice for H <= 256 (H % 16 == 0), process-wide:
 * ASR_RNN_RECUR_VALU — one utterance per CU, W_hh in registers: the shortest
 *   step (~0.7-0.9 us), a whole CU per utterance;
 * ASR_RNN_RECUR_MFMA — 16 utterances per workgroup on MFMA: ~2.7 us per step
 *   on the split-bf16 arithmetic at H = 256 (~4.6 us on fp32 MFMA)
 *   but ~3x less CU time per utterance (for throughput pipelines whose
 *   production runs beside other work);
 * ASR_RNN_RECUR_AUTO (default) — MFMA from B >= 4 x CUs on.
 * Results agree to fp32 rounding (different summation order), not bit for
 * bit: under AUTO an utterance's hidden states therefore depend on the batch
 * size it runs in (a batch of >= 4 x CUs and a smaller shard of it take
 * different kernels).  Callers that need an utterance's bits to be
 * independent of the batch (utterance sharding over GPUs, re-decoding a
 * shard) pin a kind with asr_rnn_set_recurrence.  Thread-local overrides
 * set by asr_pipeline_* never leak out of the pipeline's own calls. */
enum { ASR_RNN_RECUR_AUTO = 0, ASR_RNN_RECUR_VALU = 1, ASR_RNN_RECUR_MFMA = 2 };
int asr_rnn_set_recurrence(int kind);
int asr_rnn_get_recurrence(int* kind);

/* Arithmetic of the dense fp32 contractions (GEMMs with K <= 256 and N >= 64,
 * the MFMA recurrence and the fused emission recurrence at H = 64 / 128 / 256),
 * process-wide:
 * ASR_DENSE_F32 — v_mfma_f32_16x16x4_f32 (fp32 operands);
 * ASR_DENSE_SPLIT_BF16 (default; ASR_DENSE=f32 in the environment selects
 *   the other at start-up) — every fp32 operand split into three bf16 pieces
 *   (x = h + m + l exactly) and the six significant piece products summed on
 *   v_mfma_f32_16x16x32_bf16 in fp32: as accurate as the fp32 kernels
 *   (max error against fp64 / sum |x.y|: 2.2e-7 vs 3.3e-7 for an fp32 FMA
 *   chain; tests/test_dense_x3_gpu.py), 2.7x their MFMA rate.
 * Both agree with the reference's fp32 cuBLAS to fp32 rounding, not bit for
 * bit; the choice depends on this setting and the shape only (never on M),
 * so an utterance's bits do not depend on its batch.  A pipeline keeps the
 * setting it was created under for all its batches. */
enum { ASR_DENSE_F32 = 0, ASR_DENSE_SPLIT_BF16 = 1 };
int asr_set_dense_arith(int arith);
int asr_get_dense_arith(int* arith);

/* The recurrence and the emission layer in one pass — RNN::forward's
 * recurrence (RNN.cu:9-30) followed by Linear::forward (Linear.cu:42-49) with
 * the log_softmax of baseline/model.py:49, for the acoustic model's last RNN
 * layer when H <= 256 (H % 16 == 0) and V <= 32:
 *   h_t = tanh((P_t + h_{t-1}.W_hh) + (b_hh + b_ih)),
 *   emis_t = log_softmax(h_t.W_out + b_out) per row.
 * d_P [T*B, H] holds x.W_ih (read only; asr_linear_fwd(x, W_ih, NULL, P, ...,
 * ASR_EPI_NONE)); d_emis [T*B, V]; d_hiddens [T*B, H] receives the hidden
 * states, or NULL: they are never stored (the emission projection runs on
 * the recurrence's matrix cores from on-chip h_t).  Always the MFMA
 * recurrence (16 utterances per workgroup).  Emissions agree with
 * asr_rnn_recur_fwd + asr_linear_fwd(..., ASR_EPI_BIAS_LOGSOFTMAX) to fp32
 * rounding (another summation order of h.W_out), not bit for bit.
 * ASR_ERR_UNSUPPORTED outside H <= 256, H % 16 == 0, V <= 32. */
int asr_rnn_emit_fwd(const float* d_h0, const float* d_W_hh, const float* d_b_ih,
                     const float* d_b_hh, const float* d_W_out, const float* d_b_out,
                     const float* d_P, float* d_hiddens, float* d_emis, int T, int B, int H,
                     int V, asr_stream_t s);

/* Bidirectional single-layer RNN — nn.RNN(bidirectional=True) of the Python
 * baseline (baseline/model.py:30, "bidir true"); the C++
 * RNN class (RNN.h:13-20) has no such mode, so this is an added entry point.
 * Direction d = 0 runs t = 0..T-1, d = 1 runs t = T-1..0, each with its own
 * W_ih[d] [in,H], W_hh[d] [H,H], b_ih[d], b_hh[d] (RNN_Cell layout).
 * h0: [2][B][H] (NULL = zeros).  out: [T*B, 2H] time-major, row = (h_fwd, h_bwd)
 * as torch concatenates them.  work: device scratch of
 * asr_rnn_bidir_workspace_bytes(T,B,H) bytes, 16-B aligned; H % 4 == 0.  The
 * two recurrences run concurrently (the reverse one on a library side stream
 * joined back into s). */
size_t asr_rnn_bidir_workspace_bytes(int T, int B, int H);
int asr_rnn_bidir_fwd(const float* d_x, const float* d_h0, const float* const d_W_ih[2],
                      const float* const d_W_hh[2], const float* const d_b_ih[2],
                      const float* const d_b_hh[2], float* d_out, void* d_work, int T, int B,
                      int in, int H, asr_stream_t s);

/* ---- CTC prefix beam search: replaces CTCBeamSearch (CTCBeamSearch.h:107-150,
 *      CTCBeamSearch.cu:220-312) with the semantics of the CPU decoder
 *      CTCBeamSearch.cpp:50-187 (fixes F1-F3, fp64 log domain). ---- */
typedef struct asr_ctc asr_ctc_t;

/* Constructor CTCBeamSearch(char* vocab, int vocabSize, int beamWidth, int blankID)
 * (h:107).  codes[V] is the symbol code of each label (the vocab char as
 * unsigned char for the reference API; NULL = label id, the label-id
 * overload SURVEY a2 asks for large vocabularies).  Hypothesis order on
 * ties is code-string order, as std::string order in the reference.
 * V up to 4096 (V > 63 runs the large-vocabulary kernel, e.g. C5 V=1000);
 * beam_width + 1 + ties <= 256.  max_states bounds the beam incl. ties at the
 * cutoff (0 = automatic, >= beamWidth+1). */
int asr_ctc_create(const int32_t* codes, int V, int beam_width, int blank_id, int max_states,
                   asr_ctc_t** out);
int asr_ctc_destroy(asr_ctc_t* h);

/* CTCBeamSearch::decode(seqProb, timestep, batchSize) (cu:262): decode B
 * utterances of d_emis[T][B][V] (probabilities, or log-probabilities if
 * is_log).  Enqueues the decode and the best-path traceback on stream s; the
 * workspace is sized once and reused (the reference re-allocated per call,
 * cu:263).  Fetch results with asr_ctc_get_best / asr_ctc_get_beams.
 * Lifetime: d_emis must stay allocated and unmodified until the results of
 * this decode have been fetched (asr_ctc_get_best / asr_ctc_get_beams
 * returned), because an automatic-capacity handle re-decodes it when ties
 * at the cutoff overflow the beam (see asr_ctc_get_best).  Work the caller
 * queues that writes d_emis must be ordered after that fetch. */
int asr_ctc_decode(asr_ctc_t* h, const float* d_emis, int T, int B, int is_log, asr_stream_t s);

/* General form (ctcdecode-style batches): element
 * (t, b, v) of the emissions is d_emis[t*frame_stride + b*utt_stride + v]
 * (time-major [T][B][V]: B*V, V; batch-major [B][T][V]: V, T*V), and
 * utterance b has h_lengths[b] <= T frames (host array; NULL = T for all).
 * asr_ctc_decode(h, e, T, B, is_log, s) is this with time-major strides. */
int asr_ctc_decode_ex(asr_ctc_t* h, const float* d_emis, int T, int B, long frame_stride,
                      long utt_stride, const int32_t* h_lengths, int is_log, asr_stream_t s);

/* Segmented (streaming) decode — no reference counterpart (the reference
 * decodes whole utterances, CTCBeamSearch.cu:262-312): frames [t0, t1) of a
 * T-frame batch, the beam of every utterance carried on the device from one
 * segment to the next, so a producer can hand over emissions segment by
 * segment and the decode of a batch starts after its first T/S frames.
 * Segments come in order on one handle: t0 = 0 first (h_lengths is read
 * then), each next t0 = the previous t1, the last ends at t1 = T; then the
 * results are fetched as after asr_ctc_decode (asr_ctc_get_best ...; before
 * that, ASR_ERR_STATE).  d_emis addresses frame t0: element (t, b, v) of the
 * segment is d_emis[(t - t0)*frame_stride + b*utt_stride + v].  T, B, the
 * strides and is_log must be the same for every segment.  Results are
 * bit-identical to a whole decode of the same frames.  Runs the one-wave
 * kernel (ASR_CTC_WAVES_LIST) for V <= 63 and the large-vocabulary kernel
 * for 63 < V <= 4096 (each frame's first vocabulary tile precomputed per
 * segment); CPU semantics and timesteps off, else ASR_ERR_UNSUPPORTED;
 * ASR_ERR_STATE for a segment out of order.  Overflow
 * retry (automatic capacity): asr_ctc_get_best re-decodes the whole batch
 * from the FIRST segment's d_emis over T frames, so that pointer must then
 * address all T frames (e.g. segments of one [T][B][V] buffer); a caller
 * with a ring buffer creates the handle with an explicit max_states (an
 * overflow is then reported as ASR_ERR_BEAM_OVERFLOW).
 * asr_ctc_last_kernel_ms reports the sum of the segments' kernel times. */
int asr_ctc_decode_segment(asr_ctc_t* h, const float* d_emis, int T, int t0, int t1, int B,
                           long frame_stride, long utt_stride, const int32_t* h_lengths, int is_log,
                           asr_stream_t s);

/* Best hypothesis of each utterance (cpp:74-84: max score, first in string
 * order on ties).  Synchronises the decode stream.  h_labels[B][max_len]
 * (label ids), h_lengths[B], h_logp[B] (fp64 log-probability).
 * If an utterance had more tied survivors than max_states, the batch is
 * decoded again with a wider beam capacity (up to 256 states) before
 * returning; ASR_ERR_BEAM_OVERFLOW only if that is not enough (the result is
 * then not the reference's) or if the handle was created with an explicit
 * max_states. */
int asr_ctc_get_best(asr_ctc_t* h, int32_t* h_labels, int max_len, int32_t* h_lengths,
                     double* h_logp);

/* Full final beam of every utterance, ranked by (logp desc, string asc):
 * h_n_hyps[B], h_lengths[B][max_hyps], h_labels[B][max_hyps][max_len],
 * h_logp[B][max_hyps].  Runs a traceback over all final hypotheses. */
int asr_ctc_get_beams(asr_ctc_t* h, int max_hyps, int max_len, int32_t* h_n_hyps,
                      int32_t* h_lengths, int32_t* h_labels, double* h_logp);

/* Timesteps mode (ctcdecode's `timesteps` output, baseline/main.py:46; the
 * reference C++ decoder has none): when on, decodes also record the frame at
 * which every label of every live prefix was appended (a continuing prefix
 * keeps its frames; a new prefix is its parent's plus the current frame), at
 * 16 extra bytes per node record and slot.  Off by default; the one-wave
 * list kernel is not used while it is on.  asr_ctc_get_beams_ts returns them
 * as h_timesteps[B][max_hyps][max_len] next to the ranked labels
 * (ASR_ERR_STATE if the decode ran without timesteps).  Frames are stored in
 * 16 bits: with timesteps on, a decode of T > ASR_CTC_TS_MAX_T frames returns
 * ASR_ERR_UNSUPPORTED (nothing is enqueued). */
#define ASR_CTC_TS_MAX_T 65536
int asr_ctc_set_timesteps(asr_ctc_t* h, int on);

/* Stream for the best-path traceback and the copy of its results to host
 * memory (default NULL: the decode's own stream).  With a separate stream
 * the decode stream is free for the next batch as soon as the beam search
 * ends; asr_ctc_get_best waits for the results either way, and the next
 * decode on this handle waits for its traceback.  No reference
 * counterpart (a scheduling option). */
int asr_ctc_set_result_stream(asr_ctc_t* h, asr_stream_t s);
int asr_ctc_get_beams_ts(asr_ctc_t* h, int max_hyps, int max_len, int32_t* h_n_hyps,
                         int32_t* h_lengths, int32_t* h_labels, double* h_logp, int32_t* h_timesteps);

/* Device time of the last decode's beam-search kernel (ms, HIP events on the
 * decode stream) and its launch geometry; for roofline accounting. */
int asr_ctc_last_kernel_ms(asr_ctc_t* h, float* ms);
/* Search semantics.  ASR_CTC_SEMANTICS_CPU (default):
 * CTCBeamSearch.cpp with fixes F1-F3 — beam+1 states plus ties at the cutoff,
 * final "q"/"q$" merge after the last prune; the parity target.
 * ASR_CTC_SEMANTICS_CUDA: what CTCBeamSearch.cu computes when it works —
 * exactly min(beam, n) states per step (stable descending sort, cu:174-196;
 * ties at the cutoff resolved in a fixed slot order instead of the .cu's
 * string order), and on the last step the trailing blank is stripped before
 * the merge and the prune (cu:452-456).  Any V (the reference's char vocabs
 * have up to 256 symbols, CTCBeamSearch.h:43). */
enum { ASR_CTC_SEMANTICS_CPU = 0, ASR_CTC_SEMANTICS_CUDA = 1 };
int asr_ctc_set_semantics(asr_ctc_t* h, int semantics);

/* Tuning knobs: waves per utterance (1, 2, 4 or 8; 0 = automatic), or
 * ASR_CTC_WAVES_LIST: one wave per utterance with live-label candidate lists
 * (faster on peaked emissions, slower on flat ones).
 * get_config reports the schedule a decode will use (ASR_CTC_WAVES_LIST or 1..8). */
#define ASR_CTC_WAVES_LIST (-1)
int asr_ctc_set_waves(asr_ctc_t* h, int waves);
/* Scheduling hint: n decodes of this handle's batch size are in flight on
 * the device at once (e.g. a caller pipelining n batches on n streams;
 * default 1).  The automatic schedule is then chosen for n x B utterances
 * sharing the CUs — from two per CU on, the 4-wave kernel several
 * workgroups to a CU.  Never changes results. */
int asr_ctc_set_concurrency(asr_ctc_t* h, int n);
int asr_ctc_get_config(asr_ctc_t* h, int* max_states, int* waves, int* lds_bytes);

/* ---- throughput pipeline (no reference counterpart: the reference runs one
 *      batch at a time with host syncs between calls, main.cpp:40-72,
 *      RNN.cu:9-30, CTCBeamSearch.cu:262-312) ---------------------------------
 * RNN (one layer, h0 = 0) -> Linear + log_softmax -> CTC beam search over a
 * stream of equal-shape batches.  The library owns the streams, buffers and
 * decoder handles and overlaps the production of later batches with the
 * decodes of earlier ones, placing the kernels on the CUs for the shape
 * (DESIGN.md §7a-§7c).  Weights are caller-owned device arrays in the layouts of
 * asr_rnn_fwd / asr_linear_fwd and must outlive the pipeline. */
typedef struct asr_pipeline asr_pipeline_t;
typedef struct asr_pipeline_config {
    int T, B;            /* frames and utterances per batch */
    int in, H, V;        /* feature, hidden and vocabulary (incl. blank) sizes */
    int beam, blank;     /* decoder beam width and blank id (CPU semantics) */
    int inflight;        /* decodes in flight (0 = automatic) */
    int prod_streams;    /* production streams (0 = automatic) */
    int decode_cus;      /* chip-filling batches: CUs given to decoding (0 = automatic,
                            -1 = every stream on every CU) */
    int segments;        /* T-segments per batch (0 = automatic, 1 = whole utterances): the
                            fused production hands emissions over segment by segment and
                            the decode of a batch starts after its first T / segments
                            frames (asr_ctc_decode_segment); chip-filling batches with the
                            fused production only, else 1 */
} asr_pipeline_config;
int asr_pipeline_create(const asr_pipeline_config* cfg, const float* d_W_ih, const float* d_W_hh,
                        const float* d_b_ih, const float* d_b_hh, const float* d_W_out,
                        const float* d_b_out, asr_pipeline_t** out);
/* Enqueue one batch: features d_x [T*B, in] (time-major, device; read by the
 * batch's production, so it must stay unmodified until the batch is
 * collected).  Returns once the work is queued; when the caller is as many
 * batches behind as the pipeline has buffers, the oldest batch's results are
 * fetched internally first (asr_pipeline_collect still returns them).
 * Errors: a batch whose production could not be queued is not accepted (the
 * error is returned and the pipeline is unchanged: submit it again or
 * destroy).  If the rest of an accepted batch's work (this one's decode, or
 * the previous batch's emission projection + decode in the split schedule)
 * fails to queue, the pipeline is failed from that batch on: this and every
 * later submit, and the collect of that batch and every later one, return
 * the error; earlier batches are still collected normally. */
int asr_pipeline_submit(asr_pipeline_t* p, const float* d_x);
/* Results of the oldest uncollected batch, in submission order (blocks):
 * h_labels[B][max_len], h_lengths[B], h_logp[B] as asr_ctc_get_best, and the
 * batch's beam-search kernel time (ms; may be NULL). */
int asr_pipeline_collect(asr_pipeline_t* p, int32_t* h_labels, int max_len, int32_t* h_lengths,
                         double* h_logp, float* decode_ms);
int asr_pipeline_pending(asr_pipeline_t* p, int* n_uncollected);
/* Dynamic batching: a pipeline whose submits carry cfg->B utterances each
 * and whose launches carry group * cfg->B — `group` consecutive submits are
 * copied side by side into one batch (time-major [T][group * B][in]) and go
 * through one production and one decode; asr_pipeline_collect returns each
 * submit's B rows in submission order.  Collecting a submit whose batch is
 * not complete queues that batch with zero features in the missing columns
 * (their rows are decoded and dropped).  The results are the per-submit
 * pipeline's bits (every utterance is independent).  group = 1 is
 * asr_pipeline_create.  ASR_ERR_UNSUPPORTED unless the batch of
 * group * B runs the chip-filling schedule with the fused production
 * (H <= 256, V <= 32: the production whose bits do not depend on the batch
 * shape, its input projection on the batch's production stream).  (The
 * reference decodes one batch per call: CTCBeamSearch.cu:262-312.) */
int asr_pipeline_create_coalesced(const asr_pipeline_config* cfg, int group, const float* d_W_ih,
                                  const float* d_W_hh, const float* d_b_ih, const float* d_b_hh,
                                  const float* d_W_out, const float* d_b_out, asr_pipeline_t** out);
/* group, utterances per submit, and the column (0 .. group - 1) of the
 * submit collected last inside its batch (asr_pipeline_peek_emissions then
 * returns the whole batch's [T][group * B][V] emissions). */
int asr_pipeline_get_coalesce(asr_pipeline_t* p, int* group, int* batch, int* column);
/* The schedule chosen: mode (0 CU groups for small batches, 1 chip-filling
 * batches, 2 CU groups for H > 256), decodes in flight, production streams,
 * CUs per decode group / decode partition, and the decoder's waves per
 * utterance in the last decode.  Any pointer may be NULL.
 * asr_pipeline_get_segments: T-segments per batch in use.
 * asr_pipeline_get_groups: batches whose recurrences run as one (mode 2,
 * H > 256: one per-frame step launch for G batches; a batch's production
 * then starts when its group is complete or its results are asked for). */
int asr_pipeline_get_segments(asr_pipeline_t* p, int* segments);
/* The drain schedule (T-segmented batches): the last decode segment of the
 * newest `held_batches` batches is held back; a newer batch releases the
 * oldest onto its decode stream, and when the caller drains (collects a
 * batch within `inflight` of a held one) every held segment is queued on its
 * batch's production stream behind that stream's last production, so the
 * drain's decodes also use the production CUs.  first_segment_share: the
 * first T-segment's share of T (0.5 = equal halves).  Either may be NULL. */
int asr_pipeline_get_drain(asr_pipeline_t* p, int* held_batches, double* first_segment_share);
int asr_pipeline_get_groups(asr_pipeline_t* p, int* group);
int asr_pipeline_describe(asr_pipeline_t* p, int* mode, int* inflight, int* prod_streams, int* decode_cus,
                          int* decode_waves);
/* How the pipeline produces a batch's emissions: fused = 1 when the
 * recurrence and the emission projection + log_softmax run as one kernel
 * (chip-filling batches with H % 16 == 0, V <= 32: asr_linear_fwd(x, W_ih,
 * NULL, P, ..., ASR_EPI_NONE) then asr_rnn_emit_fwd(NULL, W_hh, b_ih, b_hh,
 * W_out, b_out, P, NULL, emis, ...) gives its bits), 0 when it is
 * asr_rnn_fwd then asr_linear_fwd(..., ASR_EPI_BIAS_LOGSOFTMAX);
 * decode_cu_rows: input-projection rows run on the decode CUs; recurrence:
 * the recurrence kind the unfused production pins (ASR_RNN_RECUR_*; AUTO =
 * the process-wide choice), so a caller can reproduce the emissions bit for
 * bit.  Any pointer may be NULL. */
int asr_pipeline_get_production(asr_pipeline_t* p, int* fused, long long* decode_cu_rows, int* recurrence);
/* Streams the pipeline created and the process's HIP hardware queues
 * (GPU_MAX_HW_QUEUES as read at create; HIP's default is 4).  HIP maps the
 * UNMASKED streams round-robin onto those queues (streams that share a queue
 * serialise); a CU-masked stream gets a hardware queue of its own.  The
 * pipeline's chip-filling and CU-group schedules mask their decode and
 * production streams, so they need no GPU_MAX_HW_QUEUES setting (measured
 * at HIP's default of 4: the same frames/s as at 24);
 * only the unmasked ones (every stream with decode_cus = -1, the small-batch
 * mode's GEMM streams) are fitted to the queues (no input-projection share
 * on the decode CUs, then fewer production streams down to half the
 * decodes in flight, then both), unless the caller fixed inflight /
 * prod_streams.  asr_pipeline_get_queue_use: how many of the streams share
 * HIP's queues and how many have a queue of their own. */
int asr_pipeline_get_streams(asr_pipeline_t* p, int* streams, int* hw_queues);
int asr_pipeline_get_queue_use(asr_pipeline_t* p, int* shared_queue_streams, int* dedicated_queue_streams);
/* Where the pipeline's streams run: for each stream it created, its role
 * (ASR_PIPE_ROLE_*) and the CU range [cu_lo, cu_hi) of its CU mask
 * (hipExtStreamCreateWithCUMask bits; [0, ncu) = unmasked).  *n = streams
 * created; the first min(cap, *n) entries are written. */
enum { ASR_PIPE_ROLE_DECODE = 0, ASR_PIPE_ROLE_PRODUCTION = 1, ASR_PIPE_ROLE_DECODE_CU_GEMM = 2,
       ASR_PIPE_ROLE_GEMM = 3 };
#define ASR_MAX_XCC 16
int asr_pipeline_get_placement(asr_pipeline_t* p, int cap, int* n, int* role, int* cu_lo, int* cu_hi);
/* Diagnostic: the physical CUs the first stream of `role` reaches, counted per
 * XCD (cus_per_xcc[ASR_MAX_XCC], *n_xcc = XCDs seen): one probe launch of
 * 8192 short workgroups on that stream that read HW_REG_XCC_ID / HW_REG_HW_ID
 * (synchronises the stream).  Workgroups are dealt round-robin over the XCDs
 * whatever the mask, so a role runs evenly only when its mask holds the same
 * number of CUs in every XCD (mask bit i lands on XCD i % 8; an XCD the mask
 * leaves out gets all of its CUs); DESIGN.md §10c. */
int asr_pipeline_probe_placement(asr_pipeline_t* p, int role, int* cus_per_xcc, int* n_xcc);
/* The emissions [T][B][V] (log-probabilities, device) that the decode of the
 * batch last returned by asr_pipeline_collect consumed — the exact bytes, for
 * parity checks of the pipelined path.  Valid until the next submit that
 * reuses the buffer; ASR_ERR_STATE if nothing was collected yet or the
 * buffer has been reused. */
int asr_pipeline_peek_emissions(asr_pipeline_t* p, const float** d_emis);
/* Timeline (measurement): with timing on, every batch submitted from now on
 * records four timing events — its production's start and end on the
 * production stream(s) and its decode's start (the first decode kernel
 * queued behind its emissions) and end on its decode stream — read back when
 * the batch is collected, as ms after the moment of this call.  Call it on
 * a drained pipeline (it synchronises the device); it clears the timeline.
 * A decode's "start" is when its stream reached it, which may be before
 * its workgroups get CUs.  asr_pipeline_get_timeline: *n = batches recorded;
 * the first min(cap, *n) as batch[i] and t[i][4] = (production start,
 * production end, decode start, decode end). */
int asr_pipeline_set_timing(asr_pipeline_t* p, int on);
int asr_pipeline_get_timeline(asr_pipeline_t* p, int cap, int* n, long long* batch, float* t);
int asr_pipeline_destroy(asr_pipeline_t* p);

#ifdef __cplusplus
}
#endif
#endif /* ASR_AMD_H_ */
