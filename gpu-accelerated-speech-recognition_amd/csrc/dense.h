// Host/device interface of the dense fp32 kernels (dense.hip).
#pragma once
#include "asr_internal.h"

namespace asr {

enum GemmEpilogue {
    EPI_NONE = 0,        // C = A.B
    EPI_BIAS = 1,        // C = A.B + b1
    EPI_BIAS_RELU = 2,   // C = max(A.B + b1, 0)
    EPI_LOGSOFTMAX = 3,  // C = log_softmax(A.B + b1) per row (fused for N <= 64)
    EPI_DUAL_TANH = 4,   // C = tanh((A.B + A2.B2) + (b2 + b1))
    EPI_ADD_TANH = 5     // C = tanh((D + A.B) + (b2 + b1)); C may alias D
};

struct GemmArgs {
    const float* A;   // A(m,k) = A[m*sam + k*sak]
    const float* B;   // B(k,n) = B[k*sbk + n*sbn]
    const float* A2;  // EPI_DUAL_TANH: [M][K2] row-major
    const float* B2;  // EPI_DUAL_TANH: [K2][N] row-major
    const float* b1;
    const float* b2;
    const float* D;   // EPI_ADD_TANH addend, [M][ldc]
    float* C;         // [M][ldc]
    int M, N, K, K2;
    long sam, sak, sbk, sbn, ldc;
};

int gemm_launch(const GemmArgs& g, int epi, hipStream_t s);
int rnn_recur_launch(const float* h0, const float* Whh, const float* b_ih, const float* b_hh,
                     float* hid, int T, int B, int H, hipStream_t s);
// The same recurrence on MFMA, 16 utterances per workgroup (H <= 256, H % 16 == 0).
int rnn_recur_mfma_launch(const float* h0, const float* Whh, const float* b_ih, const float* b_hh,
                          float* hid, int T, int B, int H, hipStream_t s);
// The MFMA recurrence with the emission projection + log_softmax fused
// (V <= 32): P [T][B][H] read only, hidden states to hout (NULL: not stored);
// hlast [B][H] (optional, may be h0): h_{T-1}, the h0 of a next segment.
int rnn_emit_mfma_launch(const float* h0, const float* Whh, const float* b_ih, const float* b_hh,
                         const float* P, float* hout, const float* Wout, const float* bout, float* emis,
                         int T, int B, int H, int V, hipStream_t s, float* hlast = nullptr, bool pfrag = false);
int bias_tanh_launch(float* p, const float* b_ih, const float* b_hh, long n, int H, hipStream_t s);
int axpy_launch(const float* x, const float* y, float* z, long n, float lam, hipStream_t s);
int row_logsoftmax_launch(float* C, long ldc, int M, int N, hipStream_t s);
// MFMA recurrence step (H % 128 == 0); ASR_ERR_UNSUPPORTED otherwise.
int rnn_step_mfma_launch(float* ht, const float* hp, const float* Whh, const float* b_ih,
                         const float* b_hh, int B, int H, hipStream_t s);
// The whole H > 256 recurrence in one launch with W_hh in registers and the
// workgroups handing h_t to each other in memory (same bits as the step
// launches); ASR_ERR_UNSUPPORTED outside 384 <= H <= 1024, H % 128 == 0,
// B <= 256, or when its (H / 32) x ceil(B / 16) workgroups exceed `cus`
// (the CUs the caller's stream gives this launch; <= 0: half of the device's
// CUs less those of other such launches in flight), or while the stream is
// capturing.  Fail-safe: a launch whose workgroups are not all resident gives
// up after 0.5 s without progress and a recovery kernel on the same stream
// finishes its frames with the same bits.
int rnn_recur_persist_launch(const float* h0, const float* Whh, const float* b_ih, const float* b_hh, float* hid,
                             int T, int B, int H, int cus, hipStream_t s);
// Process-wide counts of one-launch recurrences and of those that completed
// through the recovery kernel (counted once their stream passed them).
int rnn_persist_stats(long long* launches, long long* recoveries);
constexpr int STEP_MAXB = 4;
// The same step for nb <= STEP_MAXB batches of B rows at once (one launch; batch j:
// h_t at hts[j], h_{t-1} at hps[j]); nb > 1 needs B % 16 == 0.  Same bits.
int rnn_step_mfma_multi_launch(float* const* hts, const float* const* hps, int nb, const float* Whh,
                               const float* b_ih, const float* b_hh, int B, int H, hipStream_t s);
int rnn_step_launch(float* ht, const float* hp, const float* Whh, const float* b_ih,
                    const float* b_hh, int B, int H, hipStream_t s);

// Split-bf16 arithmetic (dense_x3.hip): fp32-accurate products on the bf16
// matrix cores.  The setting (asr_set_dense_arith) picks it for every shape
// below that it applies to; the fp32 kernels otherwise.
int dense_arith();
void dense_arith_set(int a);
bool dense_x3_on();
bool gemm_x3_applies(const GemmArgs& g, int epi);
// tpw > 0: runs of tpw 16-row tiles per workgroup (short workgroups); 0: persistent.
int gemm_x3_launch(const GemmArgs& g, int epi, int tpw, hipStream_t s);
bool rnn_x3_applies(int B, int H);
int rnn_recur_x3_launch(const float* h0, const float* Whh, const float* b_ih, const float* b_hh, float* hid,
                        int T, int B, int H, hipStream_t s);
// pfrag: P in the fragment-major layout written by gemm_x3_frag_launch (B % 16 == 0).
int rnn_emit_x3_launch(const float* h0, const float* Whh, const float* b_ih, const float* b_hh, const float* P,
                       float* hout, const float* Wout, const float* bout, float* emis, int T, int B, int H, int V,
                       hipStream_t s, float* hlast, bool pfrag = false);
// The input projection P = A.W (K <= 256, H = N <= 256, H % 32 == 0, M % 16 == 0)
// stored in the fragment-major layout the split-bf16 recurrence reads with
// two 16-byte loads per lane and step (rnn_emit_x3_launch(..., pfrag = true)).
// Internal to the pipeline: the values are asr_linear_fwd's, the layout is not row-major.
int gemm_x3_frag_launch(const float* A, const float* W, float* P, int M, int K, int H, int tpw, hipStream_t s);

// Bidirectional RNN plumbing (H % 4 == 0, 16-B aligned buffers).
int time_reverse_launch(float* p, int T, long n, hipStream_t s);
int bidir_concat_launch(const float* hf, const float* hr, float* out, int T, int B, int H,
                        hipStream_t s);

}  // namespace asr
