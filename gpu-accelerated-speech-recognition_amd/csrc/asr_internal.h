// Internal declarations shared by the HIP translation units of libasr_amd.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "asr_amd.h"

#define ASR_HIP_TRY(expr)                                                        \
    do {                                                                         \
        hipError_t e_ = (expr);                                                  \
        if (e_ != hipSuccess) {                                                  \
            asr_internal_set_error(#expr, hipGetErrorString(e_), __FILE__, __LINE__); \
            return e_ == hipErrorOutOfMemory ? ASR_ERR_OOM : ASR_ERR_HIP;        \
        }                                                                        \
    } while (0)

#define ASR_LAUNCH_TRY()                                                         \
    do {                                                                         \
        hipError_t e_ = hipGetLastError();                                       \
        if (e_ != hipSuccess) {                                                  \
            asr_internal_set_error("kernel launch", hipGetErrorString(e_), __FILE__, __LINE__); \
            return ASR_ERR_HIP;                                                  \
        }                                                                        \
    } while (0)

void asr_internal_set_error(const char* what, const char* msg, const char* file, int line);

#include <mutex>
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) of one kernel, once per
// device, safe under concurrent first calls (pipeline threads, several
// devices in one process).  One static instance per kernel instantiation.
struct AsrAttrOnce {
    std::mutex m;
    uint64_t done = 0;   // bit d: set on device d
    int set(const void* fn, int bytes) {
        int dev = 0;
        ASR_HIP_TRY(hipGetDevice(&dev));
        const uint64_t bit = (dev >= 0 && dev < 64) ? (1ull << dev) : 0ull;
        std::lock_guard<std::mutex> g(m);
        if (bit && (done & bit)) return ASR_OK;
        ASR_HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
        done |= bit;
        return ASR_OK;
    }
};

static inline hipStream_t asr_stream(asr_stream_t s) { return (hipStream_t)s; }

// Recurrence kernel for this thread's next RNN calls (ASR_RNN_RECUR_*; -1:
// the process-wide asr_rnn_set_recurrence choice).  Set by the pipeline
// around its production so that it never changes the process-wide state.
extern thread_local int asr_internal_rnn_kind;
// Set by the pipeline around GEMMs that share CUs with decodes: use the tiled
// kernel (short-lived workgroups) instead of the persistent wide one, so that
// a decode launched meanwhile waits at most one tile for its CUs.  Same bits.
// The value is the split-bf16 kernel's row tiles per workgroup (0: off).
extern thread_local int asr_internal_gemm_tiled;
// Set by the pipeline around its productions: capture the per-frame
// recurrence launches (H > 256) into the library's HIP graph at their first
// use, not the second (a pipeline's buffers recur; one-off calls stay eager).
extern thread_local int asr_internal_graph_now;
// Set by the pipeline around its productions: the CUs one recurrence may
// count on (its production streams' CU share), for the one-launch H > 256
// recurrence whose workgroups must all be resident (0: no hint).
extern thread_local int asr_internal_persist_cus;
// Dense arithmetic for this thread's next dense calls (ASR_DENSE_*; -1: the
// process-wide asr_set_dense_arith setting).  A pipeline latches the setting
// it was created under and sets this around its own calls, so a later change
// of the process-wide setting never changes a running pipeline's bits.
extern thread_local int asr_internal_dense_arith;
// One-wave decoder workgroups (utterances) that fit on one CU for this
// handle's layout (the occupancy query); 0 when the one-wave kernel does not
// apply (V > 63, .cu semantics, timesteps).  For the pipeline's schedule.
struct asr_ctc;
int asr_internal_ctc_wave_occupancy(asr_ctc* h);
// The wide decoder's first-tile precompute (ctc_tile0_kernel) queued by the
// caller instead of ahead of each decode launch: _external(h, B, T) sizes the
// handle's workspace for B x T and switches the decode's own precompute off
// (ASR_ERR_UNSUPPORTED when the handle takes none: V <= 65); _tile0 fills
// frames [t0, t1) of the B utterances from d_emis (at frame t0) on stream s.
// The records are the decode's own (same kernel), so the bits do not change;
// the caller orders them before the decode of those frames.
int asr_internal_ctc_tile0_external(asr_ctc* h, int B, int T);
int asr_internal_ctc_tile0(asr_ctc* h, const float* d_emis, int T, int t0, int t1, int B, long frame_stride,
                           long utt_stride, hipStream_t s);
// The recurrence (h0 = 0) of nb <= 4 equal-shape batches at once, in place
// over each hids[j] [T*B, H] (holding x.W_ih on entry): H > 256 runs one
// per-frame MFMA step launch for all of them (the step is latency-bound, so
// a step of 2-4 batches costs about one); bit-identical to nb separate
// asr_rnn_recur_fwd calls.  ASR_ERR_UNSUPPORTED for H <= 256 with nb > 1 or
// B % 16 != 0.
int asr_internal_rnn_recur_multi(const float* W_hh, const float* b_ih, const float* b_hh, float* const* hids,
                                 int nb, int T, int B, int H, hipStream_t st);

// Order-preserving bijection fp64 <-> u64: a < b  <=>  key(a) < key(b).
// -0.0 is folded onto +0.0 (they compare equal as doubles).  Key 0 is never
// produced for a non-NaN value (-inf maps to 0x000FFFFFFFFFFFFF), so it marks
// an absent candidate.
__host__ __device__ static inline uint64_t asr_d2key(double x) {
    x = x + 0.0;
    uint64_t u = __builtin_bit_cast(uint64_t, x);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__host__ __device__ static inline double asr_key2d(uint64_t k) {
    uint64_t u = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
    return __builtin_bit_cast(double, u);
}
