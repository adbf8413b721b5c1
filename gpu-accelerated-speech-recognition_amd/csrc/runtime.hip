// ============================================================================
// libasr_amd.so host runtime: the C ABI of include/asr_amd.h.
// Memory (MemoryMonitor / cuMatrix transfers), dense ops (Linear / RNN_Cell /
// RNN / matrixMul / matrixAdd) and the CTC decoder handle (CTCBeamSearch).
// ============================================================================
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <atomic>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "ctc_beam.h"
#include "dense.h"

namespace {
thread_local std::string g_last_error;
}

thread_local int asr_internal_rnn_kind = -1;
thread_local int asr_internal_graph_now = 0;
thread_local int asr_internal_persist_cus = 0;
thread_local int asr_internal_gemm_tiled = 0;

void asr_internal_set_error(const char* what, const char* msg, const char* file, int line) {
    char buf[512];
    snprintf(buf, sizeof buf, "%s: %s (%s:%d)", what, msg, file, line);
    g_last_error = buf;
    if (getenv("ASR_VERBOSE")) fprintf(stderr, "[asr] %s\n", buf);
}

extern "C" {

const char* asr_status_string(int status) {
    switch (status) {
        case ASR_OK: return "ok";
        case ASR_ERR_ARG: return "invalid argument";
        case ASR_ERR_HIP: return g_last_error.empty() ? "HIP runtime error" : g_last_error.c_str();
        case ASR_ERR_OOM: return "out of memory";
        case ASR_ERR_BEAM_OVERFLOW: return "beam overflow: more tied survivors than max_states";
        case ASR_ERR_UNSUPPORTED: return "unsupported shape";
        case ASR_ERR_STATE: return "invalid call order";
        case ASR_ERR_INTERNAL: return "internal decoder self-check failed";
        default: return "unknown status";
    }
}

const char* asr_version(void) { return "libasr_amd gfx950 r1"; }

// ------------------------------------------------------------- device/memory
int asr_get_device_count(int* count) {
    if (!count) return ASR_ERR_ARG;
    ASR_HIP_TRY(hipGetDeviceCount(count));
    return ASR_OK;
}
int asr_set_device(int device) {
    ASR_HIP_TRY(hipSetDevice(device));
    return ASR_OK;
}
int asr_get_device(int* device) {
    if (!device) return ASR_ERR_ARG;
    ASR_HIP_TRY(hipGetDevice(device));
    return ASR_OK;
}
int asr_device_malloc(void** p, size_t bytes) {
    if (!p) return ASR_ERR_ARG;
    *p = nullptr;
    if (bytes == 0) return ASR_OK;
    ASR_HIP_TRY(hipMalloc(p, bytes));
    ASR_HIP_TRY(hipMemset(*p, 0, bytes));   // cuMatrix.h:222 zero-fills on allocation
    return ASR_OK;
}
int asr_device_free(void* p) {
    if (p) ASR_HIP_TRY(hipFree(p));
    return ASR_OK;
}
int asr_host_malloc(void** p, size_t bytes) {
    if (!p) return ASR_ERR_ARG;
    *p = nullptr;
    if (bytes == 0) return ASR_OK;
    ASR_HIP_TRY(hipHostMalloc(p, bytes, hipHostMallocPortable));
    memset(*p, 0, bytes);
    return ASR_OK;
}
int asr_host_free(void* p) {
    if (p) ASR_HIP_TRY(hipHostFree(p));
    return ASR_OK;
}
static int copy(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, asr_stream_t s) {
    if (bytes == 0) return ASR_OK;
    if (!dst || !src) return ASR_ERR_ARG;
    ASR_HIP_TRY(hipMemcpyAsync(dst, src, bytes, kind, asr_stream(s)));
    if (kind != hipMemcpyDeviceToDevice) ASR_HIP_TRY(hipStreamSynchronize(asr_stream(s)));
    return ASR_OK;
}
int asr_memcpy_h2d(void* d, const void* h, size_t n, asr_stream_t s) { return copy(d, h, n, hipMemcpyHostToDevice, s); }
int asr_memcpy_d2h(void* h, const void* d, size_t n, asr_stream_t s) { return copy(h, d, n, hipMemcpyDeviceToHost, s); }
int asr_memcpy_d2d(void* d, const void* e, size_t n, asr_stream_t s) { return copy(d, e, n, hipMemcpyDeviceToDevice, s); }
int asr_memset(void* d, int v, size_t n, asr_stream_t s) {
    if (n == 0) return ASR_OK;
    if (!d) return ASR_ERR_ARG;
    ASR_HIP_TRY(hipMemsetAsync(d, v, n, asr_stream(s)));
    return ASR_OK;
}
int asr_stream_create(asr_stream_t* s) {
    if (!s) return ASR_ERR_ARG;
    hipStream_t st;
    ASR_HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    *s = (asr_stream_t)st;
    return ASR_OK;
}
int asr_stream_destroy(asr_stream_t s) {
    if (s) ASR_HIP_TRY(hipStreamDestroy(asr_stream(s)));
    return ASR_OK;
}
int asr_stream_sync(asr_stream_t s) {
    ASR_HIP_TRY(hipStreamSynchronize(asr_stream(s)));
    return ASR_OK;
}
int asr_device_sync(void) {
    ASR_HIP_TRY(hipDeviceSynchronize());
    return ASR_OK;
}

// ----------------------------------------------------------------- dense ops
static asr::GemmArgs gemm_args(const float* A, const float* B, float* C, int M, int K, int N) {
    asr::GemmArgs g{};
    g.A = A; g.B = B; g.C = C;
    g.M = M; g.N = N; g.K = K;
    g.sam = K; g.sak = 1; g.sbk = N; g.sbn = 1; g.ldc = N;
    return g;
}

int asr_matmul(const float* x, const float* y, float* z, int M, int K, int N, asr_stream_t s) {
    if (!x || !y || !z || M <= 0 || K <= 0 || N <= 0) return ASR_ERR_ARG;
    return asr::gemm_launch(gemm_args(x, y, z, M, K, N), asr::EPI_NONE, asr_stream(s));
}
int asr_matmul_ta(const float* x, const float* y, float* z, int M, int K, int N, asr_stream_t s) {
    // z[K,N] = x[M,K]^T . y[M,N]: GEMM rows = K, inner = M.
    if (!x || !y || !z || M <= 0 || K <= 0 || N <= 0) return ASR_ERR_ARG;
    asr::GemmArgs g = gemm_args(x, y, z, K, M, N);
    g.sam = 1; g.sak = K;   // A(r, m) = x[m][r]
    return asr::gemm_launch(g, asr::EPI_NONE, asr_stream(s));
}
int asr_matmul_tb(const float* x, const float* y, float* z, int M, int K, int N, asr_stream_t s) {
    // z[M,N] = x[M,K] . y[N,K]^T
    if (!x || !y || !z || M <= 0 || K <= 0 || N <= 0) return ASR_ERR_ARG;
    asr::GemmArgs g = gemm_args(x, y, z, M, K, N);
    g.sbk = 1; g.sbn = K;   // B(k, n) = y[n][k]
    return asr::gemm_launch(g, asr::EPI_NONE, asr_stream(s));
}
int asr_matadd(const float* x, const float* y, float* z, int M, int N, float lambda, asr_stream_t s) {
    if (!x || !y || !z || M <= 0 || N <= 0) return ASR_ERR_ARG;
    return asr::axpy_launch(x, y, z, (long)M * N, lambda, asr_stream(s));
}
int asr_linear_fwd(const float* x, const float* W, const float* b, float* y, int M, int K, int N,
                   int epilogue, asr_stream_t s) {
    if (!x || !W || !y || M <= 0 || K <= 0 || N <= 0) return ASR_ERR_ARG;
    if (epilogue != ASR_EPI_NONE && !b) return ASR_ERR_ARG;
    asr::GemmArgs g = gemm_args(x, W, y, M, K, N);
    g.b1 = b;
    int epi;
    switch (epilogue) {
        case ASR_EPI_NONE: epi = asr::EPI_NONE; break;
        case ASR_EPI_BIAS: epi = asr::EPI_BIAS; break;
        case ASR_EPI_BIAS_RELU: epi = asr::EPI_BIAS_RELU; break;
        case ASR_EPI_BIAS_LOGSOFTMAX: epi = asr::EPI_LOGSOFTMAX; break;
        default: return ASR_ERR_ARG;
    }
    return asr::gemm_launch(g, epi, asr_stream(s));
}
int asr_rnn_cell_fwd(const float* x, const float* h_prev, const float* W_ih, const float* W_hh,
                     const float* b_ih, const float* b_hh, float* h_out, int B, int in, int H,
                     asr_stream_t s) {
    if (!x || !h_prev || !W_ih || !W_hh || !b_ih || !b_hh || !h_out || B <= 0 || in <= 0 || H <= 0)
        return ASR_ERR_ARG;
    asr::GemmArgs g = gemm_args(x, W_ih, h_out, B, in, H);
    g.A2 = h_prev; g.B2 = W_hh; g.K2 = H;
    g.b1 = b_ih; g.b2 = b_hh;
    return asr::gemm_launch(g, asr::EPI_DUAL_TANH, asr_stream(s));
}
// H <= 256: the VALU kernel (one utterance per CU, W_hh in registers) has
// the shortest step, ~0.9 us, but costs a whole CU per utterance; the MFMA
// kernel carries 16 utterances per CU at ~3.4 us per step (H = 256).  With
// B utterances on n CUs the VALU kernel needs ceil(B / n) rounds, the MFMA
// kernel ceil(B / 16n) rounds of ~3.7x the step: MFMA from B >= 4n on (and
// it leaves CUs free for concurrent work well before that).
// ASR_RNN_MFMA=0/1 forces the choice (A/B timing).
static std::atomic<int> g_rnn_recur_kind{ASR_RNN_RECUR_AUTO};   // asr_rnn_set_recurrence

static bool rnn_use_mfma(int B, int H) {
    if ((H & 15) != 0) return false;
    if (const char* f = getenv("ASR_RNN_MFMA")) return atoi(f) != 0;
    const int kind = asr_internal_rnn_kind >= 0 ? asr_internal_rnn_kind
                                                : g_rnn_recur_kind.load(std::memory_order_relaxed);
    if (kind != ASR_RNN_RECUR_AUTO) return kind == ASR_RNN_RECUR_MFMA;
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
        return false;
    return B >= 4 * ncu;
}

// Recurrence over a hid buffer that already holds the input projection
// P_t = x_t . W_ih, in place: hid[t] = tanh((P_t + h_{t-1}.W_hh) + (b_hh + b_ih)).
static int rnn_frames_eager(const float* h0, const float* W_hh, const float* b_ih, const float* b_hh,
                            float* const* hids, int nb, int T, int B, int H, hipStream_t st);

// The T per-frame launches of a (pointers, shape) recurrence, captured once
// into a HIP graph and replayed: the host then queues one graph launch per
// sequence instead of T kernel launches (C5: 2,000 per batch, BL: 200), and
// the device runs them back to back.  Captured at the second call with the
// same key (a one-off call runs eagerly), replayed on the caller's stream;
// never inside the caller's own stream capture (then the launches are
// captured into that graph as they are).  A small cache, evicting the least
// recently used.  ASR_RNN_GRAPH=0: always eager (A/B).
struct RecurGraphKey {
    int dev, T, B, H, nb;
    const void *h0, *W_hh, *b_ih, *b_hh;
    const void* hid[asr::STEP_MAXB];
    bool operator==(const RecurGraphKey& o) const {
        if (!(dev == o.dev && T == o.T && B == o.B && H == o.H && nb == o.nb && h0 == o.h0 && W_hh == o.W_hh &&
              b_ih == o.b_ih && b_hh == o.b_hh))
            return false;
        for (int j = 0; j < nb; j++)
            if (hid[j] != o.hid[j]) return false;
        return true;
    }
};
struct RecurGraph {
    RecurGraphKey key;
    int uses = 0;
    hipGraphExec_t exec = nullptr;
    unsigned long last = 0;
};
static std::mutex g_graph_mu;
static std::vector<RecurGraph> g_graphs;
static unsigned long g_graph_tick = 0;
constexpr size_t RECUR_GRAPH_CACHE = 8;

static int rnn_recurrence_frames(const float* h0, const float* W_hh, const float* b_ih,
                                 const float* b_hh, float* const* hids, int nb, int T, int B, int H,
                                 hipStream_t st) {
    const char* ge = getenv("ASR_RNN_GRAPH");
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if ((ge && ge[0] == '0') || T < 8 || hipStreamIsCapturing(st, &cap) != hipSuccess ||
        cap != hipStreamCaptureStatusNone)
        return rnn_frames_eager(h0, W_hh, b_ih, b_hh, hids, nb, T, B, H, st);
    RecurGraphKey key{};
    key.T = T; key.B = B; key.H = H; key.nb = nb;
    key.h0 = h0; key.W_hh = W_hh; key.b_ih = b_ih; key.b_hh = b_hh;
    for (int j = 0; j < nb; j++) key.hid[j] = hids[j];
    ASR_HIP_TRY(hipGetDevice(&key.dev));
    std::lock_guard<std::mutex> lock(g_graph_mu);
    RecurGraph* e = nullptr;
    for (auto& g : g_graphs)
        if (g.key == key) e = &g;
    if (!e) {
        if (g_graphs.size() >= RECUR_GRAPH_CACHE) {   // evict the least recently used
            auto lru = std::min_element(g_graphs.begin(), g_graphs.end(),
                                        [](const RecurGraph& a, const RecurGraph& b) { return a.last < b.last; });
            if (lru->exec) hipGraphExecDestroy(lru->exec);
            g_graphs.erase(lru);
        }
        g_graphs.push_back(RecurGraph{key});
        e = &g_graphs.back();
    }
    e->last = ++g_graph_tick;
    if (++e->uses < 2 && !e->exec && !asr_internal_graph_now)   // first use: eager (nothing captured for one-offs)
        return rnn_frames_eager(h0, W_hh, b_ih, b_hh, hids, nb, T, B, H, st);
    if (!e->exec) {
        hipStream_t cs;
        ASR_HIP_TRY(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
        hipGraph_t graph = nullptr;
        int rc = ASR_OK;
        hipError_t he = hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal);
        if (he == hipSuccess) {
            rc = rnn_frames_eager(h0, W_hh, b_ih, b_hh, hids, nb, T, B, H, cs);
            he = hipStreamEndCapture(cs, &graph);
        }
        if (he == hipSuccess && rc == ASR_OK) he = hipGraphInstantiate(&e->exec, graph, nullptr, nullptr, 0);
        if (graph) hipGraphDestroy(graph);
        hipStreamDestroy(cs);
        if (rc) return rc;
        if (he != hipSuccess) {   // no graph: stay eager for this key
            e->exec = nullptr;
            return rnn_frames_eager(h0, W_hh, b_ih, b_hh, hids, nb, T, B, H, st);
        }
    }
    ASR_HIP_TRY(hipGraphLaunch(e->exec, st));
    return ASR_OK;
}

static int rnn_recurrence(const float* h0, const float* W_hh, const float* b_ih,
                          const float* b_hh, float* hid, int T, int B, int H, hipStream_t st) {
    if (H <= 256) {
        if (rnn_use_mfma(B, H)) return asr::rnn_recur_mfma_launch(h0, W_hh, b_ih, b_hh, hid, T, B, H, st);
        return asr::rnn_recur_launch(h0, W_hh, b_ih, b_hh, hid, T, B, H, st);
    }
    // one launch for all T frames where every workgroup fits beside the rest
    const int rc = asr::rnn_recur_persist_launch(h0, W_hh, b_ih, b_hh, hid, T, B, H, asr_internal_persist_cus, st);
    if (rc != ASR_ERR_UNSUPPORTED) return rc;
    return rnn_recurrence_frames(h0, W_hh, b_ih, b_hh, &hid, 1, T, B, H, st);
}

// H > 256: one small-M step kernel per frame, h_t = tanh((P_t +
// h_{t-1}.W_hh) + bias) in place: MFMA with an 8-way K split when
// H % 128 == 0, else the VALU kernel with W_hh slices in LDS.
static int rnn_frames_eager(const float* h0, const float* W_hh, const float* b_ih, const float* b_hh,
                            float* const* hids, int nb, int T, int B, int H, hipStream_t st) {
    int rc = ASR_OK;
    if (nb > 1) {   // several batches per step (h0 = zeros): one MFMA step launch for all
        if (h0 || (H & 127) != 0 || (B & 15) != 0 || nb > asr::STEP_MAXB) return ASR_ERR_UNSUPPORTED;
        for (int t = 0; t < T && !rc; t++) {
            float* hts[asr::STEP_MAXB];
            const float* hps[asr::STEP_MAXB];
            for (int j = 0; j < nb; j++) {
                hts[j] = hids[j] + (size_t)t * B * H;
                hps[j] = t ? hids[j] + (size_t)(t - 1) * B * H : nullptr;
            }
            if (t == 0) {
                for (int j = 0; j < nb && !rc; j++) rc = asr::bias_tanh_launch(hts[j], b_ih, b_hh, (long)B * H, H, st);
            } else {
                rc = asr::rnn_step_mfma_multi_launch(hts, hps, nb, W_hh, b_ih, b_hh, B, H, st);
            }
        }
        return rc;
    }
    float* hid = hids[0];
    for (int t = 0; t < T; t++) {
        float* ht = hid + (size_t)t * B * H;
        const float* hp = t == 0 ? h0 : hid + (size_t)(t - 1) * B * H;
        if (!hp) {   // h_{-1} = 0 (RNN.h:15-16 zero-filled h_0s)
            rc = asr::bias_tanh_launch(ht, b_ih, b_hh, (long)B * H, H, st);
        } else if ((H & 127) == 0 && ((uintptr_t)hp & 15) == 0) {
            rc = asr::rnn_step_mfma_launch(ht, hp, W_hh, b_ih, b_hh, B, H, st);
        } else if ((H & 7) == 0) {
            rc = asr::rnn_step_launch(ht, hp, W_hh, b_ih, b_hh, B, H, st);
        } else {   // odd widths: the fused cell GEMM
            asr::GemmArgs g = gemm_args(hp, W_hh, ht, B, H, H);
            g.D = ht; g.b1 = b_ih; g.b2 = b_hh;
            rc = asr::gemm_launch(g, asr::EPI_ADD_TANH, st);
        }
        if (rc) return rc;
    }
    return ASR_OK;
}

int asr_set_dense_arith(int arith) {
    if (arith != ASR_DENSE_F32 && arith != ASR_DENSE_SPLIT_BF16) return ASR_ERR_ARG;
    asr::dense_arith_set(arith);
    return ASR_OK;
}

int asr_get_dense_arith(int* arith) {
    if (!arith) return ASR_ERR_ARG;
    *arith = asr::dense_arith();
    return ASR_OK;
}

int asr_rnn_set_recurrence(int kind) {
    if (kind != ASR_RNN_RECUR_AUTO && kind != ASR_RNN_RECUR_VALU && kind != ASR_RNN_RECUR_MFMA) return ASR_ERR_ARG;
    g_rnn_recur_kind.store(kind, std::memory_order_relaxed);
    return ASR_OK;
}

int asr_rnn_get_recurrence(int* kind) {
    if (!kind) return ASR_ERR_ARG;
    *kind = g_rnn_recur_kind.load(std::memory_order_relaxed);
    return ASR_OK;
}

int asr_rnn_fwd(const float* x, const float* h0, const float* W_ih, const float* W_hh,
                const float* b_ih, const float* b_hh, float* hid, int T, int B, int in, int H,
                asr_stream_t s) {
    if (!x || !W_ih || !W_hh || !b_ih || !b_hh || !hid || T <= 0 || B <= 0 || in <= 0 || H <= 0)
        return ASR_ERR_ARG;
    if (x == hid) return ASR_ERR_ARG;
    const hipStream_t st = asr_stream(s);
    // 1. input projection for all T at once: hid = x . W_ih   ([T*B, in] x [in, H])
    int rc = asr::gemm_launch(gemm_args(x, W_ih, hid, T * B, in, H), asr::EPI_NONE, st);
    if (rc) return rc;
    // 2. recurrence, in place over hid.
    return rnn_recurrence(h0, W_hh, b_ih, b_hh, hid, T, B, H, st);
}

int asr_rnn_recur_fwd(const float* h0, const float* W_hh, const float* b_ih, const float* b_hh,
                      float* hid, int T, int B, int H, asr_stream_t s) {
    if (!W_hh || !b_ih || !b_hh || !hid || T <= 0 || B <= 0 || H <= 0) return ASR_ERR_ARG;
    return rnn_recurrence(h0, W_hh, b_ih, b_hh, hid, T, B, H, asr_stream(s));
}

int asr_rnn_persist_stats(long long* launches, long long* recoveries) {
    return asr::rnn_persist_stats(launches, recoveries);
}

int asr_rnn_emit_fwd(const float* h0, const float* W_hh, const float* b_ih, const float* b_hh,
                     const float* W_out, const float* b_out, const float* P, float* hiddens,
                     float* emis, int T, int B, int H, int V, asr_stream_t s) {
    if (!W_hh || !b_ih || !b_hh || !W_out || !b_out || !P || !emis || T <= 0 || B <= 0 || H <= 0 || V <= 0)
        return ASR_ERR_ARG;
    if ((const float*)emis == P || (hiddens && (hiddens == emis || hiddens == h0))) return ASR_ERR_ARG;
    return asr::rnn_emit_mfma_launch(h0, W_hh, b_ih, b_hh, P, hiddens, W_out, b_out, emis, T, B, H, V,
                                     asr_stream(s));
}

size_t asr_rnn_bidir_workspace_bytes(int T, int B, int H) {
    if (T <= 0 || B <= 0 || H <= 0) return 0;
    return 2 * (size_t)T * B * H * sizeof(float);
}

int asr_rnn_bidir_fwd(const float* x, const float* h0, const float* const W_ih[2],
                      const float* const W_hh[2], const float* const b_ih[2],
                      const float* const b_hh[2], float* out, void* work, int T, int B, int in,
                      int H, asr_stream_t s) {
    if (!x || !W_ih || !W_hh || !b_ih || !b_hh || !out || !work || T <= 0 || B <= 0 || in <= 0 ||
        H <= 0)
        return ASR_ERR_ARG;
    for (int d = 0; d < 2; d++)
        if (!W_ih[d] || !W_hh[d] || !b_ih[d] || !b_hh[d]) return ASR_ERR_ARG;
    if ((H & 3) || (((uintptr_t)out | (uintptr_t)work) & 15)) return ASR_ERR_UNSUPPORTED;
    const size_t n = (size_t)T * B * H;
    float* hf = static_cast<float*>(work);
    float* hr = hf + n;
    if ((const float*)out == x || (hf < x + (size_t)T * B * in && x < hr + n)) return ASR_ERR_ARG;
    const hipStream_t st = asr_stream(s);
    // Both input projections on the caller's stream (one GEMM each, full chip);
    // the reverse direction's P is then flipped in time so that its recurrence
    // is the forward recurrence over hr.
    int rc = asr::gemm_launch(gemm_args(x, W_ih[0], hf, T * B, in, H), asr::EPI_NONE, st);
    if (!rc) rc = asr::gemm_launch(gemm_args(x, W_ih[1], hr, T * B, in, H), asr::EPI_NONE, st);
    if (!rc) rc = asr::time_reverse_launch(hr, T, (long)B * H, st);
    if (rc) return rc;
    // The two recurrences are independent and each is latency-bound on a few
    // CUs: the reverse one runs on a side stream of this device.
    static thread_local hipStream_t side[64] = {};
    static thread_local hipEvent_t ev_fork[64] = {}, ev_join[64] = {};
    int dev = 0;
    ASR_HIP_TRY(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return ASR_ERR_UNSUPPORTED;
    if (!side[dev]) {
        ASR_HIP_TRY(hipStreamCreateWithFlags(&side[dev], hipStreamNonBlocking));
        ASR_HIP_TRY(hipEventCreateWithFlags(&ev_fork[dev], hipEventDisableTiming));
        ASR_HIP_TRY(hipEventCreateWithFlags(&ev_join[dev], hipEventDisableTiming));
    }
    ASR_HIP_TRY(hipEventRecord(ev_fork[dev], st));
    ASR_HIP_TRY(hipStreamWaitEvent(side[dev], ev_fork[dev], 0));
    rc = rnn_recurrence(h0 ? h0 + (size_t)B * H : nullptr, W_hh[1], b_ih[1], b_hh[1], hr, T, B, H,
                        side[dev]);
    // Join the side stream back into the caller's stream on every path,
    // errors included: kernels already queued there still write `work`,
    // which the caller may free once this returns.
    const hipError_t je = hipEventRecord(ev_join[dev], side[dev]);
    if (je != hipSuccess) {
        hipStreamSynchronize(side[dev]);
        ASR_HIP_TRY(je);
    }
    if (!rc) rc = rnn_recurrence(h0, W_hh[0], b_ih[0], b_hh[0], hf, T, B, H, st);
    ASR_HIP_TRY(hipStreamWaitEvent(st, ev_join[dev], 0));
    if (rc) return rc;
    return asr::bidir_concat_launch(hf, hr, out, T, B, H, st);
}

}  // extern "C"

// ---------------------------------------------------------------- CTC handle
struct asr_ctc {
    int V, beam, blank, K, kcap, waves_override;
    int cu_mode = 0;                // ASR_CTC_SEMANTICS_CUDA
    int ncu = 0;                    // compute units of the handle's device (auto_waves)
    int occ8 = -1, occ4 = -1;       // workgroups per CU of the 8- / 4-wave kernels (-1: not queried)
    int occw = 0;                   // ... of the one-wave kernel (0: not a candidate)
    int concurrency = 1;            // decodes of this size in flight on the device (asr_ctc_set_concurrency)
    std::vector<int32_t> codes;
    uint64_t blank_less;
    int device;
    // workspace (device)
    int capB = 0, capT = 0;
    int4* d_nodes = nullptr;
    int *d_fin_n = nullptr, *d_fin_node = nullptr, *d_status = nullptr;   // d_status: in d_res
    uint64_t* d_fin_tail = nullptr;
    int* d_chain = nullptr;         // traceback scratch [B][2][T/4+1]
    double* d_fin_score = nullptr;
    // per-decode results, packed so that one copy brings them to the host:
    // [score f64 x B][len i32 x B][status i32 x B][labels i32 x B x T]
    unsigned char* d_res = nullptr;
    int *d_best_lab = nullptr, *d_best_len = nullptr;
    double* d_best_score = nullptr;
    int* d_codes = nullptr;
    int *d_all_lab = nullptr, *d_all_len = nullptr, *d_all_ts = nullptr;
    int ts = 0;                      // timesteps mode (asr_ctc_set_timesteps)
    int4* d_nodes_ts = nullptr;      // [B][T*kcap] append frames per node record
    uint64_t* d_fin_ts = nullptr;    // [B][kcap][2] append frames of the final tails
    uint32_t* d_tile0 = nullptr;     // [B][T] first label tile per frame (wide kernel, V > 65)
    bool tile0 = true;               // precompute first tiles (ASR_CTC_TILE0=0: in-kernel, for A/B timing)
    bool tile0_ext = false;          // the caller queues the precompute (asr_internal_ctc_tile0)
    int diag = 0;                    // CtcArgs::diag (ASR_CTC_WIDE_FALLBACK=1: bit 0, ASR_CTC_WIDE_ADOPT_CAP=1: bit 1)
    size_t cap_all = 0;
    // pinned host mirrors of the best-path results
    unsigned char* h_res = nullptr;   // pinned mirror of d_res
    unsigned char* hd_res = nullptr;  // h_res as the device sees it (the kernels write there directly)
    bool res_direct = true;           // kernels write results into h_res (else: copy d_res)
    int *h_best_lab = nullptr, *h_best_len = nullptr, *h_status = nullptr;
    double* h_best_score = nullptr;
    // last decode
    bool have = false;
    int lastT = 0, lastB = 0, last_waves = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t ev_res = nullptr;    // traceback done, results in the pinned mirror
    hipEvent_t ev_dec = nullptr;    // decode done (fork to the result stream)
    hipStream_t res_stream = nullptr;   // traceback + result copy (asr_ctc_set_result_stream); null: the decode's
    bool res_fork = false;          // a traceback was queued on res_stream
    asr::CtcArgs args{};
    uint64_t* d_stamps = nullptr;   // diagnostic build only
    int cap_stamps = 0;
    bool auto_cap = true;           // max_states chosen by the library
    asr_ctc* wide = nullptr;        // re-decode handle for tie overflow
    const float* last_emis = nullptr;
    long last_tstride = 0, last_ustride = 0;
    std::vector<int32_t> last_lengths;   // empty = all T
    int last_is_log = 0;
    int* d_lengths = nullptr;        // per-utterance frames (asr_ctc_decode_ex)
    int* h_lengths = nullptr;        // pinned staging
    int cap_len = 0;
    // segmented decode (asr_ctc_decode_segment)
    int seg_next = 0;                // first frame of the next segment (0: none in progress)
    int seg_waves = 0;               // the segmented decode's kernel (one-wave list kernel or wide)
    int seg_T = 0, seg_B = 0, seg_is_log = 0;
    long seg_fs = 0, seg_us = 0;
    unsigned char* d_seg = nullptr;  // [B][seg_bytes] saved beams
    size_t cap_seg = 0;
    std::vector<hipEvent_t> seg_ev;  // (start, end) of each segment's kernel, for last_kernel_ms
    int nseg = 0;                    // segments of the current / last segmented decode
};

namespace {

asr::CtcGeom plan(const asr_ctc* h, int waves);

// Automatic schedule for a batch of B utterances (one workgroup each).
// The 8-wave kernel is the fastest per utterance but, at 153
// VGPRs x 2 waves per SIMD, one workgroup fills a CU; the 4-wave kernel fits
// three per CU (167 VGPRs, ctc_waves_per_eu).  Measured on MI355X, C4 shapes
// on the bench's emissions (tools/occupancy_sweep.py, profiles/r03/): per-
// utterance frame time relative to the 8-wave kernel alone on a CU is 1.13
// (4 waves alone), 1.25 (two 4-wave workgroups sharing a CU), 1.46 (three).
// With u = ceil(B / ncu) utterances per CU the 8-wave kernel runs u rounds;
// the 4-wave kernel floor(u / n) rounds of n per CU plus one of the rest:
// 4 waves whenever that is shorter, i.e. from B > ncu on.  The per-CU fit n
// is the runtime's occupancy query of the instantiated kernels (registers,
// LDS, wave slots), so a layout that does not fit several to a CU keeps 8
// waves.  ASR_CTC_WAVES_LIST (-1) selects the one-wave list kernel
// (ctc_wave_kernel.inc), faster only on peaked emissions.  valid_waves
// lowers an explicit count where a narrower instantiation is required.
constexpr double REL_4W[4] = {0.0, 1.13, 1.25, 1.46};
double rel_4w(int n) { return n <= 3 ? REL_4W[n] : REL_4W[3] * n / 3.0; }
// The one-wave kernel (ctc_wave_kernel.inc, beam capacity <= 64): per-
// utterance frame time relative to the 8-wave kernel alone with n of them
// on a CU (measured, tools/occupancy_sweep.py, profiles/r03/: 5.86 / 6.00 /
// 6.24 / 7.09 / 8.09 / 8.12 / 9.35 / 11.13 us per frame at 1 / 2 / 3 / 4 / 6 /
// 8 / 12 / 16 per CU against 3.18 us; between the points linear).  Alone it
// is ~1.8x slower than the 8-wave kernel, but a CU holds 16 of them: from 4
// utterances per CU on it decodes a batch fastest.
constexpr double REL_W[17] = {0.0,  1.84, 1.89, 1.96, 2.23, 2.39, 2.54, 2.55, 2.55,
                              2.65, 2.74, 2.84, 2.94, 3.08, 3.22, 3.36, 3.50};
// Two rows per lane (beam capacity 65-128, C3's beam 100): against the
// 8-wave kernel alone (4.79 us per frame), 2.69 / 2.82 / 2.88 / 3.43 at 1 / 2
// / 4 / 8 per CU (tools/occupancy_sweep.py --beam 100, profiles/r04/), a CU
// holding ~9 (LDS); between the points linear.
constexpr double REL_W2[10] = {0.0, 2.69, 2.82, 2.85, 2.88, 3.02, 3.16, 3.29, 3.43, 3.57};
double rel_w(int n, int kcap) {
    if (kcap > 64) return n <= 9 ? REL_W2[n] : REL_W2[9] * n / 9.0;
    return n <= 16 ? REL_W[n] : REL_W[16] * n / 16.0;
}
int auto_waves(asr_ctc* h, int B) {
    if (h->cu_mode || h->V + 1 > 64 || h->V + 1 <= 8 || B <= 0) return 8;
    if (h->occ8 < 0) {   // once per handle: the layout is fixed at creation
        h->occ8 = asr::ctc_occupancy(plan(h, 8), 8);
        h->occ4 = asr::ctc_occupancy(plan(h, 4), 4);
        h->occw = h->kcap <= 128 && asr::ctc_wave_supported(plan(h, -1), 0) ? asr::ctc_occupancy_wave(plan(h, -1)) : 0;
    }
    if (h->ncu <= 0 || h->occ8 < 1 || h->occ4 < 1) return 8;
    const int u = (B + h->ncu - 1) / h->ncu;   // utterances on the busiest CU
    const double cost8 = (double)((u + h->occ8 - 1) / h->occ8);
    const int n4 = h->occ4;
    const double cost4 = (u / n4) * rel_4w(n4) + (u % n4 ? rel_4w(u % n4) : 0.0);
    const int nw = h->occw;
    const double costw = nw >= 1 ? (u / nw) * rel_w(nw, h->kcap) + (u % nw ? rel_w(u % nw, h->kcap) : 0.0) : 1e30;
    if (costw < cost4 && costw < cost8) return ASR_CTC_WAVES_LIST;
    return cost4 < cost8 ? 4 : 8;
}

// A (waves, vocab class, rows/thread) combination that ctc_beam_v*.hip instantiates.
int valid_waves(const asr_ctc* h, int waves) {
    if (waves < 0) return asr::ctc_wave_supported(plan(h, 0), h->cu_mode) ? -1 : valid_waves(h, 8);
    if (h->V + 1 <= 8 && waves == 8) return 4;   // 8 waves need >= 2 columns per thread
    if (h->kcap > 128 && waves < 4) return 4;   // 4 rows per thread only with 4 or 8 waves
    if (h->V + 1 > 32 && waves == 1) return 2;
    return waves;
}

asr::CtcGeom plan(const asr_ctc* h, int waves) {
    asr::CtcGeom g{};
    g.V = h->V;
    g.blank = h->blank;
    g.K = h->K;
    g.kcap = h->kcap;
    g.sb = (h->V + 1) <= 32 ? 5 : 6;
    g.lbits = (h->V + 1) <= 64 ? 8 : 16;   // labels in node records: 8 x 8 bits or 4 x 16 bits
    (void)waves;
    g.ch = std::max(1, std::min(32, 1024 / h->V));   // chunk = ch*V <= 1024 emissions (16 per thread at 1 wave)
    g.ht = 4 * asr::ctc_row_capacity(h->kcap);
    g.ts = h->ts ? 1 : 0;
    return g;
}

void free_ws(asr_ctc* h) {
    hipFree(h->d_nodes); hipFree(h->d_fin_n); hipFree(h->d_fin_node);
    hipFree(h->d_fin_tail); hipFree(h->d_chain);
    h->d_fin_tail = nullptr; h->d_chain = nullptr;
    hipFree(h->d_fin_score); hipFree(h->d_res);
    hipFree(h->d_nodes_ts); hipFree(h->d_fin_ts); hipFree(h->d_tile0);
    h->d_nodes_ts = nullptr; h->d_fin_ts = nullptr; h->d_tile0 = nullptr;
    hipHostFree(h->h_res);
    h->d_res = nullptr; h->h_res = nullptr; h->hd_res = nullptr;
    h->d_nodes = nullptr; h->d_fin_n = h->d_fin_node = h->d_status = nullptr;
    h->d_fin_score = nullptr; h->d_best_lab = h->d_best_len = nullptr; h->d_best_score = nullptr;
    h->h_best_lab = h->h_best_len = h->h_status = nullptr; h->h_best_score = nullptr;
    h->capB = h->capT = 0;
}

// The wide kernel (V + 1 > 64) takes every frame's first tile from a
// precompute pass when the vocabulary spans more than one tile.
bool use_tile0(const asr_ctc* h) { return h->tile0 && h->V - 1 > 64 && h->V <= asr::WIDE_VMAX; }

int ensure_ws(asr_ctc* h, int B, int T) {
    if (B <= h->capB && T <= h->capT) {
        if (h->ts && !h->d_nodes_ts) {   // timesteps switched on after the workspace was sized
            const size_t kc = (size_t)h->kcap;
            ASR_HIP_TRY(hipMalloc(&h->d_nodes_ts, sizeof(int4) * (size_t)h->capB * h->capT * kc));
            ASR_HIP_TRY(hipMalloc(&h->d_fin_ts, sizeof(uint64_t) * 2 * (size_t)h->capB * kc));
        }
        return ASR_OK;
    }
    // Grow geometrically in B and T so that repeated decodes do not thrash.
    const int nB = std::max(B, h->capB), nT = std::max(T, h->capT);
    hipDeviceSynchronize();
    free_ws(h);
    const size_t kc = (size_t)h->kcap;
    ASR_HIP_TRY(hipMalloc(&h->d_nodes, sizeof(int4) * (size_t)nB * nT * kc));
    ASR_HIP_TRY(hipMalloc(&h->d_fin_tail, sizeof(uint64_t) * nB * kc));
    ASR_HIP_TRY(hipMalloc(&h->d_chain, sizeof(int) * (size_t)nB * 2 * (nT / 4 + 1)));
    ASR_HIP_TRY(hipMalloc(&h->d_fin_n, sizeof(int) * nB));
    ASR_HIP_TRY(hipMalloc(&h->d_fin_node, sizeof(int) * nB * kc));
    ASR_HIP_TRY(hipMalloc(&h->d_fin_score, sizeof(double) * nB * kc));
    const size_t res_bytes = 16 * (size_t)nB + sizeof(int) * (size_t)nB * nT;
    ASR_HIP_TRY(hipMalloc(&h->d_res, res_bytes));
    ASR_HIP_TRY(hipHostMalloc((void**)&h->h_res, res_bytes, 0));
    ASR_HIP_TRY(hipHostGetDevicePointer((void**)&h->hd_res, h->h_res, 0));
    if (h->ts) {
        ASR_HIP_TRY(hipMalloc(&h->d_nodes_ts, sizeof(int4) * (size_t)nB * nT * kc));
        ASR_HIP_TRY(hipMalloc(&h->d_fin_ts, sizeof(uint64_t) * 2 * (size_t)nB * kc));
    }
    if (use_tile0(h)) ASR_HIP_TRY(hipMalloc(&h->d_tile0, asr::ctc_tile0_bytes(nB, nT)));
    h->capB = nB;
    h->capT = nT;
    return ASR_OK;
}

// String order of two label sequences under the symbol codes.
bool code_less(const asr_ctc* h, const int* a, int la, const int* b, int lb) {
    const int n = std::min(la, lb);
    for (int i = 0; i < n; i++) {
        const int ca = h->codes[a[i]], cb = h->codes[b[i]];
        if (ca != cb) return ca < cb;
    }
    return la < lb;
}

// Status word of an utterance: bit 0 = beam overflow, bit 1 = self-check.
int status_code(const int* status, int B) {
    int any = 0;
    for (int b = 0; b < B; b++) any |= status[b];
    if (any & 2) return ASR_ERR_INTERNAL;
    if (any & 1) return ASR_ERR_BEAM_OVERFLOW;
    return ASR_OK;
}

}  // namespace

int asr_internal_rnn_recur_multi(const float* W_hh, const float* b_ih, const float* b_hh, float* const* hids,
                                 int nb, int T, int B, int H, hipStream_t st) {
    if (nb == 1) return rnn_recurrence(nullptr, W_hh, b_ih, b_hh, hids[0], T, B, H, st);
    if (H <= 256) return ASR_ERR_UNSUPPORTED;   // the register-resident kernels: one batch each
    return rnn_recurrence_frames(nullptr, W_hh, b_ih, b_hh, hids, nb, T, B, H, st);
}

int asr_internal_ctc_wave_occupancy(asr_ctc* h) {
    if (!h || h->cu_mode || h->ts || !asr::ctc_wave_supported(plan(h, -1), 0)) return 0;
    return asr::ctc_occupancy_wave(plan(h, -1));
}

int asr_internal_ctc_tile0_external(asr_ctc* h, int B, int T) {
    if (!h || B < 1 || T < 1) return ASR_ERR_ARG;
    if (!use_tile0(h)) return ASR_ERR_UNSUPPORTED;
    if (int rc = ensure_ws(h, B, T)) return rc;
    h->tile0_ext = true;
    return ASR_OK;
}

int asr_internal_ctc_tile0(asr_ctc* h, const float* d_emis, int T, int t0, int t1, int B, long frame_stride,
                           long utt_stride, hipStream_t s) {
    if (!h || !d_emis || !h->tile0_ext || t0 < 0 || t1 <= t0 || t1 > T || B < 1) return ASR_ERR_ARG;
    if (B > h->capB || T > h->capT || !h->d_tile0) return ASR_ERR_STATE;   // sized by _external
    asr::CtcArgs a{};
    a.g = plan(h, 8);   // the wide kernel's geometry (V, blank)
    a.emis = d_emis;
    a.tstride = frame_stride;
    a.ustride = utt_stride;
    a.T = T;
    a.B = B;
    a.t0 = t0;
    a.t1 = t1;
    a.tile0 = h->d_tile0;
    return asr::ctc_launch_tile0(a, s);
}

extern "C" {

int asr_ctc_create(const int32_t* codes, int V, int beam_width, int blank_id, int max_states,
                   asr_ctc_t** out) {
    if (!out) return ASR_ERR_ARG;
    *out = nullptr;
    if (V < 2 || beam_width < 1 || blank_id < 0 || blank_id >= V) return ASR_ERR_ARG;
    if (V > asr::WIDE_VMAX) return ASR_ERR_UNSUPPORTED;
    asr_ctc* h = new asr_ctc();
    h->V = V;
    h->beam = beam_width;
    h->blank = blank_id;
    h->K = beam_width + 1;
    h->codes.resize(V);
    for (int v = 0; v < V; v++) h->codes[v] = codes ? codes[v] : v;
    for (int v = 0; v < V; v++)
        for (int u = 0; u < v; u++)
            if (h->codes[u] == h->codes[v]) { delete h; return ASR_ERR_ARG; }
    h->blank_less = 0;
    for (int v = 0; v < V; v++)
        if (v < 64 && h->codes[blank_id] < h->codes[v]) h->blank_less |= 1ull << v;
    // Automatic capacity: K plus room for ties at the cutoff; an overflow is
    // detected on the device and the decode is re-run with more room.
    h->auto_cap = max_states <= 0;
    int kcap = max_states > 0 ? max_states : h->K + std::max(8, h->K / 8);
    if (kcap < h->K) { delete h; return ASR_ERR_ARG; }
    kcap = (kcap + 31) & ~31;
    if (kcap > 256) { delete h; return ASR_ERR_UNSUPPORTED; }
    h->kcap = kcap;
    h->waves_override = 0;
    if (const char* w = getenv("ASR_CTC_WAVES")) h->waves_override = atoi(w);
    if (const char* t0 = getenv("ASR_CTC_TILE0")) h->tile0 = atoi(t0) != 0;
    if (const char* fb = getenv("ASR_CTC_WIDE_FALLBACK")) h->diag = atoi(fb) != 0 ? 1 : 0;
    // ASR_CTC_WIDE_ADOPT_CAP=1 (tests): the wide kernel lists no orphan-filter
    // hit for the block-wide adoption scan: every hit takes the one-thread
    // scan (the path past 128 hits per frame)
    if (const char* ac = getenv("ASR_CTC_WIDE_ADOPT_CAP")) h->diag |= atoi(ac) != 0 ? 2 : 0;
    if (asr::ctc_lds_bytes(plan(h, 8)) > 160 * 1024) { delete h; return ASR_ERR_UNSUPPORTED; }
    int rc = asr::ctc_set_max_lds();
    if (rc) { delete h; return rc; }
    if (hipGetDevice(&h->device) != hipSuccess ||
        hipDeviceGetAttribute(&h->ncu, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess ||
        hipMalloc(&h->d_codes, sizeof(int) * V) != hipSuccess ||
        hipMemcpy(h->d_codes, h->codes.data(), sizeof(int) * V, hipMemcpyHostToDevice) != hipSuccess ||
        hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_res, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_dec, hipEventDisableTiming) != hipSuccess) {
        delete h;
        return ASR_ERR_HIP;
    }
    *out = h;
    return ASR_OK;
}

int asr_ctc_destroy(asr_ctc_t* h) {
    if (!h) return ASR_OK;
    hipDeviceSynchronize();
    free_ws(h);
    hipFree(h->d_codes);
    hipFree(h->d_lengths);
    hipHostFree(h->h_lengths);
    hipFree(h->d_all_lab);
    hipFree(h->d_all_len);
    hipFree(h->d_all_ts);
    hipFree(h->d_stamps);
    hipFree(h->d_seg);
    for (auto e : h->seg_ev) hipEventDestroy(e);
    if (h->wide) asr_ctc_destroy(h->wide);
    if (h->ev0) hipEventDestroy(h->ev0);
    if (h->ev1) hipEventDestroy(h->ev1);
    if (h->ev_res) hipEventDestroy(h->ev_res);
    if (h->ev_dec) hipEventDestroy(h->ev_dec);
    delete h;
    return ASR_OK;
}

int asr_ctc_set_semantics(asr_ctc_t* h, int semantics) {
    if (!h || (semantics != ASR_CTC_SEMANTICS_CPU && semantics != ASR_CTC_SEMANTICS_CUDA))
        return ASR_ERR_ARG;
    h->cu_mode = semantics == ASR_CTC_SEMANTICS_CUDA ? 1 : 0;
    h->K = h->cu_mode ? h->beam : h->beam + 1;   // exactly beam states vs beam+1 and ties
    h->have = false;
    return ASR_OK;
}

int asr_ctc_set_result_stream(asr_ctc_t* h, asr_stream_t s) {
    if (!h) return ASR_ERR_ARG;
    h->res_stream = s ? asr_stream(s) : nullptr;
    return ASR_OK;
}

int asr_ctc_set_timesteps(asr_ctc_t* h, int on) {
    if (!h) return ASR_ERR_ARG;
    const int prev = h->ts;
    h->ts = on ? 1 : 0;
    // the workgroup kernel's timestep arrays are allocated only in this mode
    if (h->ts && h->V + 1 <= 64 && asr::ctc_lds_bytes(plan(h, 8)) > 160 * 1024) {
        h->ts = prev;
        return ASR_ERR_UNSUPPORTED;
    }
    if (h->wide) h->wide->ts = h->ts;
    if (h->ts != prev) h->occ8 = h->occ4 = -1;   // the layout changed: re-query the occupancy
    h->have = false;
    return ASR_OK;
}

int asr_ctc_set_concurrency(asr_ctc_t* h, int n) {
    if (!h || n < 1) return ASR_ERR_ARG;
    h->concurrency = n;
    return ASR_OK;
}

int asr_ctc_set_waves(asr_ctc_t* h, int waves) {
    if (!h || !(waves == ASR_CTC_WAVES_LIST || waves == 0 || waves == 1 || waves == 2 || waves == 4 ||
                waves == 8))
        return ASR_ERR_ARG;
    h->waves_override = waves;
    return ASR_OK;
}

int asr_ctc_get_config(asr_ctc_t* h, int* max_states, int* waves, int* lds_bytes) {
    if (!h) return ASR_ERR_ARG;
    // the last decode's schedule; before the first decode, that of a batch
    // with at most one utterance per CU
    const int w = h->have ? h->last_waves
                          : valid_waves(h, h->waves_override && !h->cu_mode ? h->waves_override : auto_waves(h, 1));
    if (max_states) *max_states = h->kcap;
    if (waves) *waves = w;
    if (lds_bytes)
        *lds_bytes = (int)(w < 0 ? asr::ctc_lds_bytes_wave(plan(h, w)) : asr::ctc_lds_bytes(plan(h, w)));
    return ASR_OK;
}

int asr_ctc_decode(asr_ctc_t* h, const float* d_emis, int T, int B, int is_log, asr_stream_t s) {
    if (!h) return ASR_ERR_ARG;
    return asr_ctc_decode_ex(h, d_emis, T, B, (long)B * h->V, h->V, nullptr, is_log, s);
}

}  // extern "C"

namespace {

int finish_decode(asr_ctc* h, hipStream_t st, int B, int T, int waves);

// Queue the decode kernel (with its timing events) of frames [t0, t1).
int launch_decode_events(asr_ctc* h, int waves, hipStream_t st, bool segmented) {
    hipEvent_t e0 = h->ev0, e1 = h->ev1;
    if (segmented) {   // one event pair per segment; last_kernel_ms sums them
        const size_t need = 2 * (size_t)(h->nseg + 1);
        while (h->seg_ev.size() < need) {
            hipEvent_t e = nullptr;
            ASR_HIP_TRY(hipEventCreate(&e));
            h->seg_ev.push_back(e);
        }
        e0 = h->seg_ev[2 * h->nseg];
        e1 = h->seg_ev[2 * h->nseg + 1];
        h->nseg++;
    }
    ASR_HIP_TRY(hipEventRecord(e0, st));
    int rc = asr::ctc_launch_decode(h->args, waves, st);
    if (rc) return rc;
    ASR_HIP_TRY(hipEventRecord(e1, st));
    return ASR_OK;
}

// The decode of frames [t0, t1) of T: a whole decode (0, T, !segmented) or
// one segment of asr_ctc_decode_segment.  Everything but the kernel launch
// is set up at the first frame; the traceback follows the last.
int decode_frames(asr_ctc* h, const float* d_emis, int T, int B, long frame_stride, long utt_stride,
                  const int32_t* h_lengths, int is_log, asr_stream_t s, int t0, int t1, bool segmented) {
    int rc = ASR_OK;
    const hipStream_t st = asr_stream(s);
    if (t0 > 0) {   // a later segment: the first one set everything up
        h->args.emis = d_emis;
        h->args.t0 = t0;
        h->args.t1 = t1;
        rc = launch_decode_events(h, h->seg_waves, st, true);
        if (rc) return rc;
        if (t1 < T) return ASR_OK;
        return finish_decode(h, st, B, T, h->seg_waves);
    }
    rc = ensure_ws(h, B, T);
    if (rc) return rc;
    const hipStream_t st0 = asr_stream(s);
    if (h_lengths) {   // stage the lengths through pinned memory (stream-ordered)
        if (h->cap_len < B) {
            hipStreamSynchronize(st0);
            hipFree(h->d_lengths);
            hipHostFree(h->h_lengths);
            h->d_lengths = nullptr; h->h_lengths = nullptr; h->cap_len = 0;
            ASR_HIP_TRY(hipMalloc(&h->d_lengths, sizeof(int) * B));
            ASR_HIP_TRY(hipHostMalloc((void**)&h->h_lengths, sizeof(int) * B, 0));
            h->cap_len = B;
        }
        ASR_HIP_TRY(hipStreamSynchronize(st0));   // the pinned copy may still be in flight
        std::memcpy(h->h_lengths, h_lengths, sizeof(int) * B);
        ASR_HIP_TRY(hipMemcpyAsync(h->d_lengths, h->h_lengths, sizeof(int) * B, hipMemcpyHostToDevice, st0));
    }
    // .cu-semantics kernels exist for the automatic wave count only; the
    // one-wave list kernel does not track timesteps
    const long Beff = std::min<long>((long)B * h->concurrency, 1L << 30);
    int waves = valid_waves(h, h->waves_override && !h->cu_mode ? h->waves_override : auto_waves(h, (int)Beff));
    if (h->ts && waves < 0) waves = valid_waves(h, 8);
    // segmented: the one-wave kernel, or the wide one for V > 63 (checked by the caller)
    if (segmented) waves = h->V + 1 > 64 ? 8 : ASR_CTC_WAVES_LIST;
    h->seg_waves = waves;
    asr::CtcArgs& a = h->args;
    a.g = plan(h, waves);
    a.emis = d_emis;
    a.tstride = frame_stride;
    a.ustride = utt_stride;
    a.lengths = h_lengths ? h->d_lengths : nullptr;
    a.T = T;
    a.B = B;
    a.is_log = is_log ? 1 : 0;
    a.cu_mode = h->cu_mode;
    a.blank_less = h->blank_less;
    a.codes = h->d_codes;
    a.nodes = h->d_nodes;
    a.fin_n = h->d_fin_n;
    a.fin_node = h->d_fin_node;
    a.fin_tail = h->d_fin_tail;
    a.fin_score = h->d_fin_score;
    a.nodes_ts = h->ts ? h->d_nodes_ts : nullptr;
    a.fin_ts = h->ts ? h->d_fin_ts : nullptr;
    a.tile0 = use_tile0(h) ? h->d_tile0 : nullptr;
    a.tile0_ext = a.tile0 && h->tile0_ext ? 1 : 0;
    a.diag = h->diag;
    a.t0 = 0;
    a.t1 = segmented ? t1 : T;
    a.seg_state = nullptr;
    a.seg_bytes = 0;
    if (segmented) {
        const size_t sb = waves < 0 ? asr::ctc_seg_bytes_wave(a.g) : asr::ctc_seg_bytes_wide(asr::ctc_row_capacity(a.g.kcap));
        const size_t need = sb * (size_t)B;
        if (h->cap_seg < need) {
            hipStreamSynchronize(st);
            hipFree(h->d_seg);
            h->d_seg = nullptr;
            h->cap_seg = 0;
            ASR_HIP_TRY(hipMalloc(&h->d_seg, need));
            h->cap_seg = need;
        }
        a.seg_state = h->d_seg;
        a.seg_bytes = (int)sb;
    }
    // packed result layout for this (B, T)
    // The decode and traceback kernels write the packed results either
    // straight into the pinned host buffer (default: no copy to queue — a
    // small device-to-host copy was measured to block the host until the
    // stream's earlier copies finish, 7-9 ms with several batches in
    // flight) or into d_res, copied behind the traceback (A/B).
    unsigned char* const res = h->res_direct ? h->hd_res : h->d_res;
    h->d_best_score = reinterpret_cast<double*>(res);
    h->d_best_len = reinterpret_cast<int*>(res + 8 * (size_t)B);
    h->d_status = reinterpret_cast<int*>(res + 12 * (size_t)B);
    h->d_best_lab = reinterpret_cast<int*>(res + 16 * (size_t)B);
    h->h_best_score = reinterpret_cast<double*>(h->h_res);
    h->h_best_len = reinterpret_cast<int*>(h->h_res + 8 * (size_t)B);
    h->h_status = reinterpret_cast<int*>(h->h_res + 12 * (size_t)B);
    h->h_best_lab = reinterpret_cast<int*>(h->h_res + 16 * (size_t)B);
    a.status = h->d_status;
    a.best_lab = h->d_best_lab;
    a.best_len = h->d_best_len;
    a.best_score = h->d_best_score;
#if defined(ASR_CTC_STAMPS) || defined(ASR_CTC_WSTAMPS)
    if (h->cap_stamps < B) {
        hipFree(h->d_stamps);
        ASR_HIP_TRY(hipMalloc(&h->d_stamps, sizeof(uint64_t) * asr::NSTAMP * B));
        h->cap_stamps = B;
    }
    a.stamps = h->d_stamps;
#endif
    // the previous traceback of this handle (on the result stream) reads the
    // node records this decode overwrites
    if (h->res_fork) ASR_HIP_TRY(hipStreamWaitEvent(st, h->ev_res, 0));
    h->nseg = 0;
    h->have = false;
    h->last_emis = d_emis;
    h->last_tstride = frame_stride;
    h->last_ustride = utt_stride;
    h->last_lengths.assign(h_lengths ? h_lengths : nullptr, h_lengths ? h_lengths + B : nullptr);
    h->last_is_log = is_log ? 1 : 0;
    rc = launch_decode_events(h, waves, st, segmented);
    if (rc) return rc;
    if (segmented && t1 < T) return ASR_OK;
    return finish_decode(h, st, B, T, waves);
}

// After the last frames: the best-path traceback and its results.
int finish_decode(asr_ctc* h, hipStream_t st, int B, int T, int waves) {
    asr::CtcArgs& a = h->args;
    // traceback and result copy: on the result stream when one is set, so
    // that the decode stream can start the next batch at once
    const hipStream_t rs = h->res_stream ? h->res_stream : st;
    h->res_fork = rs != st;
    if (h->res_fork) {
        ASR_HIP_TRY(hipEventRecord(h->ev_dec, st));
        ASR_HIP_TRY(hipStreamWaitEvent(rs, h->ev_dec, 0));
    }
    int rc = asr::ctc_launch_best(a, h->d_codes, h->d_chain, rs);
    if (rc) return rc;
    // One copy of the packed results to the pinned mirror right behind the
    // traceback: asr_ctc_get_best waits for this event only, not for work the
    // caller queued on the stream afterwards (e.g. the next batch's decode).
    if (!h->res_direct)
        ASR_HIP_TRY(hipMemcpyAsync(h->h_res, h->d_res, 16 * (size_t)B + sizeof(int) * (size_t)B * T,
                                   hipMemcpyDeviceToHost, rs));
    ASR_HIP_TRY(hipEventRecord(h->ev_res, rs));
    h->have = true;
    h->lastT = T;
    h->lastB = B;
    h->last_waves = waves;
    h->stream = st;
    return ASR_OK;
}

}  // namespace

extern "C" {

int asr_ctc_decode_ex(asr_ctc_t* h, const float* d_emis, int T, int B, long frame_stride,
                      long utt_stride, const int32_t* h_lengths, int is_log, asr_stream_t s) {
    if (!h || !d_emis || T < 1 || B < 1 || frame_stride < 1 || utt_stride < 1) return ASR_ERR_ARG;
    if (h_lengths)
        for (int b = 0; b < B; b++)
            if (h_lengths[b] < 0 || h_lengths[b] > T) return ASR_ERR_ARG;
    // timesteps are stored as 16-bit frame numbers next to the labels (slot
    // tails, node records, ctc_trace.hip frame_field): frames >= 65536 would wrap
    if (h->ts && T > ASR_CTC_TS_MAX_T) return ASR_ERR_UNSUPPORTED;
    h->seg_next = 0;   // a whole decode ends any segmented one in progress
    return decode_frames(h, d_emis, T, B, frame_stride, utt_stride, h_lengths, is_log, s, 0, T, false);
}

int asr_ctc_decode_segment(asr_ctc_t* h, const float* d_emis, int T, int t0, int t1, int B, long frame_stride,
                           long utt_stride, const int32_t* h_lengths, int is_log, asr_stream_t s) {
    if (!h || !d_emis || T < 1 || B < 1 || frame_stride < 1 || utt_stride < 1 || t0 < 0 || t1 <= t0 || t1 > T)
        return ASR_ERR_ARG;
    if (t0 != h->seg_next) return ASR_ERR_STATE;   // segments in order, starting at frame 0
    if (t0 > 0 && (T != h->seg_T || B != h->seg_B || frame_stride != h->seg_fs || utt_stride != h->seg_us ||
                   (is_log ? 1 : 0) != h->seg_is_log))
        return ASR_ERR_ARG;
    if (t0 == 0) {
        if (h_lengths)
            for (int b = 0; b < B; b++)
                if (h_lengths[b] < 0 || h_lengths[b] > T) return ASR_ERR_ARG;
        // the one-wave kernel (V <= 63) or the wide kernel (V > 63) carries
        // the beam across segments: CPU semantics, no timesteps
        const bool wide = h->V + 1 > 64 && h->V <= asr::WIDE_VMAX;
        if (h->ts || h->cu_mode || (!wide && !asr::ctc_wave_supported(plan(h, ASR_CTC_WAVES_LIST), 0)))
            return ASR_ERR_UNSUPPORTED;
    }
    const int rc = decode_frames(h, d_emis, T, B, frame_stride, utt_stride, t0 == 0 ? h_lengths : nullptr,
                                 is_log, s, t0, t1, true);
    if (rc) {
        h->seg_next = 0;
        return rc;
    }
    if (t0 == 0) {
        h->seg_T = T;
        h->seg_B = B;
        h->seg_fs = frame_stride;
        h->seg_us = utt_stride;
        h->seg_is_log = is_log ? 1 : 0;
    }
    h->seg_next = t1 < T ? t1 : 0;
    return ASR_OK;
}

int asr_ctc_get_best(asr_ctc_t* h, int32_t* labels, int max_len, int32_t* lengths, double* logp) {
    if (!h || (!labels && max_len > 0)) return ASR_ERR_ARG;
    if (!h->have) return ASR_ERR_STATE;
    const int B = h->lastB, T = h->lastT;
    // the decode enqueued the traceback and the copy of its packed results
    ASR_HIP_TRY(hipEventSynchronize(h->ev_res));
    const int pitch = T;   // rows of the pinned label mirror
    const int stc = status_code(h->h_status, B);
    if (stc == ASR_ERR_BEAM_OVERFLOW && h->auto_cap && h->kcap < 256) {
        // More ties at the cutoff than room: decode again with twice the
        // capacity (rare; exact results, never a silent truncation).
        if (!h->wide) {
            int rc = asr_ctc_create(h->codes.data(), h->V, h->beam, h->blank,
                                    std::min(256, 2 * h->kcap), &h->wide);
            if (rc) return rc;
            h->wide->auto_cap = true;
            h->wide->cu_mode = h->cu_mode;
            h->wide->K = h->K;
            h->wide->ts = h->ts;
        }
        int rc = asr_ctc_decode_ex(h->wide, h->last_emis, T, B, h->last_tstride, h->last_ustride,
                                   h->last_lengths.empty() ? nullptr : h->last_lengths.data(),
                                   h->last_is_log, h->stream);
        if (rc) return rc;
        return asr_ctc_get_best(h->wide, labels, max_len, lengths, logp);
    }
    for (int b = 0; b < B; b++) {
        const int len = h->h_best_len[b];
        if (lengths) lengths[b] = len;
        if (logp) logp[b] = h->h_best_score[b];
        if (labels) {
            const int* fwd = h->h_best_lab + (size_t)b * pitch;
            const int n = std::min(len, max_len);
            if (n > 0) std::memcpy(labels + (size_t)b * max_len, fwd, sizeof(int) * (size_t)n);
        }
    }
    return stc;
}

int asr_ctc_get_beams(asr_ctc_t* h, int max_hyps, int max_len, int32_t* n_hyps, int32_t* lengths,
                      int32_t* labels, double* logp) {
    return asr_ctc_get_beams_ts(h, max_hyps, max_len, n_hyps, lengths, labels, logp, nullptr);
}

int asr_ctc_get_beams_ts(asr_ctc_t* h, int max_hyps, int max_len, int32_t* n_hyps, int32_t* lengths,
                         int32_t* labels, double* logp, int32_t* timesteps) {
    if (!h || max_hyps < 1 || max_len < 0) return ASR_ERR_ARG;
    if (timesteps && !h->ts) return ASR_ERR_STATE;   // the decode did not track them
    if (!h->have) return ASR_ERR_STATE;
    const int B = h->lastB, T = h->lastT, kc = h->kcap;
    const hipStream_t st = h->stream;
    const size_t need = (size_t)B * kc * T;
    if (need > h->cap_all) {
        hipStreamSynchronize(st);
        hipFree(h->d_all_lab);
        hipFree(h->d_all_len);
        hipFree(h->d_all_ts);
        h->d_all_lab = nullptr; h->d_all_len = nullptr; h->d_all_ts = nullptr; h->cap_all = 0;
        ASR_HIP_TRY(hipMalloc(&h->d_all_lab, sizeof(int) * need));
        ASR_HIP_TRY(hipMalloc(&h->d_all_len, sizeof(int) * (size_t)B * kc));
        h->cap_all = need;
    }
    if (timesteps && !h->d_all_ts) ASR_HIP_TRY(hipMalloc(&h->d_all_ts, sizeof(int) * h->cap_all));
    int rc = asr::ctc_launch_all(h->args, h->d_all_lab, h->d_all_len, timesteps ? h->d_all_ts : nullptr, st);
    if (rc) return rc;
    std::vector<int> fin_n(B), all_len((size_t)B * kc), status(B);
    std::vector<double> score((size_t)B * kc);
    std::vector<int> lab(need), tsv(timesteps ? need : 0);
    ASR_HIP_TRY(hipMemcpyAsync(fin_n.data(), h->d_fin_n, sizeof(int) * B, hipMemcpyDeviceToHost, st));
    if (!h->res_direct)
        ASR_HIP_TRY(hipMemcpyAsync(status.data(), h->d_status, sizeof(int) * B, hipMemcpyDeviceToHost, st));
    ASR_HIP_TRY(hipMemcpyAsync(score.data(), h->d_fin_score, sizeof(double) * B * kc, hipMemcpyDeviceToHost, st));
    ASR_HIP_TRY(hipMemcpyAsync(all_len.data(), h->d_all_len, sizeof(int) * B * kc, hipMemcpyDeviceToHost, st));
    ASR_HIP_TRY(hipMemcpyAsync(lab.data(), h->d_all_lab, sizeof(int) * need, hipMemcpyDeviceToHost, st));
    if (timesteps)
        ASR_HIP_TRY(hipMemcpyAsync(tsv.data(), h->d_all_ts, sizeof(int) * need, hipMemcpyDeviceToHost, st));
    ASR_HIP_TRY(hipStreamSynchronize(st));
    if (h->res_direct) std::memcpy(status.data(), h->h_status, sizeof(int) * B);   // written by the decode
    const int stc = status_code(status.data(), B);
    if (stc == ASR_ERR_BEAM_OVERFLOW && h->auto_cap && h->kcap < 256) {
        if (!h->wide) {
            rc = asr_ctc_create(h->codes.data(), h->V, h->beam, h->blank, std::min(256, 2 * h->kcap),
                                &h->wide);
            if (rc) return rc;
            h->wide->auto_cap = true;
            h->wide->cu_mode = h->cu_mode;
            h->wide->K = h->K;   // keeps doubling, up to 256 states
            h->wide->ts = h->ts;
        }
        rc = asr_ctc_decode_ex(h->wide, h->last_emis, T, B, h->last_tstride, h->last_ustride,
                               h->last_lengths.empty() ? nullptr : h->last_lengths.data(),
                               h->last_is_log, st);
        if (rc) return rc;
        return asr_ctc_get_beams_ts(h->wide, max_hyps, max_len, n_hyps, lengths, labels, logp, timesteps);
    }
    std::vector<std::vector<int>> fwd;
    for (int b = 0; b < B; b++) {
        const int n = fin_n[b];
        fwd.assign(n, {});
        std::vector<int> order(n);
        for (int i = 0; i < n; i++) {
            const int len = all_len[(size_t)b * kc + i];
            const int* src = lab.data() + ((size_t)b * kc + i) * T;
            fwd[i].assign(src, src + len);
            order[i] = i;
        }
        const double* sc = score.data() + (size_t)b * kc;
        std::sort(order.begin(), order.end(), [&](int x, int y) {
            if (sc[x] != sc[y]) return sc[x] > sc[y];
            return code_less(h, fwd[x].data(), (int)fwd[x].size(), fwd[y].data(), (int)fwd[y].size());
        });
        if (n_hyps) n_hyps[b] = n;
        for (int k = 0; k < std::min(n, max_hyps); k++) {
            const int i = order[k];
            const size_t base = (size_t)b * max_hyps + k;
            if (lengths) lengths[base] = (int)fwd[i].size();
            if (logp) logp[base] = sc[i];
            if (labels)
                for (int x = 0; x < (int)fwd[i].size() && x < max_len; x++)
                    labels[base * max_len + x] = fwd[i][x];
            if (timesteps) {
                const int* src = tsv.data() + ((size_t)b * kc + i) * T;
                for (int x = 0; x < (int)fwd[i].size() && x < max_len; x++) timesteps[base * max_len + x] = src[x];
            }
        }
    }
    return stc;
}

#if defined(ASR_CTC_STAMPS) || defined(ASR_CTC_WSTAMPS)
// Diagnostic build only: per-utterance phase clocks of the last decode.
int asr_debug_ctc_stamps(asr_ctc_t* h, uint64_t* out) {
    if (!h || !out || !h->have) return ASR_ERR_ARG;
    ASR_HIP_TRY(hipStreamSynchronize(h->stream));
    ASR_HIP_TRY(hipMemcpy(out, h->d_stamps, sizeof(uint64_t) * asr::NSTAMP * h->lastB, hipMemcpyDeviceToHost));
    return ASR_OK;
}
#endif

int asr_ctc_last_kernel_ms(asr_ctc_t* h, float* ms) {
    if (!h || !ms) return ASR_ERR_ARG;
    if (!h->have) return ASR_ERR_STATE;
    if (h->nseg > 0) {   // a segmented decode: the sum of its segments' kernels
        float sum = 0.f;
        for (int i = 0; i < h->nseg; i++) {
            float x = 0.f;
            ASR_HIP_TRY(hipEventSynchronize(h->seg_ev[2 * i + 1]));
            ASR_HIP_TRY(hipEventElapsedTime(&x, h->seg_ev[2 * i], h->seg_ev[2 * i + 1]));
            sum += x;
        }
        *ms = sum;
        return ASR_OK;
    }
    ASR_HIP_TRY(hipEventSynchronize(h->ev1));
    ASR_HIP_TRY(hipEventElapsedTime(ms, h->ev0, h->ev1));
    return ASR_OK;
}

}  // extern "C"
