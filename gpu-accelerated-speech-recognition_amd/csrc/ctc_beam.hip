// ============================================================================
// CTC prefix beam search on gfx950 — one workgroup per utterance, the whole
// beam resident in LDS for all T frames.
//
// Semantics: the reference CPU decoder CTCBeamSearch.cpp:50-187 with fixes
// F1-F3 in fp64 log domain:
//   * a state is (prefix q, flag ends-in-blank) — the reference's state
//     string "q" or "q$";
//   * every frame: extend all states by all labels (cpp:120-167), merge equal
//     states by log-sum-exp in the reference's std::set iteration order
//     (cpp:159-164), prune to the states scoring >= the (beam+1)-th largest
//     score (cpp:97-118 with F1/F2);
//   * finally strip the trailing blank and merge "q" with "q$" (cpp:169-187).
//
// Design:
//   * The beam is kept per PREFIX ("slot"): 64-bit prefix hash, parent-prefix
//     hash, last label, node id and the two state scores (not-blank, blank).
//   * Merging is structural instead of the reference's string sort
//     (CTCBeamSearch.cu:150-172, 460-489): a target (q+c, not) can only
//     receive from (q, not), (q, blank) and (q+c, not).  A per-frame LDS hash
//     table of live prefixes links each slot to its parent slot; candidate
//     rows are then generated with no search.  The fold order of those three
//     contributions is the reference's set order ("q" < "q$" ? "qc"), decided
//     by comparing the blank's code with c's code.
//   * Candidates live in an LDS array of order-preserving u64 keys; the
//     (beam+1)-th largest is found by MSB radix select over 8-bit digits with
//     an LDS histogram (typically 2-3 passes, early exit).
//   * Survivors are compacted with wave ballots into the next slot buffer;
//     new prefixes append one (parent node, label) record to a per-utterance
//     node table in HBM, node id = t*max_states + slot.  Strings are rebuilt
//     once at the end by chasing node ids (traceback kernels below).
//   * Emission rows are prefetched CH frames ahead into registers and staged
//     in LDS; the decode never waits on HBM inside a chunk.
// ============================================================================
#include "ctc_beam.h"

namespace asr {

constexpr uint32_t META_LAST = 0xFFFFu;
constexpr uint32_t META_HAS_NB = 1u << 16;
constexpr uint32_t META_HAS_B = 1u << 17;
constexpr uint32_t META_HAS_PAR = 1u << 18;
constexpr uint64_t ROOT_HASH = 0x243F6A8885A308D3ull;

// Hash of prefix q+c from the hash of q.  splitmix64 finaliser (a bijection)
// of h + phi*(c+1): distinct labels under one parent never collide; distinct
// parents collide with probability ~2^-63.  Bit 0 forced to 1 so that 0 marks
// an empty hash-table cell.
__device__ __forceinline__ uint64_t mix_hash(uint64_t h, uint32_t c) {
    uint64_t x = h + 0x9E3779B97F4A7C15ull * (uint64_t)(c + 1u);
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x | 1ull;
}

// log(exp(a) + exp(b)); identical formula to the oracle's lse().
__device__ __forceinline__ double lse2(double a, double b) {
    if (a == -INFINITY) return b;
    if (b == -INFINITY) return a;
    double m = fmax(a, b);
    return m + log1p(exp(-fabs(a - b)));
}

// Left fold with "first insert, then +=" semantics (cpp:159-164).
struct Fold {
    double acc;
    bool have;
    __device__ __forceinline__ Fold() : acc(0.0), have(false) {}
    __device__ __forceinline__ void push(double x) {
        if (have) acc = lse2(acc, x);
        else { acc = x; have = true; }
    }
};

__device__ __forceinline__ uint64_t shr64(uint64_t x, int s) { return s >= 64 ? 0ull : (x >> s); }

// ---------------------------------------------------------------- LDS plan
// Every LDS array is addressed as smem + a 32-bit byte offset so that the
// compiler emits ds_* instructions (a struct of generic pointers lowers to
// flat_* accesses and spills).
extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

struct LdsOff {
    uint32_t le;           // double[64]   log emissions of the current frame
    uint32_t ebuf;         // float[ch*V]  staged emission rows
    uint32_t h[2];         // u64[kcap]    prefix hash            (slot buffers 0/1)
    uint32_t hp[2];        // u64[kcap]    parent prefix hash (valid iff META_HAS_PAR)
    uint32_t snb[2];       // double[kcap] score of (q, not-blank)
    uint32_t sb[2];        // double[kcap] score of (q, blank)
    uint32_t node[2];      // int[kcap]    node id of q (-1 = empty prefix)
    uint32_t meta[2];      // u32[kcap]    last label | flags
    uint32_t cand;         // u64[kcap<<sb] candidate keys (0 = none)
    uint32_t plink;        // int[kcap]    parent slot or -1
    uint32_t child;        // u64[kcap]    bit c: live child prefix q+c exists
    uint32_t hkey;         // u64[ht]
    uint32_t hval;         // int[ht]
    uint32_t hist;         // u32[256]
    uint32_t red;          // u64[32]      cross-wave reduction scratch
    uint32_t misc;         // int[16]
    uint32_t total;
};

__host__ __device__ inline uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

__host__ __device__ inline LdsOff lds_plan(const CtcGeom& g) {
    LdsOff o;
    uint32_t off = 0;
    auto take = [&](uint32_t bytes) {
        uint32_t r = off;
        off = align16(off + bytes);
        return r;
    };
    const uint32_t kc = (uint32_t)g.kcap;
    o.le = take(64 * 8);
    o.ebuf = take((uint32_t)(g.ch * g.V) * 4);
    for (int k = 0; k < 2; k++) {
        o.h[k] = take(kc * 8);
        o.hp[k] = take(kc * 8);
        o.snb[k] = take(kc * 8);
        o.sb[k] = take(kc * 8);
        o.node[k] = take(kc * 4);
        o.meta[k] = take(kc * 4);
    }
    o.cand = take((kc << g.sb) * 8);
    o.plink = take(kc * 4);
    o.child = take(kc * 8);
    o.hkey = take((uint32_t)g.ht * 8);
    o.hval = take((uint32_t)g.ht * 4);
    o.hist = take(256 * 4);
    o.red = take(32 * 8);
    o.misc = take(16 * 4);
    o.total = off;
    return o;
}

size_t ctc_lds_bytes(const CtcGeom& g) { return lds_plan(g).total; }

template <typename T>
__device__ __forceinline__ T* lds(uint32_t off) { return reinterpret_cast<T*>(smem + off); }

// ------------------------------------------------------ block-level helpers
template <int NW, int OP>   // OP 0 = sum, 1 = max, 2 = min
__device__ __forceinline__ uint64_t block_reduce_u64(uint64_t v, uint64_t* red, int slot) {
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t x = __shfl_xor(v, o);
        v = OP == 0 ? v + x : OP == 1 ? (x > v ? x : v) : (x < v ? x : v);
    }
    if (NW == 1) return v;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[slot * 4 + wid] = v;
    __syncthreads();
    uint64_t s = red[slot * 4];
    for (int w = 1; w < NW; w++) {
        const uint64_t x = red[slot * 4 + w];
        s = OP == 0 ? s + x : OP == 1 ? (x > s ? x : s) : (x < s ? x : s);
    }
    return s;
}

// Exclusive count of set ballot bits below this lane.
__device__ __forceinline__ int wave_prefix(uint64_t ballot) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(ballot >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)ballot, 0u));
}

// Threshold tau such that exactly the keys >= tau are the survivors: tau is
// the need-th largest nonzero key of cand[0, N) (MSB radix select, 8-bit
// digits, starting below the bits all keys share; exits as soon as the
// selected bucket is taken whole).  Uniform across the block.
template <int NW>
__device__ __forceinline__ uint64_t radix_threshold(const uint64_t* cand, uint32_t* hist, int* misc,
                                                    int N, int need, uint64_t kmax,
                                                    uint64_t kmin) {
    constexpr int NT = 64 * NW;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (kmax == kmin) return kmax;
    int top = 63 - __clzll((long long)(kmax ^ kmin));   // highest differing bit
    int hi = top + 1;                                    // all keys agree on bits >= hi
    uint64_t pref = shr64(kmax, hi);
    for (;;) {
        const int lo = top - 7 > 0 ? top - 7 : 0;
        const int nb = top - lo + 1;
        const uint64_t mask = (1ull << nb) - 1ull;
        for (int i = tid; i < 256; i += NT) hist[i] = 0u;
        __syncthreads();
        for (int k = tid; k < N; k += NT) {
            const uint64_t key = cand[k];
            if (key != 0ull && shr64(key, hi) == pref)
                atomicAdd(&hist[(uint32_t)((key >> lo) & mask)], 1u);
        }
        __syncthreads();
        if (wid == 0) {
            const uint32_t c0 = hist[4 * lane], c1 = hist[4 * lane + 1];
            const uint32_t c2 = hist[4 * lane + 2], c3 = hist[4 * lane + 3];
            const uint32_t s = c0 + c1 + c2 + c3;
            uint32_t S = s;   // inclusive suffix sum over lanes >= lane
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t v = __shfl_down(S, o);
                if (lane + o < 64) S += v;
            }
            if (S >= (uint32_t)need && S - s < (uint32_t)need) {
                uint32_t above = S - s;
                int d;
                uint32_t cd;
                if (above + c3 >= (uint32_t)need) { d = 3; cd = c3; }
                else if (above + c3 + c2 >= (uint32_t)need) { d = 2; cd = c2; above += c3; }
                else if (above + c3 + c2 + c1 >= (uint32_t)need) { d = 1; cd = c1; above += c3 + c2; }
                else { d = 0; cd = c0; above += c3 + c2 + c1; }
                misc[0] = 4 * lane + d;
                misc[1] = (int)cd;
                misc[2] = need - (int)above;
            }
        }
        __syncthreads();
        const int bucket = misc[0], cnt = misc[1];
        need = misc[2];
        pref = (pref << nb) | (uint64_t)bucket;
        hi = lo;
        top = lo - 1;
        __syncthreads();   // misc[] is rewritten by the next pass
        if (cnt == need || lo == 0) return pref << lo;
    }
}

// ------------------------------------------------------------ main kernel
template <int NW>
__global__ __launch_bounds__(64 * NW) void ctc_beam_kernel(CtcArgs a) {
    constexpr int NT = 64 * NW;
    constexpr int PF = 16;   // prefetch registers per thread
    const CtcGeom g = a.g;
    const LdsOff o = lds_plan(g);

    const int tid = threadIdx.x, wid = tid >> 6;
    const int b = blockIdx.x;
    const int V = g.V, blank = g.blank, kcap = g.kcap, sb = g.sb, ch = g.ch;
    const int S = 1 << sb;
    const uint32_t hmask = (uint32_t)(g.ht - 1);
    int2* nodes = a.nodes + (size_t)b * a.T * kcap;
    const float* ecol = a.emis + (size_t)b * V;          // utterance b's row at t=0
    const size_t tstride = (size_t)a.B * V;              // floats between frames

    double* le = lds<double>(o.le);
    float* ebuf = lds<float>(o.ebuf);
    uint64_t* cand = lds<uint64_t>(o.cand);
    int* plink = lds<int>(o.plink);
    uint64_t* child = lds<uint64_t>(o.child);
    uint64_t* hkey = lds<uint64_t>(o.hkey);
    int* hval = lds<int>(o.hval);
    uint32_t* hist = lds<uint32_t>(o.hist);
    uint64_t* red = lds<uint64_t>(o.red);
    int* misc = lds<int>(o.misc);

    // Root slot: empty prefix in the blank state with log-score 0.  One
    // extend+prune from it is exactly initialPath + prune (cpp:87-95).
    if (tid == 0) {
        lds<uint64_t>(o.h[0])[0] = ROOT_HASH;
        lds<uint64_t>(o.hp[0])[0] = 0ull;
        lds<double>(o.snb[0])[0] = -INFINITY;
        lds<double>(o.sb[0])[0] = 0.0;
        lds<int>(o.node[0])[0] = -1;
        lds<uint32_t>(o.meta[0])[0] = META_LAST | META_HAS_B;
    }
    int cur = 0;
    int P = 1;
    int overflow = 0;

    // Emission prefetch: a chunk of ch frames = ch*V floats, PF per thread.
    float pf[PF];
    const int chunk_elems = ch * V;
#define ASR_LOAD_CHUNK(t0)                                                     \
    _Pragma("unroll") for (int j = 0; j < PF; j++) {                           \
        const int e = tid + j * NT;                                            \
        pf[j] = 0.f;                                                           \
        if (e < chunk_elems) {                                                 \
            const int s_ = e / V, v_ = e - s_ * V;                             \
            if ((t0) + s_ < a.T) pf[j] = ecol[(size_t)((t0) + s_) * tstride + v_]; \
        }                                                                      \
    }
    ASR_LOAD_CHUNK(0)

    for (int t = 0; t < a.T; t++) {
        const int si = t % ch;
        if (si == 0) {
#pragma unroll
            for (int j = 0; j < PF; j++) {
                const int e = tid + j * NT;
                if (e < chunk_elems) ebuf[e] = pf[j];
            }
            __syncthreads();
            if (t + ch < a.T) { ASR_LOAD_CHUNK(t + ch) }
        }
        const uint64_t* c_h = lds<uint64_t>(cur ? o.h[1] : o.h[0]);
        const uint64_t* c_hp = lds<uint64_t>(cur ? o.hp[1] : o.hp[0]);
        const double* c_snb = lds<double>(cur ? o.snb[1] : o.snb[0]);
        const double* c_sb = lds<double>(cur ? o.sb[1] : o.sb[0]);
        const int* c_node = lds<int>(cur ? o.node[1] : o.node[0]);
        const uint32_t* c_meta = lds<uint32_t>(cur ? o.meta[1] : o.meta[0]);
        uint64_t* n_h = lds<uint64_t>(cur ? o.h[0] : o.h[1]);
        uint64_t* n_hp = lds<uint64_t>(cur ? o.hp[0] : o.hp[1]);
        double* n_snb = lds<double>(cur ? o.snb[0] : o.snb[1]);
        double* n_sb = lds<double>(cur ? o.sb[0] : o.sb[1]);
        int* n_node = lds<int>(cur ? o.node[0] : o.node[1]);
        uint32_t* n_meta = lds<uint32_t>(cur ? o.meta[0] : o.meta[1]);

        // A. log emissions; clear per-frame tables.
        if (tid < V) {
            const double x = (double)ebuf[si * V + tid];
            le[tid] = a.is_log ? x : log(x);
        }
        for (int i = tid; i < g.ht; i += NT) hkey[i] = 0ull;
        for (int i = tid; i < P; i += NT) child[i] = 0ull;
        __syncthreads();

        // B. hash table of live prefixes.
        for (int i = tid; i < P; i += NT) {
            const uint64_t key = c_h[i];
            uint32_t pos = (uint32_t)key & hmask;
            for (;;) {
                const unsigned long long prev =
                    atomicCAS((unsigned long long*)&hkey[pos], 0ull, (unsigned long long)key);
                if (prev == 0ull) { hval[pos] = i; break; }
                pos = (pos + 1u) & hmask;
            }
        }
        __syncthreads();

        // C. parent links and child masks.
        for (int j = tid; j < P; j += NT) {
            const uint32_t m = c_meta[j];
            int p = -1;
            if (m & META_HAS_PAR) {
                const uint64_t key = c_hp[j];
                uint32_t pos = (uint32_t)key & hmask;
                for (;;) {
                    const uint64_t k2 = hkey[pos];
                    if (k2 == 0ull) break;
                    if (k2 == key) { p = hval[pos]; break; }
                    pos = (pos + 1u) & hmask;
                }
            }
            plink[j] = p;
            if (p >= 0) atomicOr((unsigned long long*)&child[p], 1ull << (m & META_LAST));
        }
        __syncthreads();

        // D. candidates.  Row i of the candidate array holds, at column c:
        //    c == blank : (q_i, blank)                                BLANK(i)
        //    c != blank : (q_i + c, not), unless q_i + c is a live slot
        //    c == V     : (q_i, not), merged with the parent's extension by
        //                 q_i's last label when the parent prefix is live.
        const int N = P << sb;
        uint64_t nvalid = 0, kmax = 0, kmin = ~0ull;
        for (int k = tid; k < N; k += NT) {
            const int i = k >> sb, c = k & (S - 1);
            Fold f;
            if (c < V) {
                const uint32_t m = c_meta[i];
                const bool hasnb = m & META_HAS_NB, hasb = m & META_HAS_B;
                const double e = le[c];
                if (c == blank) {
                    if (hasnb) f.push(c_snb[i] + e);
                    if (hasb) f.push(c_sb[i] + e);
                } else if (!((child[i] >> c) & 1ull)) {
                    if (hasnb && (int)(m & META_LAST) != c) f.push(c_snb[i] + e);
                    if (hasb) f.push(c_sb[i] + e);
                }
            } else if (c == V) {
                const uint32_t m = c_meta[i];
                const int lc = (int)(m & META_LAST);
                const int p = plink[i];
                const bool hasnb = m & META_HAS_NB;
                if (p >= 0) {
                    const double e = le[lc];
                    const uint32_t mp = c_meta[p];
                    if ((mp & META_HAS_NB) && (int)(mp & META_LAST) != lc) f.push(c_snb[p] + e);
                    // "q$" precedes "qc" in string order iff code(blank) < code(c).
                    if ((a.blank_less >> lc) & 1ull) {
                        if (mp & META_HAS_B) f.push(c_sb[p] + e);
                        if (hasnb) f.push(c_snb[i] + e);
                    } else {
                        if (hasnb) f.push(c_snb[i] + e);
                        if (mp & META_HAS_B) f.push(c_sb[p] + e);
                    }
                } else if (hasnb) {
                    f.push(c_snb[i] + le[lc]);
                }
            }
            uint64_t key = 0ull;
            if (f.have) {
                key = asr_d2key(f.acc);
                nvalid++;
                kmax = key > kmax ? key : kmax;
                kmin = key < kmin ? key : kmin;
            }
            cand[k] = key;
        }
        nvalid = block_reduce_u64<NW, 0>(nvalid, red, 0);
        kmax = block_reduce_u64<NW, 1>(kmax, red, 1);
        kmin = block_reduce_u64<NW, 2>(kmin, red, 2);
        __syncthreads();

        // E. prune threshold (cpp:97-118, F1/F2): keep keys >= tau; tau >= 1
        //    also excludes empty cells.
        uint64_t tau = 1ull;
        if ((int)nvalid > g.K) tau = radix_threshold<NW>(cand, hist, misc, N, g.K, kmax, kmin);

        // F. compaction of survivors into the next slot buffer, in
        //    (row, column) order; the row's own prefix goes at the blank column.
        int carry = 0;
        for (int base = 0; base < N; base += NT) {
            const int k = base + tid;
            const int i = k >> sb, c = k & (S - 1);
            bool emit = false;
            if (k < N && c < V) {
                if (c == blank) emit = cand[k] >= tau || cand[(i << sb) + V] >= tau;
                else emit = cand[k] >= tau;
            }
            const uint64_t bal = __ballot(emit);
            int idx = carry + wave_prefix(bal);
            int tile_total;
            if (NW == 1) {
                tile_total = __popcll(bal);
            } else {
                uint64_t* wt = red + 12 + ((base / NT) & 1) * 4;   // parity double buffer
                if ((tid & 63) == 0) wt[wid] = (uint64_t)__popcll(bal);
                __syncthreads();
                tile_total = 0;
                for (int w = 0; w < NW; w++) {
                    if (w < wid) idx += (int)wt[w];
                    tile_total += (int)wt[w];
                }
            }
            if (emit && idx < kcap) {
                if (c == blank) {
                    const uint64_t kb = cand[k], knb = cand[(i << sb) + V];
                    uint32_t m = c_meta[i] & (META_LAST | META_HAS_PAR);
                    n_h[idx] = c_h[i];
                    n_hp[idx] = c_hp[i];
                    n_node[idx] = c_node[i];
                    if (kb >= tau) { m |= META_HAS_B; n_sb[idx] = asr_key2d(kb); }
                    else n_sb[idx] = -INFINITY;
                    if (knb >= tau) { m |= META_HAS_NB; n_snb[idx] = asr_key2d(knb); }
                    else n_snb[idx] = -INFINITY;
                    n_meta[idx] = m;
                } else {
                    const int nid = t * kcap + idx;
                    nodes[nid] = make_int2(c_node[i], c);
                    n_h[idx] = mix_hash(c_h[i], (uint32_t)c);
                    n_hp[idx] = c_h[i];
                    n_node[idx] = nid;
                    n_snb[idx] = asr_key2d(cand[k]);
                    n_sb[idx] = -INFINITY;
                    n_meta[idx] = (uint32_t)c | META_HAS_NB | META_HAS_PAR;
                }
            }
            carry += tile_total;
        }
        if (carry > kcap) { overflow = 1; carry = kcap; }
        P = carry;
        cur ^= 1;
        __syncthreads();
    }
#undef ASR_LOAD_CHUNK

    // Final merge (cpp:169-187 with F3): strip the trailing blank, "q" + "q$".
    const double* c_snb = lds<double>(cur ? o.snb[1] : o.snb[0]);
    const double* c_sb = lds<double>(cur ? o.sb[1] : o.sb[0]);
    const int* c_node = lds<int>(cur ? o.node[1] : o.node[0]);
    const uint32_t* c_meta = lds<uint32_t>(cur ? o.meta[1] : o.meta[0]);
    for (int i = tid; i < P; i += NT) {
        const uint32_t m = c_meta[i];
        double s;
        if ((m & META_HAS_NB) && (m & META_HAS_B)) s = lse2(c_snb[i], c_sb[i]);
        else s = (m & META_HAS_NB) ? c_snb[i] : c_sb[i];
        a.fin_score[(size_t)b * kcap + i] = s;
        a.fin_node[(size_t)b * kcap + i] = c_node[i];
    }
    if (tid == 0) {
        a.fin_n[b] = P;
        a.status[b] = overflow;
    }
}

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
        for (int x = fn[i]; x >= 0; x = nodes[x].x) li++;
        for (int x = fn[bi]; x >= 0; x = nodes[x].x) lb++;
        // k-th symbol from the front of slot s: walk (len-1-k) parents.
        bool less = false, decided = false;
        const int lmin = li < lb ? li : lb;
        for (int k = 0; k < lmin && !decided; k++) {
            int xi = fn[i], xb = fn[bi];
            for (int s = 0; s < li - 1 - k; s++) xi = nodes[xi].x;
            for (int s = 0; s < lb - 1 - k; s++) xb = nodes[xb].x;
            const int ci = codes[nodes[xi].y], cb = codes[nodes[xb].y];
            if (ci != cb) { less = ci < cb; decided = true; }
        }
        if (!decided) less = li < lb;
        if (less) bi = i;
    }
    int len = 0;
    for (int x = fn[bi]; x >= 0; x = nodes[x].x) {
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
    for (int i = threadIdx.x; i < n; i += 64) {
        int* out = all_lab + ((size_t)b * kcap + i) * a.T;
        int len = 0;
        for (int x = fn[i]; x >= 0; x = nodes[x].x) out[len++] = nodes[x].y;
        for (int p = 0, q = len - 1; p < q; p++, q--) {
            const int tmp = out[p];
            out[p] = out[q];
            out[q] = tmp;
        }
        all_len[(size_t)b * kcap + i] = len;
    }
}

int ctc_launch_decode(const CtcArgs& a, int waves, hipStream_t s) {
    const size_t lds = ctc_lds_bytes(a.g);
    const dim3 grid(a.B);
    switch (waves) {
        case 1: hipLaunchKernelGGL(ctc_beam_kernel<1>, grid, dim3(64), lds, s, a); break;
        case 2: hipLaunchKernelGGL(ctc_beam_kernel<2>, grid, dim3(128), lds, s, a); break;
        case 4: hipLaunchKernelGGL(ctc_beam_kernel<4>, grid, dim3(256), lds, s, a); break;
        default: return ASR_ERR_ARG;
    }
    ASR_LAUNCH_TRY();
    return ASR_OK;
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
    // Allow the full 160 KiB of LDS per workgroup for every instantiation.
    const int lim = 160 * 1024;
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_beam_kernel<1>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_beam_kernel<2>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    ASR_HIP_TRY(hipFuncSetAttribute((const void*)ctc_beam_kernel<4>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lim));
    return ASR_OK;
}

}  // namespace asr
