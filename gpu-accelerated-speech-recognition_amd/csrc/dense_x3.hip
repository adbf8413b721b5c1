// ============================================================================
// fp32-accurate dense kernels on the bf16 matrix cores (gfx950).
//
// Every fp32 operand x is split into three bf16 pieces, x = h + m + l:
// h = bf16(x), m = bf16(x - h), l = bf16(x - h - m), each rounded to nearest;
// the two subtractions are exact in fp32, and l captures the remainder exactly
// (24 bits = 8 + 8 + 8), so h + m + l == x.  A product x.y keeps the six
// piece products of order >= 2^-18 (hh, hm, mh, hl, mm, lh), each exact in
// fp32 (8 x 8 significant bits), accumulated by the MFMA in fp32; the three
// dropped ones (ml, lm, ll) are below 2^-25 |x.y|.  The result is as accurate
// as an fp32 GEMM (measured against fp64: max error / sum|x.y| 2.2e-7 vs
// 3.3e-7 for a sequential fp32 FMA chain, tools/x3_probe.hip) — a rounding
// difference, not a precision reduction.  Six v_mfma_f32_16x16x32_bf16 (16
// cycles each per SIMD) do the work of 8 v_mfma_f32_16x16x4_f32 (32 cycles):
// 2.7x the fp32 MFMA rate.
//
// The same shapes run on the fp32 kernels of dense.hip when the split
// arithmetic is off (asr_set_dense_arith(ASR_DENSE_F32)); the choice depends on
// the shape and that setting only, never on M or on the grid, so a row's bits
// do not depend on the batch it is in (utterance sharding relies on that).
// ============================================================================
#include "dense.h"

#include <atomic>
#include <mutex>
#include <cstdlib>
#include <cstring>

thread_local int asr_internal_dense_arith = -1;

namespace asr {

// ASR_DENSE_F32 / ASR_DENSE_SPLIT_BF16 (asr_set_dense_arith); initial value
// from ASR_DENSE ("f32" / "x3"), else the split arithmetic.
static std::atomic<int> g_dense_arith{-1};
int dense_arith() {
    if (asr_internal_dense_arith >= 0) return asr_internal_dense_arith;   // a pipeline's latched setting
    int a = g_dense_arith.load(std::memory_order_relaxed);
    if (a < 0) {
        const char* e = getenv("ASR_DENSE");
        a = (e && !strcmp(e, "f32")) ? ASR_DENSE_F32 : ASR_DENSE_SPLIT_BF16;
        int expect = -1;
        g_dense_arith.compare_exchange_strong(expect, a);
        a = g_dense_arith.load(std::memory_order_relaxed);
    }
    return a;
}
void dense_arith_set(int a) { g_dense_arith.store(a, std::memory_order_relaxed); }
bool dense_x3_on() { return dense_arith() == ASR_DENSE_SPLIT_BF16; }

// A/B build knobs (Makefile dvariant; measured with tools/dense_time.py, run sa:
// only the GEMM prefetch is on in the product; the others changed < 1 %)
#ifndef ASR_X3G_PF
#define ASR_X3G_PF 1     // GEMM: A fragments one chunk ahead (C4 input projection 1.345 -> 1.230 ms on 128 CUs)
#endif
#ifndef ASR_X3G_SGB
#define ASR_X3G_SGB 0    // GEMM: sched_group_barrier order of reads / MFMAs
#endif
#ifndef ASR_X3R_TANH
#define ASR_X3R_TANH 0   // recurrence: branch-free exp2 / rcp tanh (<= 1.6 ulp)
#endif
#ifndef ASR_X3R_PACK
#define ASR_X3R_PACK 0   // recurrence: k order permuted in each 32-chunk, h pieces written as bf16 pairs
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
    h = (__bf16)x;
    const float r = x - (float)h;
    m = (__bf16)r;
    l = (__bf16)(r - (float)m);
}

__device__ __forceinline__ float fbits(unsigned u) { return __builtin_bit_cast(float, u); }

// tanh of the recurrence epilogue.  ASR_X3R_TANH: branch-free, |x| >= 0.625
// as 1 - 2 / (1 + 2^(2|x| log2 e)) (v_exp_f32, v_rcp_f32), below an odd
// minimax polynomial; <= 1.6 ulp from tanhf over every fp32 input
// (tools/x3_probe.hip tanh_fast); else the device library's tanhf.
__device__ __forceinline__ float x3_tanh(float x) {
#if ASR_X3R_TANH
    const float ax = fabsf(x);
    const float y = __builtin_amdgcn_exp2f(ax * 2.8853900817779268f);
    const float big = __builtin_fmaf(__builtin_amdgcn_rcpf(1.0f + y), -2.0f, 1.0f);
    const float x2 = x * x;
    float q = __builtin_fmaf(fbits(0xbbbac73du), x2, fbits(0x3ca908c9u));
    q = __builtin_fmaf(x2, q, fbits(0xbd5c1c4eu));
    q = __builtin_fmaf(x2, q, fbits(0x3e088382u));
    q = __builtin_fmaf(x2, q, fbits(0xbeaaaa99u));
    const float small = __builtin_fmaf(x2, ax * q, ax);
    const float m = ax < 0.625f ? small : big;
    return __builtin_bit_cast(float, (__builtin_bit_cast(unsigned, m) & 0x7fffffffu) |
                                         (__builtin_bit_cast(unsigned, x) & 0x80000000u));
#else
    return tanhf(x);
#endif
}

// Position of h column n in the LDS piece rows (and of k in a 32-deep MFMA
// chunk): ASR_X3R_PACK puts columns n and n + 16 of a 32-column slice side by
// side, so the lane that produces both writes one bf16 pair per piece.  The
// B / W_out fragments follow the same k order (x3_kperm).
__device__ __forceinline__ int x3_hpos(int n) {
#if ASR_X3R_PACK
    return (n & ~31) + 2 * (n & 15) + ((n >> 4) & 1);
#else
    return n;
#endif
}
// k of element j of lane group g in chunk c (A / B fragment element order)
__device__ __forceinline__ int x3_kperm(int c, int g, int j) {
#if ASR_X3R_PACK
    return 32 * c + 16 * (j & 1) + 4 * g + (j >> 1);
#else
    return 32 * c + 8 * g + j;
#endif
}

// raw buffer resources: loads past num_records return 0, stores are dropped
// (the row tails of a tile / a step need no branches)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* base, long bytes) {
    const int n = bytes < 0x7fffffffL ? (int)bytes : 0x7fffffff;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, n, 0x00020000);
}
__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, int off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, 0);
}

// acc[ct] += A . B over one 32-k chunk for NT column tiles, the six piece
// products in ascending order of magnitude; consecutive MFMAs go to different
// accumulators (independent chains).
#define X3_PRODUCTS(NT, ACC, AH, AM, AL, BH, BM, BL, C)                                           \
    {                                                                                             \
        _Pragma("unroll") for (int ct_ = 0; ct_ < NT; ct_++) ACC[ct_] =                           \
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(AL, BH[ct_][C], ACC[ct_], 0, 0, 0);           \
        _Pragma("unroll") for (int ct_ = 0; ct_ < NT; ct_++) ACC[ct_] =                           \
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(AM, BM[ct_][C], ACC[ct_], 0, 0, 0);           \
        _Pragma("unroll") for (int ct_ = 0; ct_ < NT; ct_++) ACC[ct_] =                           \
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(AH, BL[ct_][C], ACC[ct_], 0, 0, 0);           \
        _Pragma("unroll") for (int ct_ = 0; ct_ < NT; ct_++) ACC[ct_] =                           \
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(AM, BH[ct_][C], ACC[ct_], 0, 0, 0);           \
        _Pragma("unroll") for (int ct_ = 0; ct_ < NT; ct_++) ACC[ct_] =                           \
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(AH, BM[ct_][C], ACC[ct_], 0, 0, 0);           \
        _Pragma("unroll") for (int ct_ = 0; ct_ < NT; ct_++) ACC[ct_] =                           \
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(AH, BH[ct_][C], ACC[ct_], 0, 0, 0);           \
    }

__device__ __forceinline__ void lds_barrier_x3() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ---------------------------------------------------------------------------
// GEMM C = A.B (+ bias, ReLU), K <= 256, any N (256 columns per workgroup
// row of the grid): the RNN input projection (cuMatrix.cpp:33-70 /
// RNN.cu:9-30's x.W_ih) and the Linear layers (Linear.cu:3-10).
//   * 8 waves, two per SIMD (one wave's VALU issues beside the other's
//     MFMAs); wave w owns columns n0 + 32w .. + 31 as two 16-column tiles and
//     keeps their B pieces in registers for the whole launch (2 x NCH x 3
//     bf16x8 = 24 NCH registers).
//   * 16-row tiles of A: staged once per tile to LDS as the three pieces
//     (double-buffered, one barrier per tile), the next tile's A in flight
//     during this tile's MFMAs; the A fragment of MFMA (chunk c) is one
//     ds_read_b128 per piece (row c15, k = 32c + 8g .. + 7).
//   * Row tiles per workgroup: tpw > 0 a contiguous run of tpw tiles (short
//     workgroups that free their CU soon), 0 persistent (stride gridDim.x).
// ---------------------------------------------------------------------------
constexpr int X3_ROWS = 16;
constexpr int X3_WAVES = 8;
constexpr int X3_NCOL = 32 * X3_WAVES;
// Internal epilogue: C in the recurrence's fragment-major P layout (below,
// rnn_recur_x3_kernel<..., PFR>): row tile q of C (rows 16q .. 16q + 15) is
// the block C + 16 q N, and in it wave w's lane l keeps its 8 values
// (rows 4 (l >> 4) + j, columns 32 w + 16 ct + (l & 15); element 4 ct + j)
// at floats (64 w + l) * 8 .. + 7: two 16-byte stores per lane here, two
// 16-byte loads per lane in the recurrence, instead of eight 4-byte ones
// each.  N = H (one 256-column block, waves past N / 32 store nothing),
// M % 16 == 0, no bias.
constexpr int X3_EPI_FRAG = 8;

template <int NCH>
constexpr int x3_gemm_lds() {
    return 2 * 3 * X3_ROWS * (NCH * 32 + 8) * 2;
}

template <int NCH, int EPI>
__global__ __launch_bounds__(64 * X3_WAVES) void gemm_x3_kernel(GemmArgs g, int tpw) {
    constexpr int KC = NCH * 32;              // staged k columns (zero past K)
    constexpr int AS = KC + 8;                // LDS row stride (bf16): rows 16 B apart in banks
    constexpr int PIECE = X3_ROWS * AS;
    constexpr int NV4 = X3_ROWS * KC / 4;     // float4 per tile
    constexpr int NL = (NV4 + 64 * X3_WAVES - 1) / (64 * X3_WAVES);
    extern __shared__ __attribute__((aligned(16))) __bf16 x3s[];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c15 = lane & 15, gq = lane >> 4;
    const int n0 = blockIdx.y * X3_NCOL;
    bf16x8 bh[2][NCH], bm[2][NCH], bl[2][NCH];
    int ncol[2];
#pragma unroll
    for (int ct = 0; ct < 2; ct++) {
        const int n = n0 + 32 * w + 16 * ct + c15;
        ncol[ct] = n;
#pragma unroll
        for (int c = 0; c < NCH; c++)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int k = 32 * c + 8 * gq + j;
                const float b = (k < g.K && n < g.N) ? g.B[(long)k * g.sbk + (long)n * g.sbn] : 0.f;
                __bf16 h, m, l;
                split3(b, h, m, l);
                bh[ct][c][j] = h;
                bm[ct][c][j] = m;
                bl[ct][c][j] = l;
            }
    }
    float bias[2] = {0.f, 0.f};
    if (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) {
#pragma unroll
        for (int ct = 0; ct < 2; ct++) bias[ct] = ncol[ct] < g.N ? g.b1[ncol[ct]] : 0.f;
    }
    const int ntile = (g.M + X3_ROWS - 1) / X3_ROWS;
    int tile, tend, tstep;
    if (tpw > 0) {
        tile = blockIdx.x * tpw;
        tend = min(ntile, tile + tpw);
        tstep = 1;
    } else {
        tile = blockIdx.x;
        tend = ntile;
        tstep = gridDim.x;
    }
    f32x4 st[NL];
    auto load = [&](int tl) {
        const long r0 = (long)tl * X3_ROWS;
        const long rows = tl < tend ? min((long)X3_ROWS, (long)g.M - r0) : 0;
        const auto rs = brsrc(g.A + r0 * g.sam, rows * g.sam * 4);
#pragma unroll
        for (int i = 0; i < NL; i++) {
            const int idx = tid + 64 * X3_WAVES * i;
            const int row = idx / (KC / 4), k = (idx % (KC / 4)) * 4;
            f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (row * (int)g.sam + k) * 4, 0, 0));
            if (k >= g.K || idx >= NV4) v = f32x4{0.f, 0.f, 0.f, 0.f};
            st[i] = v;
        }
    };
    auto stage = [&](int buf) {
        __bf16* base = x3s + buf * 3 * PIECE;
#pragma unroll
        for (int i = 0; i < NL; i++) {
            const int idx = tid + 64 * X3_WAVES * i;
            if (NV4 % (64 * X3_WAVES) != 0 && idx >= NV4) continue;
            const int row = idx / (KC / 4), k = (idx % (KC / 4)) * 4;
            bf16x4 h, m, l;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                __bf16 a, b, c;
                split3(st[i][e], a, b, c);
                h[e] = a;
                m[e] = b;
                l[e] = c;
            }
            __bf16* p = base + row * AS + k;
            *reinterpret_cast<bf16x4*>(p) = h;
            *reinterpret_cast<bf16x4*>(p + PIECE) = m;
            *reinterpret_cast<bf16x4*>(p + 2 * PIECE) = l;
        }
    };
    load(tile);
    stage(0);
    load(tile + tstep);
    __syncthreads();
    int cur = 0;
    for (; tile < tend; tile += tstep) {
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
        const __bf16* pb = x3s + cur * 3 * PIECE;
#if ASR_X3G_PF
        // A fragments one chunk ahead (two register sets), so that a chunk's
        // MFMAs never wait on its own LDS reads
        {
            bf16x8 fa[2][3];
            auto rd = [&](int c, int sl) {
                const int off = c15 * AS + 32 * c + 8 * gq;
                fa[sl][0] = *reinterpret_cast<const bf16x8*>(pb + off);
                fa[sl][1] = *reinterpret_cast<const bf16x8*>(pb + PIECE + off);
                fa[sl][2] = *reinterpret_cast<const bf16x8*>(pb + 2 * PIECE + off);
            };
            rd(0, 0);
#pragma unroll
            for (int c = 0; c < NCH; c++) {
                if (c + 1 < NCH) rd(c + 1, (c + 1) & 1);
                X3_PRODUCTS(2, acc, fa[c & 1][0], fa[c & 1][1], fa[c & 1][2], bh, bm, bl, c)
#if ASR_X3G_SGB
                if (c + 1 < NCH) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 12, 0);
#endif
            }
        }
#else
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            const int off = c15 * AS + 32 * c + 8 * gq;
            const bf16x8 ah = *reinterpret_cast<const bf16x8*>(pb + off);
            const bf16x8 am = *reinterpret_cast<const bf16x8*>(pb + PIECE + off);
            const bf16x8 al = *reinterpret_cast<const bf16x8*>(pb + 2 * PIECE + off);
            X3_PRODUCTS(2, acc, ah, am, al, bh, bm, bl, c)
        }
#endif
        stage(cur ^ 1);
        load(tile + 2 * tstep);
        const long r0 = (long)tile * X3_ROWS;
        if (EPI == X3_EPI_FRAG) {
            if (32 * w < g.N) {
                f32x4* dst = reinterpret_cast<f32x4*>(g.C + r0 * g.N + (long)(64 * w + lane) * 8);
                dst[0] = acc[0];
                dst[1] = acc[1];
            }
        } else {
        const auto cs = brsrc(g.C + r0 * g.ldc, min((long)X3_ROWS, (long)g.M - r0) * g.ldc * 4);
#pragma unroll
        for (int ct = 0; ct < 2; ct++) {
            if (ncol[ct] < g.N) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    float y = acc[ct][j];
                    if (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) y = y + bias[ct];
                    if (EPI == EPI_BIAS_RELU && y < 0.f) y = 0.f;
                    bstore(cs, ((4 * gq + j) * (int)g.ldc + ncol[ct]) * 4, y);
                }
            }
        }
        }
        __syncthreads();
        cur ^= 1;
    }
}

template <int NCH, int EPI>
static int launch_gemm_x3_k(const GemmArgs& g, int tpw, hipStream_t s) {
    static AsrAttrOnce attr;
    if (int r_ = attr.set((const void*)gemm_x3_kernel<NCH, EPI>, x3_gemm_lds<NCH>())) return r_;
    const int ntile = (g.M + X3_ROWS - 1) / X3_ROWS;
    const int ncol = (g.N + X3_NCOL - 1) / X3_NCOL;
    int rows;
    if (tpw > 0) {
        rows = (ntile + tpw - 1) / tpw;
    } else {
        int dev = 0, ncu = 256;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
        rows = max(1, min(ntile, ncu / max(1, ncol)));   // one workgroup per CU (2 waves per SIMD)
    }
    hipLaunchKernelGGL((gemm_x3_kernel<NCH, EPI>), dim3((unsigned)rows, (unsigned)ncol), dim3(64 * X3_WAVES),
                       x3_gemm_lds<NCH>(), s, g, tpw);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

template <int EPI>
static int launch_gemm_x3_epi(const GemmArgs& g, int tpw, hipStream_t s) {
    if (g.K <= 32) return launch_gemm_x3_k<1, EPI>(g, tpw, s);
    if (g.K <= 64) return launch_gemm_x3_k<2, EPI>(g, tpw, s);
    if (g.K <= 128) return launch_gemm_x3_k<4, EPI>(g, tpw, s);
    return launch_gemm_x3_k<8, EPI>(g, tpw, s);
}

// ---------------------------------------------------------------------------
// GEMM C = A.B (+ bias, ReLU) on the split arithmetic for K > 256 (C5's
// input projection [T*B, 1024] x [1024, 1024] and emission layer [T*B, 1024]
// x [1024, 1000]; BL's K = 2048), where the K <= 256 kernel's B-in-registers
// scheme cannot hold B.  Round 6.
//   * B is split ONCE per call into its three pieces, stored fragment-major
//     (x3k_split_b_kernel: for 32-k chunk c and 16-column tile nt, the 64
//     lanes' 16-byte MFMA B fragments are one contiguous KiB), into a
//     stream-ordered scratch allocation, so the GEMM moves B with
//     global_load_lds (LDS-DMA: a KiB per wave-instruction, no registers)
//     and never splits it again;
//   * 128 x 128 output tiles, 8 waves (4 x 2), each wave 32 x 64: per 32-k
//     chunk 2 x 4 tiles x 6 products = 48 v_mfma_f32_16x16x32_bf16;
//   * A (fp32) is loaded into registers one chunk ahead, split, and written
//     fragment-major into LDS (conflict-free ds_read_b128 fragment reads);
//     LDS double-buffered, one barrier per chunk;
//   * the six products per tile in the K <= 256 kernel's order (ascending
//     magnitude), chunks in k order: fp32-accurate, and a row's bits depend
//     on the shape only (never on M: utterance sharding relies on that).
// Workgroups map to tiles XCD-aware: the 8 column tiles of a row block run
// on one XCD (its L2 keeps the A rows they share).
// ---------------------------------------------------------------------------
constexpr int XK_BM = 128, XK_BN = 128;
constexpr int XK_WAVES = 8;
constexpr int XK_RT = XK_BM / 16, XK_CT = XK_BN / 16;    // 16-row / 16-column tiles per workgroup tile
constexpr int XK_FRAG = 512;                             // bf16 per fragment block (64 lanes x 8)
constexpr int XK_ASTAGE = 3 * XK_RT * XK_FRAG;           // bf16 of one A stage (three pieces)
constexpr int XK_BSTAGE = 3 * XK_CT * XK_FRAG;           // bf16 of one B stage
constexpr int XK_LDS = 2 * (XK_ASTAGE + XK_BSTAGE) * 2;  // bytes, double-buffered

// B (k, n) = B[k * sbk + n * sbn] -> Bf[p][c][nt][lane][8]: lane l = 16 gq + c15
// holds n = 16 nt + c15, k = 32 c + 8 gq + j; zero past K and N.  nct: column
// tiles stored (a multiple of XK_CT).
__global__ __launch_bounds__(256) void x3k_split_b_kernel(const float* __restrict__ Bm, long sbk, long sbn, int K,
                                                          int N, int nch, int nct, __bf16* __restrict__ Bf) {
    const long f = (long)blockIdx.x * 256 + threadIdx.x;   // one lane-fragment per thread
    const long nfrag = (long)nch * nct * 64;
    if (f >= nfrag) return;
    const int l = (int)(f & 63), nt = (int)((f >> 6) % nct), c = (int)(f / (64L * nct));
    const int gq = l >> 4, c15 = l & 15;
    const int n = 16 * nt + c15;
    bf16x8 ph, pm, pl;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const int k = 32 * c + 8 * gq + j;
        const float b = (k < K && n < N) ? Bm[(long)k * sbk + (long)n * sbn] : 0.f;
        __bf16 h, m, lo;
        split3(b, h, m, lo);
        ph[j] = h;
        pm[j] = m;
        pl[j] = lo;
    }
    const long piece = (long)nch * nct * XK_FRAG;
    bf16x8* dst = reinterpret_cast<bf16x8*>(Bf + ((long)c * nct + nt) * XK_FRAG) + l;
    dst[0] = ph;
    dst[piece / 8] = pm;
    dst[2 * piece / 8] = pl;
}

template <int EPI>
__global__ __launch_bounds__(64 * XK_WAVES) void gemm_x3k_kernel(GemmArgs g, const __bf16* __restrict__ Bf,
                                                                 int nch, int nct, int nrt_tiles) {
    extern __shared__ __attribute__((aligned(16))) __bf16 xks[];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 1, wn = w & 1;   // wave rows 32 wm .., columns 64 wn ..
    // XCD-aware tile order: consecutive tiles (the column tiles of one row
    // block) on one XCD (workgroups are dealt to the 8 XCDs round-robin)
    const int nwg = gridDim.x;
    const int id = blockIdx.x;
    const int per = nwg / 8;
    const int lin = (id < per * 8) ? (id & 7) * per + (id >> 3) : id;
    const int nctile = nct / XK_CT;
    const int mt = lin / nctile, ntile = lin - mt * nctile;
    if (mt >= nrt_tiles) return;
    const long r0 = (long)mt * XK_BM;
    const int n0 = ntile * XK_BN;
    const long rows = min((long)XK_BM, (long)g.M - r0);
    const auto rsA = brsrc(g.A + r0 * g.sam, rows * g.sam * 4);
    const long piece = (long)nch * nct * XK_FRAG;
    // A staging: 128 rows x 32 k per chunk = 1024 float4, two per thread
    f32x4 st[2];
    auto load_a = [&](int c) {
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int idx = tid + 512 * i;
            const int row = idx >> 3, kq = idx & 7;
            const int k = 32 * c + 4 * kq;
            f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                    rsA, (row * (int)g.sam + k) * 4, 0, 0));
            if (k >= g.K) v = f32x4{0.f, 0.f, 0.f, 0.f};
            st[i] = v;
        }
    };
    auto stage_a = [&](int buf) {
        __bf16* base = xks + buf * (XK_ASTAGE + XK_BSTAGE);
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int idx = tid + 512 * i;
            const int row = idx >> 3, kq = idx & 7;
            const int rt = row >> 4, c15 = row & 15, gq = kq >> 1, half = kq & 1;
            bf16x4 h, m, l;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                __bf16 a, b, cc;
                split3(st[i][e], a, b, cc);
                h[e] = a;
                m[e] = b;
                l[e] = cc;
            }
            __bf16* p = base + (rt * 64 + gq * 16 + c15) * 8 + half * 4;
            *reinterpret_cast<bf16x4*>(p) = h;
            *reinterpret_cast<bf16x4*>(p + XK_RT * XK_FRAG) = m;
            *reinterpret_cast<bf16x4*>(p + 2 * XK_RT * XK_FRAG) = l;
        }
    };
    // B stage: 3 pieces x XK_CT column tiles = 24 fragment blocks of 1 KiB,
    // three per wave, by LDS-DMA
    auto load_b = [&](int c, int buf) {
        __bf16* base = xks + buf * (XK_ASTAGE + XK_BSTAGE) + XK_ASTAGE;
#pragma unroll
        for (int q = 0; q < 3; q++) {
            const int blk = w * 3 + q;              // 0 .. 23
            const int p = blk / XK_CT, ctl = blk - p * XK_CT;
            const __bf16* src = Bf + p * piece + ((long)c * nct + (n0 >> 4) + ctl) * XK_FRAG + lane * 8;
            __builtin_amdgcn_global_load_lds(const_cast<__bf16*>(src),
                                             (__attribute__((address_space(3))) void*)(base + blk * XK_FRAG), 16, 0,
                                             0);
        }
    };
    f32x4 acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    load_a(0);
    load_b(0, 0);
    stage_a(0);
    if (nch > 1) load_a(1);
    __syncthreads();
    int cur = 0;
    for (int c = 0; c < nch; c++) {
        if (c + 1 < nch) load_b(c + 1, cur ^ 1);
        const __bf16* ab = xks + cur * (XK_ASTAGE + XK_BSTAGE);
        const __bf16* bb = ab + XK_ASTAGE;
        bf16x8 fa[2][3], fb[4][3];
#pragma unroll
        for (int rt = 0; rt < 2; rt++)
#pragma unroll
            for (int p = 0; p < 3; p++)
                fa[rt][p] = *reinterpret_cast<const bf16x8*>(ab + ((p * XK_RT + 2 * wm + rt) * 64 + lane) * 8);
#pragma unroll
        for (int ct = 0; ct < 4; ct++)
#pragma unroll
            for (int p = 0; p < 3; p++)
                fb[ct][p] = *reinterpret_cast<const bf16x8*>(bb + ((p * XK_CT + 4 * wn + ct) * 64 + lane) * 8);
#pragma unroll
        for (int rt = 0; rt < 2; rt++) {
            // the six piece products in ascending order of magnitude (X3_PRODUCTS)
#pragma unroll
            for (int ct = 0; ct < 4; ct++)
                acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[rt][2], fb[ct][0], acc[rt][ct], 0, 0, 0);
#pragma unroll
            for (int ct = 0; ct < 4; ct++)
                acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[rt][1], fb[ct][1], acc[rt][ct], 0, 0, 0);
#pragma unroll
            for (int ct = 0; ct < 4; ct++)
                acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[rt][0], fb[ct][2], acc[rt][ct], 0, 0, 0);
#pragma unroll
            for (int ct = 0; ct < 4; ct++)
                acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[rt][1], fb[ct][0], acc[rt][ct], 0, 0, 0);
#pragma unroll
            for (int ct = 0; ct < 4; ct++)
                acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[rt][0], fb[ct][1], acc[rt][ct], 0, 0, 0);
#pragma unroll
            for (int ct = 0; ct < 4; ct++)
                acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[rt][0], fb[ct][0], acc[rt][ct], 0, 0, 0);
        }
        if (c + 1 < nch) {
            stage_a(cur ^ 1);
            if (c + 2 < nch) load_a(c + 2);
        }
        __syncthreads();
        cur ^= 1;
    }
    // epilogue: lane (gq, c15) of tile (rt, ct) holds rows 4 gq + j, column c15
    const int gq = lane >> 4, c15 = lane & 15;
    const auto cs = brsrc(g.C + r0 * g.ldc, rows * g.ldc * 4);
#pragma unroll
    for (int ct = 0; ct < 4; ct++) {
        const int n = n0 + 64 * wn + 16 * ct + c15;
        if (n >= g.N) continue;
        float bias = 0.f;
        if (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) bias = g.b1[n];
#pragma unroll
        for (int rt = 0; rt < 2; rt++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                float y = acc[rt][ct][j];
                if (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) y = y + bias;
                if (EPI == EPI_BIAS_RELU && y < 0.f) y = 0.f;
                bstore(cs, ((32 * wm + 16 * rt + 4 * gq + j) * (int)g.ldc + n) * 4, y);
            }
    }
}

static int x3k_pool_once() {   // keep freed scratch in the pool (no release at each sync)
    static std::mutex mu;
    static uint64_t done = 0;
    int dev = 0;
    ASR_HIP_TRY(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lock(mu);
    if (dev >= 0 && dev < 64 && !(done & (1ull << dev))) {
        hipMemPool_t pool;
        if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
            uint64_t thr = ~0ull;
            (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
        }
        done |= 1ull << dev;
    }
    return ASR_OK;
}

template <int EPI>
static int launch_gemm_x3k(const GemmArgs& g, hipStream_t s) {
    static AsrAttrOnce attr;
    if (int r_ = attr.set((const void*)gemm_x3k_kernel<EPI>, XK_LDS)) return r_;
    if (int r_ = x3k_pool_once()) return r_;
    const int nch = (g.K + 31) / 32;
    const int nct = (g.N + XK_BN - 1) / XK_BN * XK_CT;
    const size_t bytes = (size_t)3 * nch * nct * XK_FRAG * sizeof(__bf16);
    void* ws = nullptr;
    ASR_HIP_TRY(hipMallocAsync(&ws, bytes, s));
    __bf16* Bf = static_cast<__bf16*>(ws);
    const long nfrag = (long)nch * nct * 64;
    hipLaunchKernelGGL(x3k_split_b_kernel, dim3((unsigned)((nfrag + 255) / 256)), dim3(256), 0, s, g.B, g.sbk, g.sbn,
                       g.K, g.N, nch, nct, Bf);
    int rc = ASR_OK;
    if (hipGetLastError() != hipSuccess) rc = ASR_ERR_HIP;
    const int nrt = (int)((g.M + XK_BM - 1) / XK_BM);
    const long nwg = (long)nrt * (nct / XK_CT);
    if (!rc) {
        hipLaunchKernelGGL((gemm_x3k_kernel<EPI>), dim3((unsigned)nwg), dim3(64 * XK_WAVES), XK_LDS, s, g, Bf, nch,
                           nct, nrt);
        if (hipGetLastError() != hipSuccess) rc = ASR_ERR_HIP;
    }
    ASR_HIP_TRY(hipFreeAsync(ws, s));
    return rc;
}

// The large-K kernel (K > 256): N >= 64, and the 32-bit buffer offsets of a
// 128-row tile and of the B scratch fit.
static bool x3k_applies(const GemmArgs& g) {
    const long nct = (g.N + XK_BN - 1) / XK_BN * XK_CT;
    return g.K > 256 && g.N >= 64 && (long)g.sam * 4 * XK_BM < 0x7fffffffL &&
           (long)g.ldc * 4 * XK_BM < 0x7fffffffL && (long)g.M / XK_BM * (nct / XK_CT) < 0x7fffffffL;
}

bool gemm_x3_applies(const GemmArgs& g, int epi) {
    if (epi != EPI_NONE && epi != EPI_BIAS && epi != EPI_BIAS_RELU) return false;
    const bool va = g.sak == 1 && (g.K % 4) == 0 && (g.sam % 4) == 0 && ((uintptr_t)g.A % 16) == 0;
    if (!va) return false;
    if (g.K > 256) return x3k_applies(g);
    return g.N >= 64 && (long)g.sam * 4 * X3_ROWS < 0x7fffffffL && (long)g.ldc * 4 * X3_ROWS < 0x7fffffffL;
}

int gemm_x3_frag_launch(const float* A, const float* W, float* P, int M, int K, int H, int tpw, hipStream_t s) {
    GemmArgs g{};
    g.A = A; g.B = W; g.C = P;
    g.M = M; g.N = H; g.K = K;
    g.sam = K; g.sak = 1; g.sbk = H; g.sbn = 1; g.ldc = H;
    if (K > 256 || !gemm_x3_applies(g, EPI_NONE) || (M % X3_ROWS) != 0 || (H % 32) != 0 || H > X3_NCOL ||
        ((uintptr_t)P % 16) != 0)
        return ASR_ERR_UNSUPPORTED;
    return launch_gemm_x3_epi<X3_EPI_FRAG>(g, tpw, s);
}

int gemm_x3_launch(const GemmArgs& g, int epi, int tpw, hipStream_t s) {
    if (!gemm_x3_applies(g, epi)) return ASR_ERR_UNSUPPORTED;
    if (g.K > 256) {
        // the B scratch is a stream-ordered allocation: not inside a capture
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone)
            return ASR_ERR_UNSUPPORTED;
        switch (epi) {
            case EPI_NONE: return launch_gemm_x3k<EPI_NONE>(g, s);
            case EPI_BIAS: return launch_gemm_x3k<EPI_BIAS>(g, s);
            default: return launch_gemm_x3k<EPI_BIAS_RELU>(g, s);
        }
    }
    switch (epi) {
        case EPI_NONE: return launch_gemm_x3_epi<EPI_NONE>(g, tpw, s);
        case EPI_BIAS: return launch_gemm_x3_epi<EPI_BIAS>(g, tpw, s);
        default: return launch_gemm_x3_epi<EPI_BIAS_RELU>(g, tpw, s);
    }
}

// ---------------------------------------------------------------------------
// RNN recurrence h_t = tanh((P_t + h_{t-1}.W_hh) + (b_hh + b_ih)) (the op
// order of RNN_Cell.cu:10-12) on the split arithmetic, 16 utterances per
// workgroup, H = 32 NCH (64, 128, 256): the fp32 rnn_recur_mfma_kernel's
// schedule (dense.hip) with
//   * NCH waves, wave w owning columns 32w .. 32w + 31: its W_hh pieces in
//     registers for the whole sequence (24 NCH registers);
//   * h_{t-1} as its three pieces in LDS, double-buffered (one barrier per
//     step); each lane splits the h values it produces (a lane's 8 values:
//     rows 4g + j, two columns);
//   * P_{t+1} and the stores of h_t as buffer ops on a per-step resource
//     (rows past B: loads read 0, stores dropped).
// EMIT (V <= 32): the emission projection + log_softmax fused as in the fp32
// kernel, after each step's h_t epilogue (its registers are free then): wave
// w contracts k-chunk w of h_{t-1} with the W_out pieces of that
// chunk (staged once in LDS in fragment order: 6 ds_read_b128 per step) into
// a 16 x 32 partial; one step later waves 0-3 sum the partials in wave order,
// add b_out and log-softmax each row (DPP over the 16 lanes of a row).
// HL: also write h_{T-1} (exact: h + m + l == h) to hlast.
// ---------------------------------------------------------------------------
constexpr int RX_VMAX = 32;

template <int NCH, bool EMIT>
constexpr int x3_recur_lds() {
    return 2 * 3 * 16 * (NCH * 32 + 8) * 2 + (EMIT ? 3 * NCH * 2 * 64 * 16 + 2 * NCH * 4 * 64 * 8 : 0);
}

template <int NCH, bool EMIT, bool HL, bool PFR>
__global__ __launch_bounds__(64 * NCH) void rnn_recur_x3_kernel(const float* h0,
                                                                const float* __restrict__ Whh,
                                                                const float* __restrict__ b_ih,
                                                                const float* __restrict__ b_hh, float* hid,
                                                                float* hout, const float* __restrict__ Wout,
                                                                const float* __restrict__ bout,
                                                                float* __restrict__ emis, int T, int B, int V,
                                                                float* hlast) {
    constexpr int H = 32 * NCH;
    constexpr int AS = H + 8;
    constexpr int PIECE = 16 * AS;
    constexpr int NW = NCH;
    extern __shared__ __attribute__((aligned(16))) __bf16 rxs[];
    __bf16* hsb = rxs;                                                       // [2][3][16][AS]
    bf16x8* wof = reinterpret_cast<bf16x8*>(rxs + 2 * 3 * PIECE);            // EMIT: [3][NCH][2][64]
    float2* ep = reinterpret_cast<float2*>(rxs + 2 * 3 * PIECE + 3 * NCH * 2 * 64 * 8);   // EMIT: [2][NW][4][64]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c15 = lane & 15, gq = lane >> 4;
    const int r0 = blockIdx.x * 16;
    bf16x8 bh[2][NCH], bm[2][NCH], bl[2][NCH];
    int ncol[2];
    float bias[2];
#pragma unroll
    for (int ct = 0; ct < 2; ct++) {
        const int n = 32 * w + 16 * ct + c15;
        ncol[ct] = n;
        bias[ct] = b_hh[n] + b_ih[n];
#pragma unroll
        for (int c = 0; c < NCH; c++)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                __bf16 h, m, l;
                split3(Whh[(long)x3_kperm(c, gq, j) * H + n], h, m, l);
                bh[ct][c][j] = h;
                bm[ct][c][j] = m;
                bl[ct][c][j] = l;
            }
    }
    // h_{-1} pieces (zeros without h0, RNN.h:15-16) into buffer 0
    for (int x = tid; x < 16 * H; x += 64 * NW) {
        const int r = x / H, k = x - r * H;
        const float v = (h0 && r0 + r < B) ? h0[(long)(r0 + r) * H + k] : 0.f;
        __bf16 a, b, c;
        split3(v, a, b, c);
        const int o = r * AS + x3_hpos(k);
        hsb[o] = a;
        hsb[PIECE + o] = b;
        hsb[2 * PIECE + o] = c;
    }
    float bo0 = 0.f, bo1 = 0.f;
    if (EMIT) {
        // W_out pieces in MFMA B-fragment order: fragment (piece, chunk, vt),
        // lane l: W_out[32 chunk + 8 (l >> 4) + j][16 vt + (l & 15)], j < 8
        for (int x = tid; x < NCH * 2 * 64; x += 64 * NW) {
            const int l = x & 63, vt = (x >> 6) & 1, c = x >> 7;
            const int col = 16 * vt + (l & 15);
            bf16x8 fh, fm, fl;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int k = x3_kperm(c, l >> 4, j);
                __bf16 a, b, cc;
                split3(col < V ? Wout[(long)k * V + col] : 0.f, a, b, cc);
                fh[j] = a;
                fm[j] = b;
                fl[j] = cc;
            }
            wof[(0 * NCH + c) * 128 + vt * 64 + l] = fh;
            wof[(1 * NCH + c) * 128 + vt * 64 + l] = fm;
            wof[(2 * NCH + c) * 128 + vt * 64 + l] = fl;
        }
        for (int x = tid; x < 2 * NW * 4 * 64; x += 64 * NW) ep[x] = float2{0.f, 0.f};
        bo0 = c15 < V ? bout[c15] : 0.f;
        bo1 = 16 + c15 < V ? bout[16 + c15] : 0.f;
    }
    const long tstride = (long)B * H;
    const long slab = tstride * 4;
    int voff[2];
#pragma unroll
    for (int ct = 0; ct < 2; ct++) voff[ct] = ((r0 + 4 * gq) * H + ncol[ct]) * 4;
    // PFR: P in the fragment-major layout (X3_EPI_FRAG; B % 16 == 0): this
    // lane's 8 values of a step are 32 contiguous bytes
    const int poff = (blockIdx.x * 16 * H + (64 * w + lane) * 8) * 4;
    float pn[2][4];
    auto pload = [&](const float* base) {
        const auto rs = brsrc(base, slab);
        if (PFR) {
#pragma unroll
            for (int ct = 0; ct < 2; ct++) {
                const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, poff + 16 * ct, 0, 0));
#pragma unroll
                for (int j = 0; j < 4; j++) pn[ct][j] = v[j];
            }
        } else {
#pragma unroll
            for (int ct = 0; ct < 2; ct++)
#pragma unroll
                for (int j = 0; j < 4; j++) pn[ct][j] = bload(rs, voff[ct] + j * H * 4);
        }
    };
    pload(hid);
    float* const hdst = EMIT ? hout : hid;
    // EMIT: partial of the h held in hs[buf] over k-chunk w
    auto emit_partial = [&](const __bf16* pb, f32x4 (&ea)[2]) {
        ea[0] = f32x4{0.f, 0.f, 0.f, 0.f};
        ea[1] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int off = c15 * AS + 32 * w + 8 * gq;
        const bf16x8 ah = *reinterpret_cast<const bf16x8*>(pb + off);
        const bf16x8 am = *reinterpret_cast<const bf16x8*>(pb + PIECE + off);
        const bf16x8 al = *reinterpret_cast<const bf16x8*>(pb + 2 * PIECE + off);
        // one vocabulary tile at a time (its three W_out fragments live
        // only for its six MFMAs: the W_hh pieces leave few registers)
#pragma unroll
        for (int vt = 0; vt < 2; vt++) {
            bf16x8 oh[1][1], om[1][1], ol[1][1];
            oh[0][0] = wof[(0 * NCH + w) * 128 + vt * 64 + lane];
            om[0][0] = wof[(1 * NCH + w) * 128 + vt * 64 + lane];
            ol[0][0] = wof[(2 * NCH + w) * 128 + vt * 64 + lane];
            f32x4 e1[1] = {ea[vt]};
            X3_PRODUCTS(1, e1, ah, am, al, oh, om, ol, 0)
            ea[vt] = e1[0];
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    auto store_partial = [&](int s, const f32x4 (&ea)[2]) {
        float2* pp = ep + ((s & 1) * NW + w) * 4 * 64;
#pragma unroll
        for (int j = 0; j < 4; j++) pp[j * 64 + lane] = float2{ea[0][j], ea[1][j]};
    };
    auto dpp_max16 = [](float x) {
        x = fmaxf(x, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false)));
        x = fmaxf(x, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x4E, 0xF, 0xF, false)));
        x = fmaxf(x, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x141, 0xF, 0xF, false)));
        x = fmaxf(x, __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x140, 0xF, 0xF, false)));
        return x;
    };
    auto dpp_sum16 = [](float x) {
        x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
        x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x4E, 0xF, 0xF, false));
        x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x141, 0xF, 0xF, false));
        x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x140, 0xF, 0xF, false));
        return x;
    };
    // emissions of frame s from partial buffer s & 1: wave j < 4 owns rows
    // 4g + j (register j of the C fragments), columns c15 and 16 + c15
    auto emit_rows = [&](int s, bool store) {
        const float2* pp = ep + (s & 1) * NW * 4 * 64;
        for (int j = w; j < 4; j += NW) {
            float v0 = 0.f, v1 = 0.f;
#pragma unroll
            for (int q = 0; q < NW; q++) {
                const float2 x = pp[(q * 4 + j) * 64 + lane];
                v0 += x.x;
                v1 += x.y;
            }
            v0 = c15 < V ? v0 + bo0 : -INFINITY;
            v1 = 16 + c15 < V ? v1 + bo1 : -INFINITY;
            const float mx = dpp_max16(fmaxf(v0, v1));
            const float se = dpp_sum16((c15 < V ? expf(v0 - mx) : 0.f) + (16 + c15 < V ? expf(v1 - mx) : 0.f));
            const float lz = mx + logf(se);
            const int row = r0 + 4 * gq + j;
            if (store && row < B) {
                float* er = emis + ((long)s * B + row) * V;
                if (c15 < V) er[c15] = v0 - lz;
                if (16 + c15 < V) er[16 + c15] = v1 - lz;
            }
        }
    };
    __syncthreads();
    int cur = 0;
    for (int t = 0; t < T; t++) {
        float p[2][4];
#pragma unroll
        for (int ct = 0; ct < 2; ct++)
#pragma unroll
            for (int j = 0; j < 4; j++) p[ct][j] = pn[ct][j];
        pload(hid + (t + 1 < T ? t + 1 : t) * tstride);
        const __bf16* pb = hsb + cur * 3 * PIECE;
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            const int off = c15 * AS + 32 * c + 8 * gq;
            const bf16x8 ah = *reinterpret_cast<const bf16x8*>(pb + off);
            const bf16x8 am = *reinterpret_cast<const bf16x8*>(pb + PIECE + off);
            const bf16x8 al = *reinterpret_cast<const bf16x8*>(pb + 2 * PIECE + off);
            X3_PRODUCTS(2, acc, ah, am, al, bh, bm, bl, c)
        }
        __bf16* hn = hsb + (cur ^ 1) * 3 * PIECE;
        const bool sth = !EMIT || hdst != nullptr;   // EMIT without hout: the hidden states are not stored
        const auto rs = brsrc(hdst + t * tstride, sth ? slab : 0);
#if ASR_X3R_PACK
        // columns n and n + 16 are adjacent in the piece rows: one bf16 pair per piece and row
#pragma unroll
        for (int j = 0; j < 4; j++) {
            __bf16 a[2], b[2], c[2];
#pragma unroll
            for (int ct = 0; ct < 2; ct++) {
                const float h = x3_tanh((p[ct][j] + acc[ct][j]) + bias[ct]);
                split3(h, a[ct], b[ct], c[ct]);
                if (sth) bstore(rs, voff[ct] + j * H * 4, h);
            }
            const int o = (4 * gq + j) * AS + 32 * w + 2 * c15;
            typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
            *reinterpret_cast<bf16x2*>(hn + o) = bf16x2{a[0], a[1]};
            *reinterpret_cast<bf16x2*>(hn + PIECE + o) = bf16x2{b[0], b[1]};
            *reinterpret_cast<bf16x2*>(hn + 2 * PIECE + o) = bf16x2{c[0], c[1]};
        }
#else
#pragma unroll
        for (int ct = 0; ct < 2; ct++) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float h = x3_tanh((p[ct][j] + acc[ct][j]) + bias[ct]);
                __bf16 a, b, c;
                split3(h, a, b, c);
                const int o = (4 * gq + j) * AS + ncol[ct];
                hn[o] = a;
                hn[PIECE + o] = b;
                hn[2 * PIECE + o] = c;
                if (sth) bstore(rs, voff[ct] + j * H * 4, h);
            }
        }
#endif
        if (EMIT) {
            // after h_t (acc, P_t dead: fewer live registers): h_{t-1}'s
            // partial (h_{t-1} is in buffer cur, not overwritten before the
            // barrier; at t = 0 a dummy into the other partial buffer, never
            // read) and h_{t-2}'s emissions
            f32x4 ea[2];
            emit_partial(pb, ea);
            emit_rows(t - 2, t >= 2);
            store_partial(t + 1, ea);
        }
        cur ^= 1;
        lds_barrier_x3();
    }
    const __bf16* pl = hsb + cur * 3 * PIECE;   // h_{T-1}
    if (HL && hlast) {
        for (int x = tid; x < 16 * H; x += 64 * NW) {
            const int r = x / H, k = x - r * H;
            const int o = r * AS + x3_hpos(k);
            if (r0 + r < B) hlast[(long)(r0 + r) * H + k] = ((float)pl[o] + (float)pl[PIECE + o]) + (float)pl[2 * PIECE + o];
        }
    }
    if (EMIT) {   // the last two frames' emissions
        f32x4 ea[2];
        emit_partial(pl, ea);
        if (T >= 2) emit_rows(T - 2, true);
        store_partial(T - 1, ea);
        lds_barrier_x3();
        emit_rows(T - 1, true);
    }
}

template <int NCH, bool EMIT, bool HL, bool PFR>
static int launch_recur_x3_k(const float* h0, const float* Whh, const float* b_ih, const float* b_hh, float* hid,
                             float* hout, const float* Wout, const float* bout, float* emis, int T, int B, int V,
                             float* hlast, hipStream_t s) {
    constexpr int lds = x3_recur_lds<NCH, EMIT>();
    static AsrAttrOnce attr;
    if (int r_ = attr.set((const void*)rnn_recur_x3_kernel<NCH, EMIT, HL, PFR>, lds)) return r_;
    hipLaunchKernelGGL((rnn_recur_x3_kernel<NCH, EMIT, HL, PFR>), dim3((unsigned)((B + 15) / 16)), dim3(64 * NCH),
                       lds, s, h0, Whh, b_ih, b_hh, hid, hout, Wout, bout, emis, T, B, V, hlast);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

template <bool EMIT, bool HL, bool PFR = false>
static int launch_recur_x3(const float* h0, const float* Whh, const float* b_ih, const float* b_hh, float* hid,
                           float* hout, const float* Wout, const float* bout, float* emis, int T, int B, int H,
                           int V, float* hlast, hipStream_t s) {
    switch (H) {
        case 64: return launch_recur_x3_k<2, EMIT, HL, PFR>(h0, Whh, b_ih, b_hh, hid, hout, Wout, bout, emis, T, B, V, hlast, s);
        case 128: return launch_recur_x3_k<4, EMIT, HL, PFR>(h0, Whh, b_ih, b_hh, hid, hout, Wout, bout, emis, T, B, V, hlast, s);
        case 256: return launch_recur_x3_k<8, EMIT, HL, PFR>(h0, Whh, b_ih, b_hh, hid, hout, Wout, bout, emis, T, B, V, hlast, s);
        default: return ASR_ERR_UNSUPPORTED;
    }
}

bool rnn_x3_applies(int B, int H) {
    return (H == 64 || H == 128 || H == 256) && B > 0 && (long)B * H * 4 < 0x7fffffffL;
}

int rnn_recur_x3_launch(const float* h0, const float* Whh, const float* b_ih, const float* b_hh, float* hid,
                        int T, int B, int H, hipStream_t s) {
    if (!rnn_x3_applies(B, H) || T <= 0) return ASR_ERR_UNSUPPORTED;
    return launch_recur_x3<false, false>(h0, Whh, b_ih, b_hh, hid, nullptr, nullptr, nullptr, nullptr, T, B, H, 0,
                                         nullptr, s);
}

int rnn_emit_x3_launch(const float* h0, const float* Whh, const float* b_ih, const float* b_hh, const float* P,
                       float* hout, const float* Wout, const float* bout, float* emis, int T, int B, int H, int V,
                       hipStream_t s, float* hlast, bool pfrag) {
    if (!rnn_x3_applies(B, H) || T <= 0 || V < 1 || V > RX_VMAX) return ASR_ERR_UNSUPPORTED;
    if (pfrag) {   // P in the fragment-major layout of gemm_x3_frag_launch
        if ((B % 16) != 0 || ((uintptr_t)P % 16) != 0) return ASR_ERR_UNSUPPORTED;
        if (hlast)
            return launch_recur_x3<true, true, true>(h0, Whh, b_ih, b_hh, const_cast<float*>(P), hout, Wout, bout,
                                                     emis, T, B, H, V, hlast, s);
        return launch_recur_x3<true, false, true>(h0, Whh, b_ih, b_hh, const_cast<float*>(P), hout, Wout, bout,
                                                  emis, T, B, H, V, nullptr, s);
    }
    if (hlast)
        return launch_recur_x3<true, true>(h0, Whh, b_ih, b_hh, const_cast<float*>(P), hout, Wout, bout, emis, T, B,
                                           H, V, hlast, s);
    return launch_recur_x3<true, false>(h0, Whh, b_ih, b_hh, const_cast<float*>(P), hout, Wout, bout, emis, T, B, H,
                                        V, nullptr, s);
}

}  // namespace asr
