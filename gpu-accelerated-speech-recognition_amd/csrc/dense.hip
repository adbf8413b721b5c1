// ============================================================================
// Dense fp32 ops of the RNN acoustic model on gfx950:
//  * an LDS-tiled GEMM on v_mfma_f32_16x16x4_f32 (exact fp32, no TF32 on
//    CDNA4) with fused epilogues — replaces cublasSgemm + the ReLU / Tanh
//    kernels of the reference (cuMatrix.cpp:33-70, Linear.cu:3-10,
//    RNN_Cell.cu:5-13);
//  * an RNN recurrence that keeps W_hh in registers for the whole
//    sequence (H <= 256), one workgroup per utterance (RNN.cu:9-30 ran
//    2 GEMMs + a GEAM + a kernel + 3 host syncs per step);
//  * z = x + lambda*y (matrixAdd, cuMatrix.cpp:147-168).
// ============================================================================
#include "dense.h"

#include <cstddef>
#include <cstring>
#include <vector>

namespace asr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 64;   // rows per workgroup: 4 waves x 16 rows

// One K stage of a 64 x BN tile in LDS.  As row stride BK + 2: the A-fragment
// reads of a half-wave (16 rows x 2 k) land in distinct banks; Bs row stride
// BN + 16: k and k+1 land 16 banks apart.
template <int BN, int BK>
struct Tile {
    static constexpr int AST = BK + 2;
    static constexpr int BST = BN + 16;
    float As[BM * AST];
    float Bs[BK * BST];
};

// Accumulate A[M,K] . B[K,N] for this workgroup's 64 x BN tile into acc[].
// A(m,k) = A[m*sam + k*sak], B(k,n) = B[k*sbk + n*sbn].  VEC bit 0: A rows
// contiguous and 16-byte aligned (sak == 1, K and sam multiples of 4), loaded
// as float4; bit 1: the same for B rows (sbn == 1, N and sbk multiples of 4).
// The two are independent so that a narrow N (the emission projection's
// V = 29) still streams the wide A operand (the hiddens) as float4.
// BK = 64 keeps 16 KB of A per workgroup in flight per stage (the emission
// projection is a latency-bound stream at BK = 16: one 4 KB stage per round
// trip); the next stage is loaded into registers during the MFMAs.
template <int BN, int BK, int VEC>
__device__ __forceinline__ void mma_tile(Tile<BN, BK>& L, const float* __restrict__ A,
                                         const float* __restrict__ Bm, int M, int N, int K,
                                         long sam, long sak, long sbk, long sbn, int m0, int n0,
                                         f32x4 (&acc)[BN / 16]) {
    constexpr int AST = Tile<BN, BK>::AST, BST = Tile<BN, BK>::BST;
    constexpr int KA4 = BK / 4;                  // float4 per A row of a stage
    constexpr int NA = BM * KA4 / 256;           // A float4 per thread (BK >= 16)
    constexpr int NB4 = BN / 4;                  // float4 per B row
    constexpr int BTOT = BK * NB4;               // B float4 per stage
    constexpr int NB = (BTOT + 255) / 256;       // B float4 per thread (some idle when BTOT < 256)
    static_assert(NA >= 1 && BM * KA4 == NA * 256, "A stage split");
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    float ra[NA][4], rb[NB][4];

    auto load = [&](int k0) {
#pragma unroll
        for (int i = 0; i < NA; i++) {
            const int idx = tid + 256 * i;
            const int ar = idx / KA4, ak = (idx % KA4) * 4;
            const int gm = m0 + ar, gk = k0 + ak;
            if ((VEC & 1) && gm < M && gk + 3 < K) {
                const float4 v = *reinterpret_cast<const float4*>(A + gm * sam + gk);
                ra[i][0] = v.x; ra[i][1] = v.y; ra[i][2] = v.z; ra[i][3] = v.w;
            } else {
#pragma unroll
                for (int e = 0; e < 4; e++)
                    ra[i][e] = (gm < M && gk + e < K) ? A[gm * sam + (long)(gk + e) * sak] : 0.f;
            }
        }
#pragma unroll
        for (int i = 0; i < NB; i++) {
            const int idx = tid + 256 * i;
            if (idx >= BTOT) continue;
            const int bkr = idx / NB4, bn = (idx % NB4) * 4;
            const int gkb = k0 + bkr, gn = n0 + bn;
            if ((VEC & 2) && gkb < K && gn + 3 < N) {
                const float4 v = *reinterpret_cast<const float4*>(Bm + gkb * sbk + gn);
                rb[i][0] = v.x; rb[i][1] = v.y; rb[i][2] = v.z; rb[i][3] = v.w;
            } else {
#pragma unroll
                for (int e = 0; e < 4; e++)
                    rb[i][e] = (gkb < K && gn + e < N) ? Bm[gkb * sbk + (long)(gn + e) * sbn] : 0.f;
            }
        }
    };

    load(0);
    for (int k0 = 0; k0 < K; k0 += BK) {
        __syncthreads();   // previous stage fully consumed
#pragma unroll
        for (int i = 0; i < NA; i++) {
            const int idx = tid + 256 * i;
            const int ar = idx / KA4, ak = (idx % KA4) * 4;
#pragma unroll
            for (int e = 0; e < 4; e++) L.As[ar * AST + ak + e] = ra[i][e];
        }
#pragma unroll
        for (int i = 0; i < NB; i++) {
            const int idx = tid + 256 * i;
            if (idx >= BTOT) continue;
            const int bkr = idx / NB4, bn = (idx % NB4) * 4;
#pragma unroll
            for (int e = 0; e < 4; e++) L.Bs[bkr * BST + bn + e] = rb[i][e];
        }
        __syncthreads();
        if (k0 + BK < K) load(k0 + BK);   // next stage in flight during the MFMAs
        // MFMA step kk = 4c + e of lane group g contracts k = 16c + 4g + e —
        // the k order of the narrow and wide kernels, so every GEMM path
        // accumulates a row in the same sequence and gives the same bits
        // (a row's result never depends on which kernel its call took)
#pragma unroll
        for (int kk = 0; kk < BK / 4; kk++) {
            const int ko = 16 * (kk >> 2) + 4 * (lane >> 4) + (kk & 3);
            const float af = L.As[(w * 16 + (lane & 15)) * AST + ko];
#pragma unroll
            for (int nt = 0; nt < BN / 16; nt++) {
                const float bf = L.Bs[ko * BST + nt * 16 + (lane & 15)];
                acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(af, bf, acc[nt], 0, 0, 0);
            }
        }
    }
}

// Epilogue of a 16-row x BN tile held in 16x16 MFMA C fragments: rows
// rbase + j (j < 4) of lane group lane >> 4, columns n0 + nt*16 + (lane & 15).
template <int BN, int EPI>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& g, const f32x4 (&acc)[BN / 16],
                                              const f32x4 (&acc2)[BN / 16], int rbase, int n0,
                                              int lane) {
    if (EPI == EPI_LOGSOFTMAX) {
        // Whole row in this workgroup (N <= BN): row r = rbase + j lives in
        // the 16 lanes of group lane>>4, across the BN/16 tiles.
#pragma unroll
        for (int j = 0; j < 4; j++) {
            float v[BN / 16];
            float mx = -INFINITY;
#pragma unroll
            for (int nt = 0; nt < BN / 16; nt++) {
                const int col = n0 + nt * 16 + (lane & 15);
                v[nt] = col < g.N ? acc[nt][j] + g.b1[col] : -INFINITY;
                mx = fmaxf(mx, v[nt]);
            }
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
            float s = 0.f;
#pragma unroll
            for (int nt = 0; nt < BN / 16; nt++) s += expf(v[nt] - mx);
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o);
            const float lz = mx + logf(s);
            const int row = rbase + j;
            if (row < g.M) {
#pragma unroll
                for (int nt = 0; nt < BN / 16; nt++) {
                    const int col = n0 + nt * 16 + (lane & 15);
                    if (col < g.N) g.C[(long)row * g.ldc + col] = v[nt] - lz;
                }
            }
        }
        return;
    }
#pragma unroll
    for (int nt = 0; nt < BN / 16; nt++) {
        const int col = n0 + nt * 16 + (lane & 15);
        if (col >= g.N) continue;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int row = rbase + j;
            if (row >= g.M) continue;
            float y = acc[nt][j];
            if (EPI == EPI_BIAS) {
                y = y + g.b1[col];
            } else if (EPI == EPI_BIAS_RELU) {   // Linear.cu:8-9
                y = y + g.b1[col];
                if (y < 0.f) y = 0.f;
            } else if (EPI == EPI_DUAL_TANH) {   // RNN_Cell.cu:10-12: (ih + hh) + (b_hh + b_ih)
                y = tanhf((y + acc2[nt][j]) + (g.b2[col] + g.b1[col]));
            } else if (EPI == EPI_ADD_TANH) {    // D holds x.W_ih for this step
                y = tanhf((g.D[(long)row * g.ldc + col] + y) + (g.b2[col] + g.b1[col]));
            }
            g.C[(long)row * g.ldc + col] = y;
        }
    }
}

// C/D layout of 16x16 MFMA tiles (dtype-independent on gfx950):
// element j of lane l is row (l>>4)*4 + j, column l & 15.
template <int BN, int BK, int EPI, int VEC>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs g) {
    __shared__ Tile<BN, BK> L;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    f32x4 acc[BN / 16], acc2[BN / 16];
#pragma unroll
    for (int nt = 0; nt < BN / 16; nt++) {
        acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        acc2[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    mma_tile<BN, BK, VEC>(L, g.A, g.B, g.M, g.N, g.K, g.sam, g.sak, g.sbk, g.sbn, m0, n0, acc);
    if (EPI == EPI_DUAL_TANH)
        mma_tile<BN, BK, VEC>(L, g.A2, g.B2, g.M, g.N, g.K2, g.K2, 1, g.N, 1, m0, n0, acc2);

    gemm_epilogue<BN, EPI>(g, acc, acc2, m0 + w * 16 + (lane >> 4) * 4, n0, lane);
}

// Narrow outputs (N <= 64: the emission projection, V = 29 / 47): a stream of
// A with nothing of it in LDS.  Each wave owns 16 rows; lane (r, g) = (lane &
// 15, lane >> 4) loads row r's float4 at k = 16i + 4g of a 256-deep chunk,
// all 16 at once (16 KB per wave in flight), and feeds element e of float4 i
// as the A fragment of MFMA step (i, e): the step's four k-slots are then
// k = 16i + 4g + e, g = 0..3 — any k order is the same sum.  B (K x N, tiny)
// is staged transposed in LDS per chunk so that the matching B fragment is one
// ds_read_b128.
// Waves per workgroup: 4 at N <= 32 (C2 14.8 us vs 15.1 at 8), 8 at N <= 64
// (BL, K = 2048: 223 us vs 315 at 4: B is staged per 256-deep chunk).
constexpr int NS_KC = 256;   // K per chunk
template <int BN, int EPI, int NS_W = (BN <= 32 ? 4 : 8)>
__global__ __launch_bounds__(64 * NS_W) void gemm_narrow_kernel(GemmArgs g) {
    constexpr int NT = BN / 16;
    constexpr int BTS = NS_KC + 4;   // B^T row stride (floats), rows 16-B aligned
    __shared__ __attribute__((aligned(16))) float Bt[BN * BTS];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, gq = lane >> 4;
    const int row = blockIdx.x * (16 * NS_W) + w * 16 + r;
    const bool rok = row < g.M;
    const float* arow = g.A + (long)(rok ? row : 0) * g.sam;
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; nt++) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < g.K; k0 += NS_KC) {
        f32x4 a[NS_KC / 16];
#pragma unroll
        for (int i = 0; i < NS_KC / 16; i++) {
            const int k = k0 + 16 * i + 4 * gq;
            a[i] = (rok && k < g.K) ? *reinterpret_cast<const f32x4*>(arow + k) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        if (k0 > 0) __syncthreads();   // the previous chunk's B^T is consumed
        {   // all of the chunk's B loads in flight at once, then the LDS stores
            constexpr int NBL = BN * NS_KC / (64 * NS_W);
            float bv[NBL];
#pragma unroll
            for (int it = 0; it < NBL; it++) {
                const int idx = tid + it * 64 * NS_W;
                const int kk = idx / BN, n = idx - kk * BN, k = k0 + kk;
                bv[it] = (k < g.K && n < g.N) ? g.B[(long)k * g.sbk + (long)n * g.sbn] : 0.f;
            }
#pragma unroll
            for (int it = 0; it < NBL; it++) {
                const int idx = tid + it * 64 * NS_W;
                const int kk = idx / BN, n = idx - kk * BN;
                Bt[n * BTS + kk] = bv[it];
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < NS_KC / 16; i++) {
#pragma unroll
            for (int nt = 0; nt < NT; nt++) {
                const f32x4 b4 = *reinterpret_cast<const f32x4*>(&Bt[(nt * 16 + r) * BTS + 16 * i + 4 * gq]);
#pragma unroll
                for (int e = 0; e < 4; e++)
                    acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][e], b4[e], acc[nt], 0, 0, 0);
            }
        }
    }
    gemm_epilogue<BN, EPI>(g, acc, acc, blockIdx.x * (16 * NS_W) + w * 16 + gq * 4, 0, lane);
}

template <int EPI>
static int launch_gemm_narrow(const GemmArgs& g, hipStream_t s) {
    if (g.N <= 32)
        hipLaunchKernelGGL((gemm_narrow_kernel<32, EPI>), dim3((g.M + 63) / 64), dim3(256), 0, s, g);
    else
        hipLaunchKernelGGL((gemm_narrow_kernel<64, EPI>), dim3((g.M + 127) / 128), dim3(512), 0, s, g);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

// Tall-skinny wide GEMMs (the RNN input projection, [T*B, in] x [in, H] with
// in <= 512, H >= 128: C4 is 2.05 M x 256 x 256 per GPU): the tiled kernel
// re-stages B through LDS for every 64-row tile and barriers twice per
// 16-deep K stage (81 TFLOP/s, 52 % of the fp32 MFMA peak).  Here a
// persistent workgroup keeps a BNW-column slice of B^T in LDS for its whole
// life (K x BNW floats, loaded once) and streams 128-row tiles of A straight
// into registers — the narrow kernel's A path: lane (r, g) holds row r's
// float4 at k = 16i + 4g, so MFMA (i, e) contracts k = 16i + 4g + e and its B
// fragment is one ds_read_b128 of B^T — with the next tile's A in flight
// during this tile's MFMAs.  No barrier after the B staging.  One workgroup
// per CU (the slice takes most of the LDS); grid = column slices x row groups.
constexpr int GW_W = 8;     // waves per workgroup: 8 x 16 = 128 rows per tile
template <int BNW, int KMAX, int EPI>
__global__ __launch_bounds__(64 * GW_W) void gemm_wide_kernel(GemmArgs g) {
    constexpr int NT = BNW / 16;
    constexpr int NI = KMAX / 16;
    constexpr int BTS = KMAX + 4;   // B^T row stride (floats)
    extern __shared__ __attribute__((aligned(16))) float smem_gw[];
    float* Bt = smem_gw;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, gq = lane >> 4;
    const int n0 = blockIdx.y * BNW;
    const int K = g.K;
    // B^T slice, zero past N and past K: the MFMA loop always runs KMAX / 16
    // chunks, and LDS left over from an earlier kernel (e.g. a decoder's u32
    // keys, NaN as floats) times a zero A element would still be NaN
    for (int idx = tid; idx < KMAX * BNW; idx += 64 * GW_W) {
        const int k = idx / BNW, n = idx - k * BNW;
        Bt[n * BTS + k] = (k < K && n0 + n < g.N) ? g.B[(long)k * g.sbk + n0 + n] : 0.f;
    }
    const int ntile = (g.M + 16 * GW_W - 1) / (16 * GW_W);
    int tile = blockIdx.x;
    f32x4 a[NI];
    auto load_a = [&](int tl) {
        const int row = tl * (16 * GW_W) + w * 16 + r;
        const bool rok = tl < ntile && row < g.M;
        const float* arow = g.A + (long)(rok ? row : 0) * g.sam;
#pragma unroll
        for (int i = 0; i < NI; i++) {
            const int k = 16 * i + 4 * gq;
            a[i] = (rok && k < K) ? *reinterpret_cast<const f32x4*>(arow + k) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
    load_a(tile);
    __syncthreads();
    for (; tile < ntile; tile += gridDim.x) {
        f32x4 acc[NT];
#pragma unroll
        for (int nt = 0; nt < NT; nt++) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        // each K quarter's registers are refilled with the next tile's A as
        // soon as its MFMAs have consumed them, so the loads of the next tile
        // are in flight during the rest of this one (64 A VGPRs in all)
        const int nrow = (tile + (int)gridDim.x) * (16 * GW_W) + w * 16 + r;
        const bool nok = tile + (int)gridDim.x < ntile && nrow < g.M;
        const float* nrowp = g.A + (long)(nok ? nrow : 0) * g.sam;
        // B fragments one k-chunk ahead (NT b128 reads), fenced so that the
        // scheduler does not hoist all NI x NT reads at once (512 VGPRs)
        const float* btp = &Bt[r * BTS + 4 * gq];
        f32x4 bc[NT], bn[NT];
#pragma unroll
        for (int nt = 0; nt < NT; nt++) bc[nt] = *reinterpret_cast<const f32x4*>(btp + nt * 16 * BTS);
#pragma unroll
        for (int q = 0; q < 4; q++) {
#pragma unroll
            for (int ii = 0; ii < NI / 4; ii++) {
                const int i = q * (NI / 4) + ii;
                if (i + 1 < NI) {
#pragma unroll
                    for (int nt = 0; nt < NT; nt++)
                        bn[nt] = *reinterpret_cast<const f32x4*>(btp + nt * 16 * BTS + 16 * (i + 1));
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int nt = 0; nt < NT; nt++) {
#pragma unroll
                    for (int e = 0; e < 4; e++)
                        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][e], bc[nt][e], acc[nt], 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int nt = 0; nt < NT; nt++) bc[nt] = bn[nt];
            }
#pragma unroll
            for (int ii = 0; ii < NI / 4; ii++) {
                const int i = q * (NI / 4) + ii;
                const int k = 16 * i + 4 * gq;
                a[i] = (nok && k < K) ? *reinterpret_cast<const f32x4*>(nrowp + k) : f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
        gemm_epilogue<BNW, EPI>(g, acc, acc, tile * (16 * GW_W) + w * 16 + gq * 4, n0, lane);
    }
}

template <int BNW, int KMAX, int EPI>
static int launch_gemm_wide_k(const GemmArgs& g, hipStream_t s) {
    const size_t lds = sizeof(float) * (size_t)BNW * (KMAX + 4);
    static AsrAttrOnce attr;
    if (int r_ = attr.set((const void*)gemm_wide_kernel<BNW, KMAX, EPI>, 160 * 1024)) return r_;
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
        ncu = 256;
    const int ncol = (g.N + BNW - 1) / BNW;
    const int ntile = (g.M + 16 * GW_W - 1) / (16 * GW_W);
    int rows = ncu / (ncol > 0 ? ncol : 1);
    rows = rows < ntile ? rows : ntile;
    rows = rows > 0 ? rows : 1;
    hipLaunchKernelGGL((gemm_wide_kernel<BNW, KMAX, EPI>), dim3((unsigned)rows, (unsigned)ncol), dim3(64 * GW_W),
                       lds, s, g);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

// ASR_GEMM_WIDE=0: the tiled kernel instead (A/B runs).
static bool wide_off() {
    if (asr_internal_gemm_tiled) return true;
    const char* e = getenv("ASR_GEMM_WIDE");
    return e && e[0] == '0';
}

// The wide kernel when its shape applies: float4 A rows, row-major B, K <= 256,
// N >= 128, a tall M (at least 4 tiles per CU so that the slice load
// amortises; C2's 32,000 rows: 62 us wide vs 50 us tiled).  Both kernels
// accumulate in the same k order, so the choice never changes a row's bits
// (an utterance's input projection is the same in a 2048-utterance batch
// and in any shard of it: utterance sharding over GPUs relies on that).
template <int EPI>
static bool try_gemm_wide(const GemmArgs& g, hipStream_t s, int& rc) {
    if (EPI != EPI_NONE && EPI != EPI_BIAS && EPI != EPI_BIAS_RELU) return false;
    const bool va = g.sak == 1 && (g.K % 4) == 0 && (g.sam % 4) == 0 && ((uintptr_t)g.A % 16) == 0;
    if (!va || g.sbn != 1 || g.N < 128 || g.K > 256 || (long)g.M < 1024L * 128 || wide_off()) return false;
    rc = launch_gemm_wide_k<128, 256, EPI>(g, s);
    return true;
}

template <int BN, int BK, int EPI>
static int launch_gemm_bk(const GemmArgs& g, hipStream_t s) {
    const dim3 grid((g.M + BM - 1) / BM, (g.N + BN - 1) / BN);
    bool va = g.sak == 1 && (g.K % 4) == 0 && (g.sam % 4) == 0 && ((uintptr_t)g.A % 16) == 0;
    bool vb = g.sbn == 1 && (g.N % 4) == 0 && (g.sbk % 4) == 0 && ((uintptr_t)g.B % 16) == 0;
    if (EPI == EPI_DUAL_TANH) {   // second operand pair: A2 [M][K2], B2 [K2][N]
        va = va && (g.K2 % 4) == 0 && ((uintptr_t)g.A2 % 16) == 0;
        vb = vb && ((uintptr_t)g.B2 % 16) == 0;
    }
    const int vec = (va ? 1 : 0) | (vb ? 2 : 0);
    if (vec == 3) hipLaunchKernelGGL((gemm_kernel<BN, BK, EPI, 3>), grid, dim3(256), 0, s, g);
    else if (vec == 1) hipLaunchKernelGGL((gemm_kernel<BN, BK, EPI, 1>), grid, dim3(256), 0, s, g);
    else hipLaunchKernelGGL((gemm_kernel<BN, BK, EPI, 0>), grid, dim3(256), 0, s, g);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

// 64-deep K stages for narrow outputs (the emission projection, N = V <= 32:
// a latency-bound stream of A; measured 27.4 -> 17.2 us at C2), 16-deep
// otherwise (wide N is MFMA-bound and keeps more workgroups per CU with the
// smaller LDS tile: the C2 input projection ran 52.8 us at BK 16, 68.0 at 64).
template <int BN, int EPI>
static int launch_gemm_bn(const GemmArgs& g, hipStream_t s) {
    const int kmin = EPI == EPI_DUAL_TANH ? (g.K < g.K2 ? g.K : g.K2) : g.K;
    if constexpr (BN == 32) {
        if (kmin >= 128) return launch_gemm_bk<BN, 64, EPI>(g, s);
    }
    return launch_gemm_bk<BN, 16, EPI>(g, s);
}

template <int EPI>
static int launch_gemm_epi(const GemmArgs& g, hipStream_t s) {
    // the A stream as float4 rows: narrow outputs take the LDS-free A path
    const bool va = g.sak == 1 && (g.K % 4) == 0 && (g.sam % 4) == 0 && ((uintptr_t)g.A % 16) == 0;
    if (EPI != EPI_DUAL_TANH && g.N <= 64 && va) return launch_gemm_narrow<EPI>(g, s);
    int rc;
    if (try_gemm_wide<EPI>(g, s, rc)) return rc;
    if (g.N <= 32) return launch_gemm_bn<32, EPI>(g, s);
    return launch_gemm_bn<64, EPI>(g, s);
}

int gemm_launch(const GemmArgs& g, int epi, hipStream_t s) {
    if (g.M <= 0 || g.N <= 0 || g.K <= 0) return ASR_ERR_ARG;
    // fp32-accurate split-bf16 kernel (dense_x3.hip) for the shapes it takes;
    // the pipeline's short-workgroup request (asr_internal_gemm_tiled) runs it
    // in runs of that many row tiles instead of persistent workgroups
    if (dense_x3_on() && gemm_x3_applies(g, epi)) {
        const int rc = gemm_x3_launch(g, epi, asr_internal_gemm_tiled, s);
        if (rc != ASR_ERR_UNSUPPORTED) return rc;   // (K > 256 under stream capture: the fp32 kernels)
    }
    if (epi == EPI_LOGSOFTMAX && g.N > 64) {
        // Rows wider than one workgroup tile (e.g. C5's V = 1000): bias GEMM,
        // then a row-wise log_softmax pass in place (model.py:49).
        const int rc = gemm_launch(g, EPI_BIAS, s);
        if (rc) return rc;
        return row_logsoftmax_launch(g.C, g.ldc, g.M, g.N, s);
    }
    switch (epi) {
        case EPI_NONE: return launch_gemm_epi<EPI_NONE>(g, s);
        case EPI_BIAS: return launch_gemm_epi<EPI_BIAS>(g, s);
        case EPI_BIAS_RELU: return launch_gemm_epi<EPI_BIAS_RELU>(g, s);
        case EPI_LOGSOFTMAX: return launch_gemm_epi<EPI_LOGSOFTMAX>(g, s);
        case EPI_DUAL_TANH: return launch_gemm_epi<EPI_DUAL_TANH>(g, s);
        case EPI_ADD_TANH: return launch_gemm_epi<EPI_ADD_TANH>(g, s);
        default: return ASR_ERR_ARG;
    }
}

// ---------------------------------------------------------------------------
// RNN recurrence, H <= 256: h_t = tanh((P_t + h_{t-1}.W_hh) + (b_hh + b_ih))
// where P = x.W_ih was produced for all T by one GEMM into `hid`, which is
// overwritten in place by h.  One 1024-thread workgroup per utterance; thread
// (j, q) holds column j of W_hh for k in quarter q (64 registers), so W_hh is
// read from HBM once per utterance instead of once per step.  h_{t-1} is
// broadcast from LDS as [quarter][68] (conflict-free ds_read_b128).
// ---------------------------------------------------------------------------
// Workgroup barrier ordering LDS only: the step's global store of h_t (and
// the prefetch of P_{t+1}) stay in flight across it.  __syncthreads() orders
// global memory too, so every step waited for its store to reach memory
// (s_waitcnt vmcnt(0) before each s_barrier).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

constexpr int RNN_HMAX = 256;
constexpr int RNN_QS = 68;   // LDS stride of one quarter (floats)

template <bool PK>
__global__ __launch_bounds__(1024) void rnn_recur_kernel(const float* __restrict__ h0,
                                                         const float* __restrict__ Whh,
                                                         const float* __restrict__ b_ih,
                                                         const float* __restrict__ b_hh,
                                                         float* __restrict__ hid, int T, int B,
                                                         int H) {
    __shared__ __attribute__((aligned(16))) float hs[2][4 * RNN_QS];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int j = tid >> 2, q = tid & 3;
    const int KQ = (H + 3) >> 2;            // k per quarter
    const bool col = j < H;
    float w[64];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        const int k = q * KQ + i;
        w[i] = (col && i < KQ && k < H) ? Whh[(long)k * H + j] : 0.f;
    }
    for (int i = tid; i < 2 * 4 * RNN_QS; i += 1024) (&hs[0][0])[i] = 0.f;
    __syncthreads();
    if (tid < H) {
        const int qq = tid / KQ, ii = tid - qq * KQ;
        hs[0][qq * RNN_QS + ii] = h0 ? h0[(long)b * H + tid] : 0.f;
    }
    const float bias = col ? (b_hh[j] + b_ih[j]) : 0.f;
    const int jq = col ? j / KQ : 0, ji = col ? j - jq * KQ : 0;
    const bool writer = col && q == 0;
    // P_t / h_t of this utterance's column j at hid[t*B*H + b*H + j], through
    // one buffer resource per step (base uniform, B*H*4 bytes): lanes other
    // than the column's writer get an out-of-range offset, so their loads
    // return 0 and their stores are dropped.  No branch around the memory
    // ops, so the wait before each step only covers the prefetch of P_{t+1},
    // never the store of h_t.
    const long tstride = (long)B * H;
    const int nbytes = (int)(tstride * 4);
    const int voff = writer ? (b * H + j) * 4 : 0x7ffffff0;
    constexpr int RSRC3 = 0x00020000;   // gfx9 buffer descriptor word 3 (raw 32-bit data)
    float pnext = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
        __builtin_amdgcn_make_buffer_rsrc(hid, 0, nbytes, RSRC3), voff, 0, 0));
    __syncthreads();
    int cur = 0;
    for (int t = 0; t < T; t++) {
        const float p = pnext;
        float* base = hid + t * tstride;
        pnext = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            __builtin_amdgcn_make_buffer_rsrc(base + tstride, 0, t + 1 < T ? nbytes : 0, RSRC3), voff, 0, 0));
        const float4* hq = reinterpret_cast<const float4*>(&hs[cur][q * RNN_QS]);
        float acc = 0.f;
        if constexpr (PK) {
        // packed fp32 FMAs (v_pk_fma_f32: two k per lane per instruction),
        // even / odd k in the two halves, summed at the end
        typedef float f2v __attribute__((ext_vector_type(2)));
        f2v acc2 = {0.f, 0.f};
#pragma unroll
        for (int i4 = 0; i4 < 16; i4++) {
            const float4 h4 = hq[i4];
            const f2v ha = {h4.x, h4.y}, hb = {h4.z, h4.w};
            const f2v wa = {w[4 * i4 + 0], w[4 * i4 + 1]}, wb = {w[4 * i4 + 2], w[4 * i4 + 3]};
            acc2 = __builtin_elementwise_fma(ha, wa, acc2);
            acc2 = __builtin_elementwise_fma(hb, wb, acc2);
        }
        acc = acc2.x + acc2.y;
        } else {
        // one FMA chain: four independent chains measured slower (C2
        // recurrence 0.35 -> 0.46 ms, gpurun_out/r3m)
#pragma unroll
        for (int i4 = 0; i4 < 16; i4++) {
            const float4 h4 = hq[i4];
            acc = fmaf(h4.x, w[4 * i4 + 0], acc);
            acc = fmaf(h4.y, w[4 * i4 + 1], acc);
            acc = fmaf(h4.z, w[4 * i4 + 2], acc);
            acc = fmaf(h4.w, w[4 * i4 + 3], acc);
        }
        }
        acc += __shfl_xor(acc, 1);
        acc += __shfl_xor(acc, 2);
        const float h = tanhf((p + acc) + bias);
        if (writer) hs[cur ^ 1][jq * RNN_QS + ji] = h;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(h),
                                              __builtin_amdgcn_make_buffer_rsrc(base, 0, nbytes, RSRC3),
                                              voff, 0, 0);
        cur ^= 1;
        lds_barrier();
    }
}

int rnn_recur_launch(const float* h0, const float* Whh, const float* b_ih, const float* b_hh,
                     float* hid, int T, int B, int H, hipStream_t s) {
    if (H > RNN_HMAX) return ASR_ERR_UNSUPPORTED;
    if ((long)B * H * 4 > 0x7fffffe0L) return ASR_ERR_UNSUPPORTED;   // one step's rows per buffer resource
    // packed FMAs (two k per instruction)
    hipLaunchKernelGGL(rnn_recur_kernel<true>, dim3(B), dim3(1024), 0, s, h0, Whh, b_ih, b_hh, hid, T, B, H);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

// ---------------------------------------------------------------------------
// RNN recurrence on MFMA for large batches, H <= 256, H % 16 == 0:
// h_t = tanh((P_t + h_{t-1}.W_hh) + (b_hh + b_ih)), in place over P (as
// rnn_recur_kernel).  The VALU kernel above runs one utterance per CU, so
// its step is a GEMV whose 65k FMAs take ~2,200 cycles of dependent latency;
// at B >> CUs that is ~36 k CU-cycles per 16 utterance-steps.  Here a
// workgroup carries 16 utterances: one step is a [16 x H] . [H x H] GEMM on
// v_mfma_f32_16x16x4f32 (exact fp32), ~8 k cycles per 16 utterance-steps at
// H = 256 — compute-bound at the MFMA rate (64 FLOP/clk/SIMD).
//   * ceil(H/32) waves; wave w owns the 16-column tiles 2w and 2w + 1 and
//     keeps their W_hh columns in registers for the whole sequence (H/2
//     floats per lane: 128 VGPRs at H = 256, two waves per SIMD), loaded once.
//   * h_{t-1} (16 x H) lives in LDS, double-buffered: one barrier per step.
//     MFMA (i, e) of lane group g = lane >> 4 contracts k = 16i + 4g + e for
//     both operands (a bijection of the H k-slots), so each lane reads its A
//     fragments with one ds_read_b128 per 16 k, shared by its two tiles.
//   * Two accumulator chains per tile (even / odd 16-k chunks), summed at
//     the end: dependent MFMA latency (40 cycles) never stalls the issue.
//   * Epilogue per lane and tile: rows 4g + j (j < 4), column
//     16 tile + (lane & 15): P_t (prefetched one step ahead) + h.W_hh,
//     + bias, tanh (op order of RNN_Cell.cu:10-12); to LDS for the next
//     step and to hid.
// Grid ceil(B / 16); block 64 * ceil(H / 32) threads.
// ---------------------------------------------------------------------------
//
// EMIT (asr_rnn_emit_fwd): the emission projection + log_softmax of every
// h_t fused into the same kernel (Linear.cu:42-49, baseline/model.py:49),
// V <= 32, so the hidden states never go to HBM (C4: 2.1 GB written and read
// back per batch by a separate GEMM) and the projection runs on the
// recurrence's matrix cores: wave w contracts its own k-slice of h_t (the
// chunks 2w, 2w + 1 it already reads as A fragments) with W_out[k-slice][32]
// held in 16 VGPRs — 16 MFMAs beside its 128 recurrence MFMAs — and writes
// the 16 x 32 partial to LDS; one step later waves 0-3 sum the partials in
// wave order, add the bias and log-softmax each row with DPP reductions over
// the 16 lanes that hold it, and store.
// Pipelined: step t issues h_{t-1}'s partials and finishes h_{t-2}'s row.
// The contraction order (8 partial chains, then a fixed sum) differs from the
// GEMM kernels' single chain: emissions agree with asr_linear_fwd to fp32
// rounding, not bit for bit.
// ---------------------------------------------------------------------------
constexpr int RM_ROWS = 16;
constexpr int RM_LD = RNN_HMAX + 4;   // LDS row stride (floats): b128 reads of a quarter-wave hit distinct banks
constexpr int RM_NCH = RNN_HMAX / 16;  // 16-k chunks at H = 256
constexpr int RE_VMAX = 32;           // EMIT: vocabulary columns (two 16-column tiles)
constexpr int RE_PART = (RNN_HMAX / 32) * RM_ROWS * RE_VMAX;   // EMIT: one buffer of 8 waves' 16 x 32 partials

// HL: also write h_{T-1} to hlast (segmented production); a separate
// instance, so that the unsegmented kernel carries no extra state.
template <bool EMIT, bool HL = false>
__global__ __launch_bounds__(512) void rnn_recur_mfma_kernel(const float* h0,
                                                             const float* __restrict__ Whh,
                                                             const float* __restrict__ b_ih,
                                                             const float* __restrict__ b_hh,
                                                             float* hid, float* hout,
                                                             const float* __restrict__ Wout,
                                                             const float* __restrict__ bout,
                                                             float* __restrict__ emis, int T, int B,
                                                             int H, int V, float* hlast) {
    __shared__ __attribute__((aligned(16))) float hs[2][RM_ROWS * RM_LD];
    __shared__ __attribute__((aligned(16))) float ep[EMIT ? 2 : 1][EMIT ? RE_PART : 1];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int g = lane >> 4, c = lane & 15;
    const int nch = H >> 4;                 // 16-k chunks = 16-column tiles
    const int r0 = blockIdx.x * RM_ROWS;
    const int nthr = (int)blockDim.x;
    bool tv[2];                             // tile 2w + tt exists
    int n[2];                               // this lane's column in tile 2w + tt
#pragma unroll
    for (int tt = 0; tt < 2; tt++) {
        tv[tt] = 2 * w + tt < nch;
        n[tt] = tv[tt] ? (2 * w + tt) * 16 + c : 0;
    }
    // W_hh columns: wb[tt][i][e] = W_hh[16i + 4g + e][n[tt]]
    float wb[2][RM_NCH][4];
#pragma unroll
    for (int tt = 0; tt < 2; tt++)
#pragma unroll
        for (int i = 0; i < RM_NCH; i++)
#pragma unroll
            for (int e = 0; e < 4; e++)
                wb[tt][i][e] = (tv[tt] && i < nch) ? Whh[(long)(16 * i + 4 * g + e) * H + n[tt]] : 0.f;
    // h_{-1}: rows of h0 (zeros when NULL, RNN.h:15-16) into buffer 0
    for (int x = tid; x < RM_ROWS * H; x += nthr) {
        const int r = x / H, k = x - r * H;
        hs[0][r * RM_LD + k] = (h0 && r0 + r < B) ? h0[(long)(r0 + r) * H + k] : 0.f;
    }
    float bias[2];
#pragma unroll
    for (int tt = 0; tt < 2; tt++) bias[tt] = tv[tt] ? b_hh[n[tt]] + b_ih[n[tt]] : 0.f;
    const long tstride = (long)B * H;
    int rowoff[4];   // B * H < 2^31 (checked at launch)
    bool ok[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int r = r0 + 4 * g + j;
        ok[j] = r < B;
        rowoff[j] = (ok[j] ? r : 0) * H;
    }
    float pn[2][4];
#pragma unroll
    for (int tt = 0; tt < 2; tt++)
#pragma unroll
        for (int j = 0; j < 4; j++) pn[tt][j] = (tv[tt] && ok[j]) ? hid[rowoff[j] + n[tt]] : 0.f;
    // EMIT: hidden states go to hout (NULL: nowhere); otherwise in place over P
    float* const hdst = EMIT ? hout : hid;
    // EMIT: wo[ii][vt][e] = W_out[16 (2w + ii) + 4g + e][16 vt + c] (zero past H or V)
    float wo[2][2][4];
    float bo0 = 0.f, bo1 = 0.f;
    if (EMIT) {
#pragma unroll
        for (int ii = 0; ii < 2; ii++)
#pragma unroll
            for (int vt = 0; vt < 2; vt++)
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const int k = 16 * (2 * w + ii) + 4 * g + e, col = 16 * vt + c;
                    wo[ii][vt][e] = (2 * w + ii < nch && col < V) ? Wout[(long)k * V + col] : 0.f;
                }
        bo0 = c < V ? bout[c] : 0.f;
        bo1 = 16 + c < V ? bout[16 + c] : 0.f;
    }
    // EMIT: wave w's partial of h . W_out over its k-slice (chunks 2w, 2w + 1
    // of the h held in hs[buf])
    auto emit_partial = [&](int buf, f32x4 (&ea)[2]) {
        ea[0] = f32x4{0.f, 0.f, 0.f, 0.f};
        ea[1] = f32x4{0.f, 0.f, 0.f, 0.f};
        const float* hr = &hs[buf][c * RM_LD + 4 * g];
#pragma unroll
        for (int ii = 0; ii < 2; ii++) {
            const int i = 2 * w + ii;
            if (i < nch) {
                const float4 a = *reinterpret_cast<const float4*>(hr + 16 * i);
#pragma unroll
                for (int vt = 0; vt < 2; vt++) {
                    ea[vt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, wo[ii][vt][0], ea[vt], 0, 0, 0);
                    ea[vt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, wo[ii][vt][1], ea[vt], 0, 0, 0);
                    ea[vt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, wo[ii][vt][2], ea[vt], 0, 0, 0);
                    ea[vt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, wo[ii][vt][3], ea[vt], 0, 0, 0);
                }
            }
        }
    };
    // ... to partial buffer s & 1, in C-fragment order: [wave][j][lane][vt]
    // (one ds_write_b64 per j, a wave's 64 lanes contiguous)
    auto store_partial = [&](int s, const f32x4 (&ea)[2]) {
        float* pp = &ep[s & 1][w * 4 * 128];
#pragma unroll
        for (int j = 0; j < 4; j++)
            *reinterpret_cast<float2*>(pp + j * 128 + 2 * lane) = float2{ea[0][j], ea[1][j]};
    };
    // EMIT: emissions of frame s from partial buffer s & 1.  Wave w < 4 owns
    // the rows 4g + w of the tile (register j = w of the C fragments): lane
    // (g, c) sums the waves' partials of its two columns c, 16 + c in wave
    // order (absent waves' buffers hold zeros), + b_out, and the row's
    // log_softmax over its 32 columns is a reduction over the 16 lanes of the
    // lane group — one DPP row (quad_perm xor 1, xor 2, half-mirror, mirror),
    // no LDS round trips.  Fewer than 4 waves (H < 128): a wave takes
    // several j.
    constexpr int NWMAX = RNN_HMAX / 32;
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
    const int nwblk = (int)blockDim.x >> 6;
    auto emit_rows = [&](int s, bool store) {
        const float* pp = ep[s & 1];
        for (int j = w; j < 4; j += nwblk) {
            float v0 = 0.f, v1 = 0.f;
#pragma unroll
            for (int q = 0; q < NWMAX; q++) {
                const float2 x = *reinterpret_cast<const float2*>(pp + (q * 4 + j) * 128 + 2 * lane);
                v0 += x.x;
                v1 += x.y;
            }
            v0 = c < V ? v0 + bo0 : -INFINITY;
            v1 = 16 + c < V ? v1 + bo1 : -INFINITY;
            const float mx = dpp_max16(fmaxf(v0, v1));
            const float se = dpp_sum16((c < V ? expf(v0 - mx) : 0.f) + (16 + c < V ? expf(v1 - mx) : 0.f));
            const float lz = mx + logf(se);
            const int row = r0 + 4 * g + j;
            if (store && row < B) {
                float* er = emis + ((long)s * B + row) * V;
                if (c < V) er[c] = v0 - lz;
                if (16 + c < V) er[16 + c] = v1 - lz;
            }
        }
    };
    if (EMIT) {
        for (int x = tid; x < 2 * RE_PART; x += nthr) (&ep[0][0])[x] = 0.f;
    }
    __syncthreads();
    int cur = 0;
    for (int t = 0; t < T; t++) {
        float p[2][4];
#pragma unroll
        for (int tt = 0; tt < 2; tt++)
#pragma unroll
            for (int j = 0; j < 4; j++) p[tt][j] = pn[tt][j];
        float* base = hid + (long)t * tstride;
        if (t + 1 < T) {
#pragma unroll
            for (int tt = 0; tt < 2; tt++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    pn[tt][j] = (tv[tt] && ok[j]) ? base[tstride + rowoff[j] + n[tt]] : 0.f;
        }
        const float* hrow = &hs[cur][c * RM_LD + 4 * g];
        f32x4 acc[2][2];
#pragma unroll
        for (int tt = 0; tt < 2; tt++)
#pragma unroll
            for (int u = 0; u < 2; u++) acc[tt][u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < RM_NCH; i++) {
            if (i < nch) {
                const float4 a = *reinterpret_cast<const float4*>(hrow + 16 * i);
#pragma unroll
                for (int tt = 0; tt < 2; tt++) {
                    f32x4& q = acc[tt][i & 1];
                    q = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, wb[tt][i][0], q, 0, 0, 0);
                    q = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, wb[tt][i][1], q, 0, 0, 0);
                    q = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, wb[tt][i][2], q, 0, 0, 0);
                    q = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, wb[tt][i][3], q, 0, 0, 0);
                }
            }
        }
        if (EMIT) {
            // beside this step's MFMAs: h_{t-1}'s partials (h_{t-1} is in
            // hs[cur]; at t = 0 a dummy into the other buffer, never read)
            // and h_{t-2}'s emissions (their partials were stored last step)
            f32x4 ea[2];
            emit_partial(cur, ea);
            emit_rows(t - 2, t >= 2);
            store_partial(t - 1 + 2, ea);
        }
        float* hn = hs[cur ^ 1];
#pragma unroll
        for (int tt = 0; tt < 2; tt++) {
            const f32x4 sum = acc[tt][0] + acc[tt][1];
            if (!tv[tt]) continue;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float h = tanhf((p[tt][j] + sum[j]) + bias[tt]);
                hn[(4 * g + j) * RM_LD + n[tt]] = h;
                if (ok[j] && (!EMIT || hdst)) hdst[(long)t * tstride + rowoff[j] + n[tt]] = h;
            }
        }
        cur ^= 1;
        lds_barrier();
    }
    if (HL && hlast) {   // h_{T-1} of this workgroup's rows (may be h0's buffer: every row is read above)
        for (int x = tid; x < RM_ROWS * H; x += nthr) {
            const int r = x / H, k = x - r * H;
            if (r0 + r < B) hlast[(long)(r0 + r) * H + k] = hs[cur][r * RM_LD + k];
        }
    }
    if (EMIT) {   // the last two frames' emissions
        f32x4 ea[2];
        emit_partial(cur, ea);   // h_{T-1}
        if (T >= 2) emit_rows(T - 2, true);
        store_partial(T - 1, ea);
        lds_barrier();
        emit_rows(T - 1, true);
    }
}

int rnn_recur_mfma_launch(const float* h0, const float* Whh, const float* b_ih, const float* b_hh,
                          float* hid, int T, int B, int H, hipStream_t s) {
    if (dense_x3_on() && rnn_x3_applies(B, H)) return rnn_recur_x3_launch(h0, Whh, b_ih, b_hh, hid, T, B, H, s);
    if (H > RNN_HMAX || (H & 15) != 0 || B <= 0) return ASR_ERR_UNSUPPORTED;
    if ((long)B * H > 0x7fffffffL) return ASR_ERR_UNSUPPORTED;   // 32-bit offsets within a step
    hipLaunchKernelGGL(rnn_recur_mfma_kernel<false>, dim3((unsigned)((B + RM_ROWS - 1) / RM_ROWS)),
                       dim3(64 * ((H / 16 + 1) / 2)), 0, s,
                       h0, Whh, b_ih, b_hh, hid, nullptr, nullptr, nullptr, nullptr, T, B, H, 0, nullptr);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

int rnn_emit_mfma_launch(const float* h0, const float* Whh, const float* b_ih, const float* b_hh,
                         const float* P, float* hout, const float* Wout, const float* bout, float* emis,
                         int T, int B, int H, int V, hipStream_t s, float* hlast, bool pfrag) {
    if (dense_x3_on() && rnn_x3_applies(B, H) && V >= 1 && V <= RE_VMAX)
        return rnn_emit_x3_launch(h0, Whh, b_ih, b_hh, P, hout, Wout, bout, emis, T, B, H, V, s, hlast, pfrag);
    if (pfrag) return ASR_ERR_UNSUPPORTED;   // the fragment-major P layout is the split-bf16 kernel's
    if (H > RNN_HMAX || (H & 15) != 0 || B <= 0 || V < 1 || V > RE_VMAX) return ASR_ERR_UNSUPPORTED;
    if ((long)B * H > 0x7fffffffL) return ASR_ERR_UNSUPPORTED;   // 32-bit offsets within a step
    if (hlast)
        hipLaunchKernelGGL((rnn_recur_mfma_kernel<true, true>), dim3((unsigned)((B + RM_ROWS - 1) / RM_ROWS)),
                           dim3(64 * ((H / 16 + 1) / 2)), 0, s,
                           h0, Whh, b_ih, b_hh, const_cast<float*>(P), hout, Wout, bout, emis, T, B, H, V, hlast);
    else
        hipLaunchKernelGGL((rnn_recur_mfma_kernel<true, false>), dim3((unsigned)((B + RM_ROWS - 1) / RM_ROWS)),
                           dim3(64 * ((H / 16 + 1) / 2)), 0, s,
                           h0, Whh, b_ih, b_hh, const_cast<float*>(P), hout, Wout, bout, emis, T, B, H, V, nullptr);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

// ---------------------------------------------------------------------------
// One recurrence step for H > 256 (W_hh too large to stay on one CU):
// h_t = tanh((P_t + h_{t-1}.W_hh) + (b_hh + b_ih)) in place over P_t
// (RNN_Cell.cu:10-12 order).  Small M (the batch) and wide N: each
// workgroup owns 8 output columns for 32 batch rows; its W_hh column slice
// [H][8] is staged in LDS once, h_{t-1} rows are read as float4 (the 8
// threads of a row read the same addresses).  Grid (H/8, ceil(B/32)).
constexpr int RS_COLS = 8;
constexpr int RS_KS = 4;   // K split: 4 x 256 threads, partial sums combined in LDS

__global__ __launch_bounds__(256 * RS_KS) void rnn_step_kernel(float* __restrict__ ht,
                                                               const float* __restrict__ hp,
                                                               const float* __restrict__ Whh,
                                                               const float* __restrict__ b_ih,
                                                               const float* __restrict__ b_hh, int B,
                                                               int H) {
    // ws[c][k]: the workgroup's W_hh columns, column-major with a padded
    // stride (float4 reads; the 8 columns of a wave hit distinct banks),
    // staged with float4 loads.  h_{t-1} rows stream from L2 as float4; the
    // K range is split over 4 thread groups so that each dependent-latency
    // chain is a quarter as long, 16 loads in flight per thread.
    extern __shared__ float ws[];
    const int ld = H + 4;
    float* part = ws + RS_COLS * ld;   // [RS_KS][256] partial sums
    const int n0 = blockIdx.x * RS_COLS, r0 = blockIdx.y * 32;
    const int tid = threadIdx.x;
    for (int i = tid; i < H * (RS_COLS / 4); i += 256 * RS_KS) {   // H % 8 == 0
        const int k = i / (RS_COLS / 4), c4 = (i - k * (RS_COLS / 4)) * 4;
        const float4 v = *reinterpret_cast<const float4*>(Whh + (long)k * H + n0 + c4);
        ws[(c4 + 0) * ld + k] = v.x;
        ws[(c4 + 1) * ld + k] = v.y;
        ws[(c4 + 2) * ld + k] = v.z;
        ws[(c4 + 3) * ld + k] = v.w;
    }
    __syncthreads();
    const int ks = tid / 256, o = tid % 256;
    const int r = r0 + o / RS_COLS, c = o % RS_COLS, n = n0 + c;
    const int q4 = H / 4, kb = ks * q4 / RS_KS, ke = (ks + 1) * q4 / RS_KS;
    float acc = 0.f;
    if (r < B) {
        const float4* h4 = reinterpret_cast<const float4*>(hp + (long)r * H);
        const float4* w4 = reinterpret_cast<const float4*>(ws + c * ld);
#pragma unroll 16
        for (int k4 = kb; k4 < ke; k4++) {
            const float4 v = h4[k4], w = w4[k4];
            acc = fmaf(v.x, w.x, acc);
            acc = fmaf(v.y, w.y, acc);
            acc = fmaf(v.z, w.z, acc);
            acc = fmaf(v.w, w.w, acc);
        }
    }
    part[ks * 256 + o] = acc;
    __syncthreads();
    if (ks != 0 || r >= B) return;
    const float hh = ((part[o] + part[256 + o]) + part[512 + o]) + part[768 + o];
    float* out = ht + (long)r * H + n;
    *out = tanhf((*out + hh) + (b_hh[n] + b_ih[n]));
}

int rnn_step_launch(float* ht, const float* hp, const float* Whh, const float* b_ih,
                    const float* b_hh, int B, int H, hipStream_t s) {
    const size_t lds = sizeof(float) * ((size_t)(H + 4) * RS_COLS + 256 * RS_KS);
    if ((H % RS_COLS) != 0) return ASR_ERR_UNSUPPORTED;   // float4 column slices
    if (lds > 160 * 1024) return ASR_ERR_UNSUPPORTED;
    static AsrAttrOnce attr;
    if (int r_ = attr.set((const void*)rnn_step_kernel, 160 * 1024)) return r_;
    const dim3 grid((unsigned)((H + RS_COLS - 1) / RS_COLS), (unsigned)((B + 31) / 32));
    hipLaunchKernelGGL(rnn_step_kernel, grid, dim3(256 * RS_KS), lds, s, ht, hp, Whh, b_ih, b_hh, B, H);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

// ---------------------------------------------------------------------------
// One recurrence step on MFMA for H % 128 == 0 (C5: H = 1024, BL: 2048):
// h_t = tanh((P_t + h_{t-1}.W_hh) + (b_hh + b_ih)) in place over P_t.
// A workgroup owns a (16 RB rows) x (16 NT columns) tile; its 8 waves split
// K eight ways (H/8 each) so that one step costs ~H/8/4 dependent MFMAs per
// tile instead of the whole K chain.  No LDS staging: every wave issues the
// operand loads of CH 16-k chunks of its K slice before their MFMAs (h rows
// as float4, W_hh columns as 64-B row segments), then one LDS exchange sums
// the eight partial tiles in a fixed order.  k assignment inside a 16-k
// chunk: MFMA j of lane group g = lane>>4 takes k = 4g + j for both operands
// (any bijection is a valid contraction).  Every output is the same chain
// (its wave's k in order, then the 8 partials in wave order) for any (RB,
// NT), so the tiling never changes a bit and can follow the shape: wider
// tiles re-read h_{t-1} and W_hh fewer times (BL, B = 256, H = 2048:
// 16-column tiles read 384 MB per step from L2 for a 2 GFLOP product).
// Grid (H / (16 NT), ceil(B / (16 RB))).
// Several batches in one step (StepRows, the pipeline's production groups,
// DESIGN.md §7d): batch j's rows are row tiles [j * tiles, (j + 1) * tiles)
// of the grid, with its own h_t / h_{t-1} pointers; B % (16 RB) == 0 then, so
// no tile straddles two batches.  Every row's arithmetic is the one-batch
// kernel's, so grouping never changes a bit.
constexpr int RSM_WAVES = 8;
struct StepRows {
    float* ht[STEP_MAXB];
    const float* hp[STEP_MAXB];
    int tiles;   // row tiles per batch
};
template <int RB, int NT>
__global__ __launch_bounds__(64 * RSM_WAVES) void rnn_step_mfma_kernel(StepRows sr,
                                                                      const float* __restrict__ Whh,
                                                                      const float* __restrict__ b_ih,
                                                                      const float* __restrict__ b_hh,
                                                                      int B, int H) {
    __shared__ f32x4 part[RSM_WAVES][RB * NT][64];
    constexpr int CH = (RB * NT >= 4) ? 4 : 8;   // 16-k chunks whose loads are in flight together
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int bj = (int)blockIdx.y / sr.tiles;
    float* __restrict__ ht = sr.ht[bj];
    const float* __restrict__ hp = sr.hp[bj];
    const int n0 = blockIdx.x * (16 * NT), r0 = ((int)blockIdx.y - bj * sr.tiles) * (16 * RB);
    const int g = lane >> 4, c = lane & 15;
    const int kw = H / RSM_WAVES, kbeg = w * kw, nchunk = kw / 16;
    const float* arow[RB];
#pragma unroll
    for (int rb = 0; rb < RB; rb++) {
        const int r = min(r0 + rb * 16 + c, B - 1);   // rows past B: valid memory, never stored
        arow[rb] = hp + (long)r * H + kbeg + 4 * g;
    }
    const float* bcol = Whh + (long)(kbeg + 4 * g) * H + n0 + c;
    f32x4 acc[RB][NT];
#pragma unroll
    for (int rb = 0; rb < RB; rb++)
#pragma unroll
        for (int nt = 0; nt < NT; nt++) acc[rb][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ch0 = 0; ch0 < nchunk; ch0 += CH) {
        float4 a[CH][RB];
        float b[CH][NT][4];
#pragma unroll
        for (int i = 0; i < CH; i++) {
            if (ch0 + i < nchunk) {
                const int k = (ch0 + i) * 16;
#pragma unroll
                for (int rb = 0; rb < RB; rb++) a[i][rb] = *reinterpret_cast<const float4*>(arow[rb] + k);
#pragma unroll
                for (int nt = 0; nt < NT; nt++)
#pragma unroll
                    for (int j = 0; j < 4; j++) b[i][nt][j] = bcol[(long)(k + j) * H + 16 * nt];
            }
        }
#pragma unroll
        for (int i = 0; i < CH; i++) {
            if (ch0 + i < nchunk) {
#pragma unroll
                for (int rb = 0; rb < RB; rb++)
#pragma unroll
                    for (int nt = 0; nt < NT; nt++) {
                        f32x4& q = acc[rb][nt];
                        q = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][rb].x, b[i][nt][0], q, 0, 0, 0);
                        q = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][rb].y, b[i][nt][1], q, 0, 0, 0);
                        q = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][rb].z, b[i][nt][2], q, 0, 0, 0);
                        q = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][rb].w, b[i][nt][3], q, 0, 0, 0);
                    }
            }
        }
    }
#pragma unroll
    for (int rb = 0; rb < RB; rb++)
#pragma unroll
        for (int nt = 0; nt < NT; nt++) part[w][rb * NT + nt][lane] = acc[rb][nt];
    __syncthreads();
    // thread -> (tile, j, lane) of the 16x16 tiles; the C/D layout: element j
    // of lane l is row (l>>4)*4 + j, column l & 15.
    for (int e = tid; e < RB * NT * 256; e += 64 * RSM_WAVES) {
        const int tl = e >> 8, j = (e >> 6) & 3, l = e & 63;
        const int rb = tl / NT, nt = tl - rb * NT;
        const int r = r0 + rb * 16 + (l >> 4) * 4 + j, n = n0 + nt * 16 + (l & 15);
        if (r >= B) continue;
        float hh = part[0][tl][l][j];
#pragma unroll
        for (int q = 1; q < RSM_WAVES; q++) hh += part[q][tl][l][j];
        float* out = ht + (long)r * H + n;
        *out = tanhf((*out + hh) + (b_hh[n] + b_ih[n]));
    }
}

template <int RB, int NT>
static void launch_step_mfma(StepRows sr, int nb, const float* Whh, const float* b_ih, const float* b_hh,
                             int B, int H, hipStream_t s) {
    sr.tiles = (B + 16 * RB - 1) / (16 * RB);
    hipLaunchKernelGGL((rnn_step_mfma_kernel<RB, NT>), dim3((unsigned)(H / (16 * NT)), (unsigned)(nb * sr.tiles)),
                       dim3(64 * RSM_WAVES), 0, s, sr, Whh, b_ih, b_hh, B, H);
}

int rnn_step_mfma_launch(float* ht, const float* hp, const float* Whh, const float* b_ih,
                         const float* b_hh, int B, int H, hipStream_t s) {
    return rnn_step_mfma_multi_launch(&ht, &hp, 1, Whh, b_ih, b_hh, B, H, s);
}

int rnn_step_mfma_multi_launch(float* const* hts, const float* const* hps, int nb, const float* Whh,
                               const float* b_ih, const float* b_hh, int B, int H, hipStream_t s) {
    if (B <= 0 || H <= 0 || (H % 128) != 0 || nb < 1 || nb > STEP_MAXB) return ASR_ERR_UNSUPPORTED;
    StepRows sr{};
    for (int j = 0; j < nb; j++) {
        if ((uintptr_t)hps[j] % 16 != 0) return ASR_ERR_UNSUPPORTED;   // float4 rows
        sr.ht[j] = hts[j];
        sr.hp[j] = hps[j];
    }
    // several batches: whole row tiles per batch
    if (nb > 1 && B % 16 != 0) return ASR_ERR_UNSUPPORTED;
    const int Btot = B * nb;
    // ASR_RNN_STEP_NT=1/2/4 forces the column tiles per workgroup (A/B)
    const char* fe = getenv("ASR_RNN_STEP_NT");
    int nt = fe ? atoi(fe) : 0;
    const long nb16 = (Btot + 15) / 16, nb32 = (Btot + 31) / 32;
    const bool rb2 = nb == 1 || B % 32 == 0;   // 32-row tiles must not straddle batches
    if (nt != 1 && nt != 2 && nt != 4) {
        // the widest tiles that still give every CU a workgroup (256 CUs:
        // BL's 256 x 2048 -> 32 x 8 = 256 workgroups of 32 x 64); narrow
        // tiles for small B (C5's 32 x 1024: latency-bound, 64 x 2)
        nt = (H / 64) * nb32 >= 256 ? 4 : ((H / 32) * nb32 >= 256 ? 2 : 1);
    }
    if (!rb2) nt = 1;
    if (nt == 4) {
        launch_step_mfma<2, 4>(sr, nb, Whh, b_ih, b_hh, B, H, s);
    } else if (nt == 2) {
        launch_step_mfma<2, 2>(sr, nb, Whh, b_ih, b_hh, B, H, s);
    } else if ((H / 16) * nb16 <= 512 || !rb2) {   // 16-row tiles while that is <= 2 per CU
        launch_step_mfma<1, 1>(sr, nb, Whh, b_ih, b_hh, B, H, s);
    } else {   // 32-row tiles (measured: 16-row tiles win up to ~2 workgroups per CU, 64-row
               // tiles and 16 waves per workgroup lose everywhere)
        launch_step_mfma<2, 1>(sr, nb, Whh, b_ih, b_hh, B, H, s);
    }
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

// ---------------------------------------------------------------------------
// The whole H > 256 recurrence in ONE launch (C5: B = 32, H = 1024, T =
// 2000), replacing the T step launches above with the same bits: every
// workgroup is the step kernel's (16 RB x 16 NT) tile with its 8-way K split,
// but its W_hh slice (K/8 x 16 NT floats per wave: 64 VGPRs at H = 1024, NT
// = 2) stays in registers for all T frames, and the workgroups hand h_t to
// each other through memory inside the launch:
//   * h_t is stored write-through (buffer stores with the sc1 bit) into hid
//     (its final place); every storing wave drains its stores (vmcnt(0)),
//     the workgroup barriers, and one lane adds 1 to the launch's step
//     counter (agent-scope atomic);
//   * before frame t a workgroup's first lane polls the counter (agent-scope
//     relaxed loads, s_sleep between) until all nWG workgroups have
//     published frame t - 1, the workgroup barriers, and every load of
//     h_{t-1} (and of P_t) is a buffer load with the sc1 bit (not served
//     from this CU's L1) — the hand-off form of cdna_hip_programming.md §6
//     Guideline 16 (one workgroup per CU: the launch requests more than half
//     of a CU's LDS);
//   * P_t does not depend on h_{t-1}: each thread loads its P_t before the
//     wait, so that load is off the step's critical path (C5 production
//     20.0 -> 18.5 ms per batch).
// Every workgroup must be resident at once.  The launcher only takes grids
// of at most `cus` workgroups (the CUs the caller's stream may use), but
// residency is not guaranteed (other work on the same CUs, another process,
// a one-launch recurrence of another stream), so the launch is fail-safe:
//   * a wait without progress for 0.5 s sets the launch's abort word, and
//     every workgroup that sees it (waiting, or dispatched late) exits;
//   * a one-workgroup recovery kernel follows on the stream: it exits at
//     once unless the abort word is set, and then computes every frame a
//     tile had not published (prog[wg], written as each workgroup leaves:
//     the frame it stopped at; it differs by at most one frame between
//     workgroups) with the same arithmetic, so the call's bits are
//     those of an undisturbed launch (slower, never wrong);
//   * each launch owns its control block (counter, abort word, prog[]) until
//     an event recorded after its recovery kernel has completed.
// The arithmetic per output is the step kernel's: each wave's K slice in
// chunk order (4 MFMAs per 16-k chunk, k = 16 i + 4 g + j), the 8 partials
// summed in wave order, tanhf((P_t + hh) + (b_hh + b_ih)); frame 0 without
// h0 is bias_tanh's tanhf(P_0 + (b_hh + b_ih)).
constexpr int RP_LDS = 96 * 1024;   // one workgroup per CU
constexpr int RP_SC1 = 16;          // buffer-instruction cache policy: sc1 (write-through / coherent)
constexpr int RP_MAXWG = (1024 / 32) * (256 / 16);        // H <= 1024 (NT = 2), B <= 256
constexpr unsigned long long RP_TIMEOUT = 50000000ull;   // 0.5 s of s_memrealtime (100 MHz)

// One launch's control block (device memory; the head is zeroed on the
// stream before the launch).
// The counter, the abort word and the progress words sit on separate
// 256-byte lines: with all three on one line (round 6's first layout) every
// workgroup's progress store contended with the polled counter (C5's
// recurrence 4.9 -> 6.4 us per frame).
struct PersistCtl {
    unsigned ctr;              // publications: one per workgroup and frame
    unsigned pad0[63];
    unsigned abort;            // 1: a workgroup gave up waiting
    unsigned pad1[63];
    unsigned prog[RP_MAXWG];   // frames published, per workgroup
};

// This thread's share of one tile: its W_hh slice, A-row offsets and
// output slots (the same for every frame).
template <int RB, int NT, int KCH>
struct RpTile {
    static constexpr int EPT = RB * NT * 256 / (64 * RSM_WAVES);   // outputs per thread
    static_assert(EPT * 64 * RSM_WAVES == RB * NT * 256, "outputs per thread");
    float bw[KCH][NT][4];
    int arow[RB];
    int eoff[EPT], etl[EPT], el[EPT], ej[EPT];
    float ebias[EPT];

    __device__ __forceinline__ void setup(const float* __restrict__ Whh, const float* __restrict__ b_ih,
                                          const float* __restrict__ b_hh, int bx, int by, int B, int H) {
        const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
        const int g = lane >> 4, c = lane & 15;
        const int n0 = bx * (16 * NT), r0 = by * (16 * RB);
        const int kbeg = w * (H / RSM_WAVES);
        // this wave's W_hh slice: chunk i, tile nt, MFMA j -> W[kbeg + 16 i + 4 g + j][n0 + 16 nt + c]
#pragma unroll
        for (int i = 0; i < KCH; i++)
#pragma unroll
            for (int nt = 0; nt < NT; nt++)
#pragma unroll
                for (int j = 0; j < 4; j++) bw[i][nt][j] = Whh[(long)(kbeg + 16 * i + 4 * g + j) * H + n0 + 16 * nt + c];
        // row offsets (floats) of this lane's A rows: rows past B read row B - 1 (never stored)
#pragma unroll
        for (int rb = 0; rb < RB; rb++) arow[rb] = min(r0 + rb * 16 + c, B - 1) * H + kbeg + 4 * g;
        // this thread's outputs: their byte offset in a frame and (b_hh + b_ih)
#pragma unroll
        for (int k = 0; k < EPT; k++) {
            const int e = tid + k * 64 * RSM_WAVES;
            const int tl = e >> 8, j = (e >> 6) & 3, l = e & 63;
            const int rb = tl / NT, nt = tl - rb * NT;
            const int r = r0 + rb * 16 + (l >> 4) * 4 + j, n = n0 + nt * 16 + (l & 15);
            eoff[k] = (r * H + n) * 4;   // rows past B: past the resource (load 0, store dropped)
            etl[k] = tl;
            el[k] = l;
            ej[k] = j;
            ebias[k] = b_hh[n] + b_ih[n];
        }
    }

    // P_t of this thread's outputs (coherent loads)
    __device__ __forceinline__ void load_p(__amdgpu_buffer_rsrc_t rs_t, float (&Pv)[EPT]) const {
#pragma unroll
        for (int k = 0; k < EPT; k++)
            Pv[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_t, eoff[k], 0, RP_SC1));
    }

    // h_t = tanhf((P_t + h_{t-1}.W_hh) + bias) of this thread's outputs (hp:
    // h_{t-1}; NULL: h_{-1} = 0, bias_tanh's formula), stored write-through.
    // rp_part: the workgroup's partial products (LDS); one barrier inside.
    template <bool HOIST>
    __device__ __forceinline__ void frame(const float* hp, int sbytes, __amdgpu_buffer_rsrc_t rs_t,
                                          const float (&Pv)[EPT], f32x4* rp_part) const {
        const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
        if (hp) {
            const auto rs_p = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(hp), (short)0, sbytes, 0x00020000);
            f32x4 acc[RB][NT];
#pragma unroll
            for (int rb = 0; rb < RB; rb++)
#pragma unroll
                for (int nt = 0; nt < NT; nt++) acc[rb][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
            f32x4 a[KCH][RB];
#pragma unroll
            for (int i = 0; i < KCH; i++)
#pragma unroll
                for (int rb = 0; rb < RB; rb++)
                    a[i][rb] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                             rs_p, (arow[rb] + 16 * i) * 4, 0, RP_SC1));
            // every load of h_{t-1} in flight before the first MFMA (the
            // scheduler otherwise keeps two in flight: KCH / 2 round trips)
            if constexpr (HOIST) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < KCH; i++)
#pragma unroll
                for (int rb = 0; rb < RB; rb++)
#pragma unroll
                    for (int nt = 0; nt < NT; nt++) {
                        f32x4& q = acc[rb][nt];
                        q = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][rb].x, bw[i][nt][0], q, 0, 0, 0);
                        q = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][rb].y, bw[i][nt][1], q, 0, 0, 0);
                        q = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][rb].z, bw[i][nt][2], q, 0, 0, 0);
                        q = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][rb].w, bw[i][nt][3], q, 0, 0, 0);
                    }
#pragma unroll
            for (int rb = 0; rb < RB; rb++)
#pragma unroll
                for (int nt = 0; nt < NT; nt++) rp_part[(w * RB * NT + rb * NT + nt) * 64 + lane] = acc[rb][nt];
            __syncthreads();
#pragma unroll
            for (int k = 0; k < EPT; k++) {
                const int tl = etl[k], l = el[k], j = ej[k];
                float hh = rp_part[tl * 64 + l][j];
#pragma unroll
                for (int q = 1; q < RSM_WAVES; q++) hh += rp_part[(q * RB * NT + tl) * 64 + l][j];
                const float y = tanhf((Pv[k] + hh) + ebias[k]);
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), rs_t, eoff[k], 0, RP_SC1);
            }
        } else {   // h_{-1} = 0: bias_tanh's formula
#pragma unroll
            for (int k = 0; k < EPT; k++) {
                const float y = tanhf(Pv[k] + ebias[k]);
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), rs_t, eoff[k], 0, RP_SC1);
            }
        }
    }
};

// fault_frame >= 1 (test hook ASR_RNN_PERSIST_FAULT): workgroup (0, 0)
// stalls before that frame, as if it had lost its CU, until the others give
// up (bounded: 2 s); then the launch ends aborted and the recovery kernel
// finishes it.
template <int RB, int NT, int KCH, bool HOIST>
__global__ __launch_bounds__(64 * RSM_WAVES) void rnn_recur_persist_kernel(const float* h0,
                                                                          const float* __restrict__ Whh,
                                                                          const float* __restrict__ b_ih,
                                                                          const float* __restrict__ b_hh,
                                                                          float* hid, int T, int B, int H,
                                                                          PersistCtl* ctl, int* host_status,
                                                                          int fault_frame) {
    extern __shared__ __attribute__((aligned(16))) f32x4 rp_part[];   // [RSM_WAVES][RB * NT][64], then the abort flag
    int& rp_abort = *reinterpret_cast<int*>(rp_part + RSM_WAVES * RB * NT * 64);
    using Tile = RpTile<RB, NT, KCH>;
    constexpr int EPT = Tile::EPT;
    const int tid = threadIdx.x;
    const unsigned nwg = gridDim.x * gridDim.y;
    const unsigned wg = blockIdx.y * gridDim.x + blockIdx.x;
    Tile tile;
    tile.setup(Whh, b_ih, b_hh, blockIdx.x, blockIdx.y, B, H);
    if (tid == 0)   // dispatched after the launch gave up: leave every frame to the recovery
        rp_abort = (int)__hip_atomic_load(&ctl->abort, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (rp_abort) return;
    const long slab = (long)B * H;
    const int sbytes = (int)(slab * 4);
    for (int t = 0; t < T; t++) {
        float* ht = hid + (long)t * slab;
        const float* hp = t > 0 ? hid + (long)(t - 1) * slab : h0;
        // P_t (the input projection, in place in h_t) does not depend on
        // h_{t-1}: loaded before the wait for frame t - 1
        const auto rs_t = __builtin_amdgcn_make_buffer_rsrc(ht, (short)0, sbytes, 0x00020000);
        float Pv[EPT];
        tile.load_p(rs_t, Pv);
        if (t > 0) {   // every workgroup has published frame t - 1
            if (tid == 0) {
                const unsigned target = nwg * (unsigned)t;
                unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                if (t == fault_frame && wg == 0) {   // test hook: stall until the launch is aborted
                    while (!__hip_atomic_load(&ctl->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &&
                           __builtin_amdgcn_s_memrealtime() - t0 < 4 * RP_TIMEOUT)
                        __builtin_amdgcn_s_sleep(8);
                    rp_abort = 1;
                }
                // the poll is one L2 round trip; the abort word and the clock
                // are read every 16th poll only (a frame's wait is a few
                // us, the abort's reaction stays far below the timeout):
                // reading both on every poll doubled its period (C5's
                // recurrence 5.9 -> 6.6 us per frame)
                bool ab = rp_abort != 0;
                unsigned spins = 0;
                while (!ab && __hip_atomic_load(&ctl->ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                    __builtin_amdgcn_s_sleep(2);
                    if ((++spins & 15u) != 0u) continue;
                    if (__hip_atomic_load(&ctl->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                        ab = true;
                    } else if (__builtin_amdgcn_s_memrealtime() - t0 > RP_TIMEOUT) {
                        ab = true;
                        __hip_atomic_store(&ctl->abort, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(host_status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                }
                if (ab) rp_abort = 1;
            }
            __syncthreads();
            if (rp_abort) {   // frames [0, t) published: the recovery starts this tile at t
                if (tid == 0) __hip_atomic_store(&ctl->prog[wg], (unsigned)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return;
            }
        }
        tile.template frame<HOIST>(hp, sbytes, rs_t, Pv, rp_part);
        // publish frame t: every wave's stores drained, then one add to the
        // counter
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(&ctl->ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the workgroup's progress is written once, when it leaves (T here, the
    // frame it stopped at on an abort, 0 from the memset if it never ran): a
    // store per frame, which the next frame's first wait drains, cost C5's
    // recurrence ~0.5 us per frame
    if (tid == 0) __hip_atomic_store(&ctl->prog[wg], (unsigned)T, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// After every one-launch recurrence, on its stream: nothing unless the launch
// was aborted; then ONE workgroup computes, frame by frame, every tile's
// frames from its prog[] on, with the persistent kernel's per-tile code (the
// W_hh slice reloaded per tile), so the bits are those of a complete launch.
template <int RB, int NT, int KCH>
__global__ __launch_bounds__(64 * RSM_WAVES) void rnn_recur_recover_kernel(const float* h0,
                                                                          const float* __restrict__ Whh,
                                                                          const float* __restrict__ b_ih,
                                                                          const float* __restrict__ b_hh,
                                                                          float* hid, int T, int B, int H,
                                                                          int gx, int gy, PersistCtl* ctl) {
    extern __shared__ __attribute__((aligned(16))) f32x4 rp_part[];
    if (!__hip_atomic_load(&ctl->abort, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) return;
    using Tile = RpTile<RB, NT, KCH>;
    constexpr int EPT = Tile::EPT;
    const int nwg = gx * gy;
    const long slab = (long)B * H;
    const int sbytes = (int)(slab * 4);
    unsigned tmin = (unsigned)T;
    for (int q = 0; q < nwg; q++) tmin = min(tmin, __hip_atomic_load(&ctl->prog[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    for (int t = (int)tmin; t < T; t++) {
        float* ht = hid + (long)t * slab;
        const float* hp = t > 0 ? hid + (long)(t - 1) * slab : h0;
        const auto rs_t = __builtin_amdgcn_make_buffer_rsrc(ht, (short)0, sbytes, 0x00020000);
        for (int q = 0; q < nwg; q++) {
            if (__hip_atomic_load(&ctl->prog[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > (unsigned)t) continue;
            Tile tile;
            tile.setup(Whh, b_ih, b_hh, q % gx, q / gx, B, H);
            float Pv[EPT];
            tile.load_p(rs_t, Pv);
            tile.template frame<false>(hp, sbytes, rs_t, Pv, rp_part);
            __syncthreads();   // rp_part is the next tile's
        }
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();   // frame t stored before any load of it
    }
}

// Per-launch control blocks: a launch owns one from its memset until an event
// recorded after its recovery kernel completes; only then is it handed out
// again (several pipelines, streams or threads may have launches in flight).
// The status word sits in pinned, device-mapped host memory, so reading it
// takes no HIP call.
namespace {
struct PersistSlot {
    PersistCtl* ctl = nullptr;
    int* status_h = nullptr;   // host view
    int* status_d = nullptr;   // device view
    hipEvent_t done = nullptr;
    bool used = false;
    int nwg = 0;               // workgroups of its launch
    bool plain = false;        // a launch without a pipeline CU hint
    hipStream_t stream = nullptr;
};
struct PersistPool {
    std::mutex mu;
    std::vector<PersistSlot> slots[64];
    long long launches = 0, recoveries = 0;
};
PersistPool& persist_pool() {
    static PersistPool* p = new PersistPool();   // never destroyed: slots outlive static destructors
    return *p;
}
// a completed slot: count its recovery, clear it (mu held)
bool persist_reap(PersistPool& pp, PersistSlot& s) {
    if (!s.used) return true;
    if (hipEventQuery(s.done) != hipSuccess) return false;
    if (__atomic_load_n(s.status_h, __ATOMIC_ACQUIRE)) {
        pp.recoveries++;
        __atomic_store_n(s.status_h, 0, __ATOMIC_RELEASE);
    }
    s.used = false;
    return true;
}
}  // namespace

template <int RB, int NT, int KCH>
static int launch_persist(const float* h0, const float* Whh, const float* b_ih, const float* b_hh, float* hid,
                          int T, int B, int H, PersistSlot& slot, int fault_frame, hipStream_t s) {
    // every load of h_{t-1} in flight at once from H = 1024 (KCH = 8) on:
    // alone (tools/step_time.py, run r6m4) 32 x 1024 5.12 -> 4.71 us per
    // frame, 64 x 1024 6.07 -> 5.44; at H = 512 (KCH = 4) slower, 3.36 -> 3.63
    constexpr bool HOIST = KCH >= 8;
    static AsrAttrOnce attr, attr_r;
    if (int r_ = attr.set((const void*)rnn_recur_persist_kernel<RB, NT, KCH, HOIST>, RP_LDS)) return r_;
    if (int r_ = attr_r.set((const void*)rnn_recur_recover_kernel<RB, NT, KCH>, RP_LDS)) return r_;
    static std::once_flag occ_once;
    static int occ = 0;
    std::call_once(occ_once, [] {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, rnn_recur_persist_kernel<RB, NT, KCH, HOIST>,
                                                         64 * RSM_WAVES, RP_LDS) != hipSuccess)
            occ = 0;
    });
    if (occ < 1) return ASR_ERR_UNSUPPORTED;   // one workgroup must fit a CU
    const int gx = H / (16 * NT), gy = (B + 16 * RB - 1) / (16 * RB);
    ASR_HIP_TRY(hipMemsetAsync(slot.ctl, 0, offsetof(PersistCtl, prog) + sizeof(unsigned) * gx * gy, s));
    hipLaunchKernelGGL((rnn_recur_persist_kernel<RB, NT, KCH, HOIST>), dim3((unsigned)gx, (unsigned)gy),
                       dim3(64 * RSM_WAVES), RP_LDS, s, h0, Whh, b_ih, b_hh, hid, T, B, H, slot.ctl, slot.status_d,
                       fault_frame);
    ASR_LAUNCH_TRY();
    hipLaunchKernelGGL((rnn_recur_recover_kernel<RB, NT, KCH>), dim3(1), dim3(64 * RSM_WAVES), RP_LDS, s, h0, Whh,
                       b_ih, b_hh, hid, T, B, H, gx, gy, slot.ctl);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

int rnn_recur_persist_launch(const float* h0, const float* Whh, const float* b_ih, const float* b_hh, float* hid,
                             int T, int B, int H, int cus, hipStream_t s) {
    // cus: the CUs this launch may count on (its share of the stream's CU mask); <= 0: none given
    // tiles: 16 x 32 (NT = 2); 256 rows at most; H / 128 chunks of 16 k per wave
    const char* e = getenv("ASR_RNN_PERSIST");
    if (e && e[0] == '0') return ASR_ERR_UNSUPPORTED;
    if (T < 2 || B <= 0 || B > 256 || (H % 128) != 0 || H < 384 || H > 1024 || ((uintptr_t)hid % 16) != 0 ||
        (h0 && ((uintptr_t)h0 % 16) != 0) || (long)B * H * 4 >= 0x7fffffffL)
        return ASR_ERR_UNSUPPORTED;
    // a captured graph would replay one control block for ever: per-frame steps there
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return ASR_ERR_UNSUPPORTED;
    const int nwg = (H / 32) * ((B + 15) / 16);
    int dev = 0;
    ASR_HIP_TRY(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return ASR_ERR_UNSUPPORTED;
    const bool plain = cus <= 0;
    PersistPool& pp = persist_pool();
    std::lock_guard<std::mutex> lock(pp.mu);
    auto& slots = pp.slots[dev];
    PersistSlot* slot = nullptr;
    // workgroups of plain launches still in flight on this device's OTHER
    // streams (a launch queued behind another on its own stream never shares
    // the CUs with it: counting those sent back-to-back calls on one stream
    // to the per-frame steps)
    int reserved = 0;
    for (auto& q : slots) {
        if (persist_reap(pp, q)) {
            if (!slot) slot = &q;
        } else if (q.plain && q.stream != s) {
            reserved += q.nwg;
        }
    }
    if (plain) {   // no hint: half of the CUs the stream's mask allows (room beside it), less other plain launches'
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return ASR_ERR_UNSUPPORTED;
        int avail = ncu;
        if (s) {   // a caller's CU-masked stream
            uint32_t m[32] = {};
            const int words = std::min(32, (ncu + 31) / 32);
            if (hipExtStreamGetCUMask(s, (uint32_t)words, m) == hipSuccess) {
                int n = 0;
                for (int i = 0; i < words; i++) n += __builtin_popcount(m[i]);
                if (n > 0) avail = std::min(avail, n);
            }
        }
        cus = avail / 2 - reserved;
    }
    if (nwg > cus) return ASR_ERR_UNSUPPORTED;   // every workgroup resident at once
    if (!slot) {
        PersistSlot n;
        ASR_HIP_TRY(hipMalloc(&n.ctl, sizeof(PersistCtl)));
        void* h = nullptr;
        ASR_HIP_TRY(hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(h, 0, 64);
        n.status_h = static_cast<int*>(h);
        void* d = nullptr;
        ASR_HIP_TRY(hipHostGetDevicePointer(&d, h, 0));
        n.status_d = static_cast<int*>(d);
        ASR_HIP_TRY(hipEventCreateWithFlags(&n.done, hipEventDisableTiming));
        slots.push_back(n);
        slot = &slots.back();
    }
    // test hook: ASR_RNN_PERSIST_FAULT=<frame> stalls one workgroup before that frame
    const char* fe = getenv("ASR_RNN_PERSIST_FAULT");
    const int fault_frame = fe ? atoi(fe) : -1;
    int rc;
    switch (H / 128) {
        case 3: rc = launch_persist<1, 2, 3>(h0, Whh, b_ih, b_hh, hid, T, B, H, *slot, fault_frame, s); break;
        case 4: rc = launch_persist<1, 2, 4>(h0, Whh, b_ih, b_hh, hid, T, B, H, *slot, fault_frame, s); break;
        case 5: rc = launch_persist<1, 2, 5>(h0, Whh, b_ih, b_hh, hid, T, B, H, *slot, fault_frame, s); break;
        case 6: rc = launch_persist<1, 2, 6>(h0, Whh, b_ih, b_hh, hid, T, B, H, *slot, fault_frame, s); break;
        case 7: rc = launch_persist<1, 2, 7>(h0, Whh, b_ih, b_hh, hid, T, B, H, *slot, fault_frame, s); break;
        default: rc = launch_persist<1, 2, 8>(h0, Whh, b_ih, b_hh, hid, T, B, H, *slot, fault_frame, s); break;
    }
    if (rc) return rc;
    ASR_HIP_TRY(hipEventRecord(slot->done, s));
    slot->used = true;
    slot->nwg = nwg;
    slot->plain = plain;
    slot->stream = s;
    pp.launches++;
    return ASR_OK;
}

int rnn_persist_stats(long long* launches, long long* recoveries) {
    PersistPool& pp = persist_pool();
    std::lock_guard<std::mutex> lock(pp.mu);
    for (auto& v : pp.slots)
        for (auto& q : v) persist_reap(pp, q);
    if (launches) *launches = pp.launches;
    if (recoveries) *recoveries = pp.recoveries;
    return ASR_OK;
}

// ---------------------------------------------------------------------------
// In-place log_softmax of each row of C[M][ldc] (first N columns): one wave
// per row, max and sum of exp by shuffle reductions.
__global__ __launch_bounds__(256) void row_logsoftmax_kernel(float* __restrict__ C, long ldc, int M,
                                                             int N) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= M) return;
    float* r = C + (long)row * ldc;
    float mx = -INFINITY;
    for (int c = lane; c < N; c += 64) mx = fmaxf(mx, r[c]);
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float sum = 0.f;
    for (int c = lane; c < N; c += 64) sum += expf(r[c] - mx);
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    const float lz = mx + logf(sum);
    for (int c = lane; c < N; c += 64) r[c] -= lz;
}

int row_logsoftmax_launch(float* C, long ldc, int M, int N, hipStream_t s) {
    if (M <= 0) return ASR_OK;
    hipLaunchKernelGGL(row_logsoftmax_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, s, C, ldc,
                       M, N);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

// ---------------------------------------------------------------------------
// z = x + lam*y (cublasSgeam with alpha = 1, beta = lam: cuMatrix.cpp:150).
template <bool VEC4>
__global__ __launch_bounds__(256) void axpy_kernel(const float* __restrict__ x,
                                                   const float* __restrict__ y,
                                                   float* __restrict__ z, long n, float lam) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (VEC4) {
        if (i < (n >> 2)) {
            const float4 a = reinterpret_cast<const float4*>(x)[i];
            const float4 c = reinterpret_cast<const float4*>(y)[i];
            reinterpret_cast<float4*>(z)[i] =
                make_float4(a.x + lam * c.x, a.y + lam * c.y, a.z + lam * c.z, a.w + lam * c.w);
        }
    } else if (i < n) {
        z[i] = x[i] + lam * y[i];
    }
}

// h_0 = tanh(P_0 + (b_hh + b_ih)) when h_{-1} = 0 (RNN_Cell.cu:10-12 with hh = 0).
__global__ __launch_bounds__(256) void bias_tanh_kernel(float* __restrict__ p,
                                                        const float* __restrict__ b_ih,
                                                        const float* __restrict__ b_hh, long n,
                                                        int H) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        const int j = (int)(i % H);
        p[i] = tanhf(p[i] + (b_hh[j] + b_ih[j]));
    }
}

int bias_tanh_launch(float* p, const float* b_ih, const float* b_hh, long n, int H, hipStream_t s) {
    if (n <= 0) return ASR_OK;
    hipLaunchKernelGGL(bias_tanh_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, b_ih,
                       b_hh, n, H);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

int axpy_launch(const float* x, const float* y, float* z, long n, float lam, hipStream_t s) {
    if (n <= 0) return ASR_OK;
    const bool vec = (n % 4) == 0 && (((uintptr_t)x | (uintptr_t)y | (uintptr_t)z) % 16) == 0;
    const long work = vec ? n / 4 : n;
    const dim3 grid((unsigned)((work + 255) / 256));
    if (vec) hipLaunchKernelGGL(axpy_kernel<true>, grid, dim3(256), 0, s, x, y, z, n, lam);
    else hipLaunchKernelGGL(axpy_kernel<false>, grid, dim3(256), 0, s, x, y, z, n, lam);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

// ---------------------------------------------------------------------------
// Bidirectional RNN plumbing (nn.RNN(bidirectional=True), model.py:30).
// In-place time reversal of a time-major [T][n] buffer: swap rows t and T-1-t.
__global__ __launch_bounds__(256) void time_reverse_kernel(float4* __restrict__ p, int T, long n4) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;   // over (T/2) * n4
    if (i >= (long)(T / 2) * n4) return;
    const long t = i / n4, k = i - t * n4;
    float4* a = p + t * n4 + k;
    float4* b = p + (long)(T - 1 - t) * n4 + k;
    const float4 va = *a, vb = *b;
    *a = vb;
    *b = va;
}

// out[t][b][0:H] = hf[t][b][:], out[t][b][H:2H] = hr[T-1-t][b][:]  (H % 4 == 0, float4 units).
__global__ __launch_bounds__(256) void bidir_concat_kernel(const float4* __restrict__ hf,
                                                           const float4* __restrict__ hr,
                                                           float4* __restrict__ out, int T, int B,
                                                           int H4) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;   // over T * B * 2 * H4 outputs
    const long rowlen = 2L * H4;
    if (i >= (long)T * B * rowlen) return;
    const long row = i / rowlen;
    const int j = (int)(i - row * rowlen);
    const long t = row / B, b = row - t * B;
    out[i] = j < H4 ? hf[row * H4 + j] : hr[((long)(T - 1 - t) * B + b) * H4 + (j - H4)];
}

int time_reverse_launch(float* p, int T, long n, hipStream_t s) {
    if (T < 2 || n <= 0) return ASR_OK;
    if ((n & 3) || ((uintptr_t)p & 15)) return ASR_ERR_UNSUPPORTED;
    const long work = (long)(T / 2) * (n / 4);
    hipLaunchKernelGGL(time_reverse_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<float4*>(p), T, n / 4);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

int bidir_concat_launch(const float* hf, const float* hr, float* out, int T, int B, int H,
                        hipStream_t s) {
    if ((H & 3) || (((uintptr_t)hf | (uintptr_t)hr | (uintptr_t)out) & 15)) return ASR_ERR_UNSUPPORTED;
    const long work = (long)T * B * 2 * (H / 4);
    hipLaunchKernelGGL(bidir_concat_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const float4*>(hf), reinterpret_cast<const float4*>(hr),
                       reinterpret_cast<float4*>(out), T, B, H / 4);
    ASR_LAUNCH_TRY();
    return ASR_OK;
}

}  // namespace asr
