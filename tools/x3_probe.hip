// Probe: fp32-accurate GEMM and RNN recurrence on bf16 MFMA by a three-way
// split (x = h + m + l, each bf16, |x - (h + m + l)| <= 2^-27 |x|; six of the
// nine piece products, the dropped ones <= 2^-26 relative).  Measures time and
// the max error against a host fp64 computation on sampled rows, next to a
// plain fp32 GPU computation of the same sums.
//   hipcc --offload-arch=gfx950 -O3 -o tools/x3_probe tools/x3_probe.hip
//   tools/x3_probe [gemm|recur|all] [M] [T] [B]
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

#ifndef X3_CTMAJOR
#define X3_CTMAJOR 0
#endif
#ifndef X3_NOEPI
#define X3_NOEPI 0
#endif
#ifndef X3_NOMFMA
#define X3_NOMFMA 0
#endif
#ifndef X3_NOLOAD
#define X3_NOLOAD 0
#endif
#ifndef X3_SGB
#define X3_SGB 0
#endif
#ifndef X3_CHAIN
#define X3_CHAIN 0
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

__device__ __forceinline__ f32x4 mma6(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh,
                                      const bf16x8& bm, const bf16x8& bl, f32x4 acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
    return acc;
}

// ---------------------------------------------------------------- GEMM
// C[M][N] = A[M][K] . B[K][N] + bias, K <= 256, N <= 256, K % 4 == 0.
// 4 waves (one per SIMD: 512 registers per lane); wave w owns columns
// 64w .. 64w + 63 with their B pieces in registers (384) for the whole
// launch; 32-row tiles of A split into pieces once while staged to LDS
// (double-buffered), persistent over tiles.
constexpr int XK = 256;
constexpr int XAS = XK + 8;       // LDS row stride (bf16): 16-B row shift
constexpr int XR = 16;            // rows per tile
constexpr int XPIECE = XR * XAS;  // one piece of one buffer

constexpr int XCT = 4;   // 16-column tiles per wave
template <int NCH>
__global__ __launch_bounds__(256) void gemm_x3_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                      const float* __restrict__ bias, float* __restrict__ C,
                                                      int M, int N, int K) {
    extern __shared__ __attribute__((aligned(16))) __bf16 xs[];   // [2][3][XR][XAS]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c15 = lane & 15, g = lane >> 4;
    constexpr int nch = NCH;   // 32-k chunks (K <= 32 NCH; pieces past K are zero)
    const int KC = nch * 32;
    bf16x8 bh[XCT][8], bm[XCT][8], bl[XCT][8];
#pragma unroll
    for (int ct = 0; ct < XCT; ct++) {
        const int n = 64 * w + 16 * ct + c15;
#pragma unroll
        for (int c = 0; c < 8; c++) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int k = 32 * c + 8 * g + j;
                const float b = (k < K && n < N) ? B[(long)k * N + n] : 0.f;
                __bf16 h, m, l;
                split3(b, h, m, l);
                bh[ct][c][j] = h;
                bm[ct][c][j] = m;
                bl[ct][c][j] = l;
            }
        }
    }
    const int ntile = (M + XR - 1) / XR;
    constexpr int NST = XR * 64 / 256;   // float4 per thread per tile
    float4 st[NST];
    auto load = [&](int tl) {
#pragma unroll
        for (int i = 0; i < NST; i++) {
            const int idx = tid + 256 * i, row = idx >> 6, k = (idx & 63) * 4;
            const int gr = tl * XR + row;
            st[i] = (tl < ntile && gr < M && k < K) ? *reinterpret_cast<const float4*>(A + (long)gr * K + k)
                                                   : float4{0.f, 0.f, 0.f, 0.f};
        }
    };
    auto stage = [&](int buf) {
#pragma unroll
        for (int i = 0; i < NST; i++) {
            const int idx = tid + 256 * i, row = idx >> 6, k = (idx & 63) * 4;
            if (k >= KC) continue;
            bf16x4 h, m, l;
            const float v[4] = {st[i].x, st[i].y, st[i].z, st[i].w};
#pragma unroll
            for (int e = 0; e < 4; e++) {
                __bf16 a, b, c;
                split3(v[e], a, b, c);
                h[e] = a;
                m[e] = b;
                l[e] = c;
            }
            __bf16* p = xs + (buf * 3) * XPIECE + row * XAS + k;
            *reinterpret_cast<bf16x4*>(p) = h;
            *reinterpret_cast<bf16x4*>(p + XPIECE) = m;
            *reinterpret_cast<bf16x4*>(p + 2 * XPIECE) = l;
        }
    };
    int tile = blockIdx.x;
    load(tile);
    stage(0);
    load(tile + gridDim.x);
    __syncthreads();
    int cur = 0;
    for (; tile < ntile; tile += gridDim.x) {
        constexpr int XRT = XR / 16;
        f32x4 acc[XRT][XCT];
#pragma unroll
        for (int rt = 0; rt < XRT; rt++)
#pragma unroll
            for (int ct = 0; ct < XCT; ct++) acc[rt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
        const __bf16* pb = xs + (cur * 3) * XPIECE;
#pragma unroll
        for (int c = 0; c < 8; c++) {
            if (c < nch) {
#pragma unroll
                for (int rt = 0; rt < XRT; rt++) {
                    const int off = (16 * rt + c15) * XAS + 32 * c + 8 * g;
                    const bf16x8 ah = *reinterpret_cast<const bf16x8*>(pb + off);
                    const bf16x8 am = *reinterpret_cast<const bf16x8*>(pb + XPIECE + off);
                    const bf16x8 al = *reinterpret_cast<const bf16x8*>(pb + 2 * XPIECE + off);
#if X3_CHAIN
#pragma unroll
                    for (int ct = 0; ct < XCT; ct++)
                        acc[rt][ct] = mma6(ah, am, al, bh[ct][c], bm[ct][c], bl[ct][c], acc[rt][ct]);
#else
                    // product-major: consecutive MFMAs go to different accumulators
#define X3P(A_, B_)                                                                                   \
    _Pragma("unroll") for (int ct = 0; ct < XCT; ct++) acc[rt][ct] =                                  \
        __builtin_amdgcn_mfma_f32_16x16x32_bf16(A_, B_[ct][c], acc[rt][ct], 0, 0, 0);
                    X3P(al, bh) X3P(am, bm) X3P(ah, bl) X3P(am, bh) X3P(ah, bm) X3P(ah, bh)
#undef X3P
#endif
                }
            }
        }
        stage(cur ^ 1);
        load(tile + 2 * (int)gridDim.x);
#pragma unroll
        for (int rt = 0; rt < XRT; rt++)
#pragma unroll
            for (int ct = 0; ct < XCT; ct++) {
                const int n = 64 * w + 16 * ct + c15;
                if (n >= N) continue;
                const float bb = bias ? bias[n] : 0.f;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int row = tile * XR + 16 * rt + 4 * g + j;
                    if (row < M) C[(long)row * N + n] = acc[rt][ct][j] + bb;
                }
            }
        __syncthreads();
        cur ^= 1;
    }
}

__global__ void gemm_f32_kernel(const float* A, const float* B, const float* bias, float* C, int M, int N, int K) {
    const long row = blockIdx.x;
    const int n = threadIdx.x;
    if (row >= M || n >= N) return;
    float s = 0.f;
    for (int k = 0; k < K; k++) s = fmaf(A[row * K + k], B[(long)k * N + n], s);
    C[row * N + n] = s + (bias ? bias[n] : 0.f);
}

// ---------------------------------------------------------------- recurrence
// h_t = tanh((P_t + h_{t-1}.W) + b), 16 utterances per workgroup, H = 256,
// 4 waves, wave w owns columns 64w .. 64w + 63 (W pieces in registers);
// h_{t-1} pieces in LDS, double-buffered, one barrier per step.
constexpr int RH = 256;
constexpr int RAS = RH + 8;
constexpr int RPIECE = 16 * RAS;

__global__ __launch_bounds__(256) void recur_x3_kernel(const float* __restrict__ W, const float* __restrict__ bias,
                                                       float* hid, int T, int B) {
    __shared__ __attribute__((aligned(16))) __bf16 hs[2][3][RPIECE];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c15 = lane & 15, g = lane >> 4;
    const int r0 = blockIdx.x * 16;
    bf16x8 bh[XCT][8], bm[XCT][8], bl[XCT][8];
    int n[XCT];
    float bb[XCT];
#pragma unroll
    for (int ct = 0; ct < XCT; ct++) {
        n[ct] = 64 * w + 16 * ct + c15;
        bb[ct] = bias[n[ct]];
#pragma unroll
        for (int c = 0; c < 8; c++)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                __bf16 h, m, l;
                split3(W[(long)(32 * c + 8 * g + j) * RH + n[ct]], h, m, l);
                bh[ct][c][j] = h;
                bm[ct][c][j] = m;
                bl[ct][c][j] = l;
            }
    }
    for (int x = tid; x < 3 * RPIECE; x += 256) (&hs[0][0][0])[x] = (__bf16)0.f;
    const long ts = (long)B * RH;
    int roff[4];
    bool ok[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int r = r0 + 4 * g + j;
        ok[j] = r < B;
        roff[j] = (ok[j] ? r : 0) * RH;
    }
    float pn[XCT][4];
#pragma unroll
    for (int ct = 0; ct < XCT; ct++)
#pragma unroll
        for (int j = 0; j < 4; j++) pn[ct][j] = ok[j] ? hid[roff[j] + n[ct]] : 0.f;
    __syncthreads();
    int cur = 0;
    for (int t = 0; t < T; t++) {
        float p[XCT][4];
#pragma unroll
        for (int ct = 0; ct < XCT; ct++)
#pragma unroll
            for (int j = 0; j < 4; j++) p[ct][j] = pn[ct][j];
        if (t + 1 < T) {
#pragma unroll
            for (int ct = 0; ct < XCT; ct++)
#pragma unroll
                for (int j = 0; j < 4; j++) pn[ct][j] = ok[j] ? hid[(t + 1) * ts + roff[j] + n[ct]] : 0.f;
        }
        f32x4 acc[XCT];
#pragma unroll
        for (int ct = 0; ct < XCT; ct++) acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
        const __bf16* pb = &hs[cur][0][0];
#pragma unroll
        for (int c = 0; c < 8; c++) {
            const int off = c15 * RAS + 32 * c + 8 * g;
            const bf16x8 ah = *reinterpret_cast<const bf16x8*>(pb + off);
            const bf16x8 am = *reinterpret_cast<const bf16x8*>(pb + RPIECE + off);
            const bf16x8 al = *reinterpret_cast<const bf16x8*>(pb + 2 * RPIECE + off);
#if X3_CHAIN
#pragma unroll
            for (int ct = 0; ct < XCT; ct++) acc[ct] = mma6(ah, am, al, bh[ct][c], bm[ct][c], bl[ct][c], acc[ct]);
#else
#define X3P(A_, B_)                                                                                   \
    _Pragma("unroll") for (int ct = 0; ct < XCT; ct++) acc[ct] =                                      \
        __builtin_amdgcn_mfma_f32_16x16x32_bf16(A_, B_[ct][c], acc[ct], 0, 0, 0);
            X3P(al, bh) X3P(am, bm) X3P(ah, bl) X3P(am, bh) X3P(ah, bm) X3P(ah, bh)
#undef X3P
#endif
        }
        __bf16* hn = &hs[cur ^ 1][0][0];
#pragma unroll
        for (int ct = 0; ct < XCT; ct++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float h = tanhf((p[ct][j] + acc[ct][j]) + bb[ct]);
                __bf16 a, b2, c2;
                split3(h, a, b2, c2);
                const int o = (4 * g + j) * RAS + n[ct];
                hn[o] = a;
                hn[RPIECE + o] = b2;
                hn[2 * RPIECE + o] = c2;
                if (ok[j]) hid[t * ts + roff[j] + n[ct]] = h;
            }
        cur ^= 1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    }
}

// ocml's tanhf without its branches (both halves computed, one selected):
// the same operations in the same order, so the same bits.
__device__ __forceinline__ float fbits(unsigned u) { return __builtin_bit_cast(float, u); }
__device__ __forceinline__ float tanh_nb(float x) {
    const float ax = fabsf(x);
    // |x| >= 0.625: 1 - 2 / (1 + e^{2|x|}); e^v = 2^(v log2 e) with the
    // product split into rndne part + (hi, lo) remainder
    const float v = ax + ax;
    const float t = v * fbits(0x3fb8aa3bu);
    const float r = __builtin_rintf(t);
    const float f = t - r;
    float e = __builtin_fmaf(v, fbits(0x3fb8aa3bu), -t);
    e = __builtin_fmaf(v, fbits(0x32a5705fu), e);
    float y = __builtin_amdgcn_exp2f(f + e);
    y = __builtin_ldexpf(y, (int)r);
    y = v > fbits(0x42b17218u) ? __builtin_inff() : y;
    const float big = __builtin_fmaf(__builtin_amdgcn_rcpf(1.0f + y), -2.0f, 1.0f);
    // |x| < 0.625: odd polynomial
    const float x2 = x * x;
    float q = __builtin_fmaf(fbits(0xbbbac73du), x2, fbits(0x3ca908c9u));
    q = __builtin_fmaf(x2, q, fbits(0xbd5c1c4eu));
    q = __builtin_fmaf(x2, q, fbits(0x3e088382u));
    q = __builtin_fmaf(x2, q, fbits(0xbeaaaa99u));
    const float small = __builtin_fmaf(x2, ax * q, ax);
    const float m = ax < 0.625f ? small : big;
    return __builtin_bit_cast(float, (__builtin_bit_cast(unsigned, m) & 0x7fffffffu) |
                                         (__builtin_bit_cast(unsigned, x) & 0x80000000u));
}

__global__ void tanh_check_kernel(const float* x, float* a, float* b, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        a[i] = tanhf(x[i]);
        b[i] = tanh_nb(x[i]);
    }
}

// v3: column tiles in two halves — the MFMAs of tiles 2, 3 are issued
// beside the epilogue of tiles 0, 1 (independent), branch-free epilogue
// (B % 16 == 0 assumed here)
__global__ __launch_bounds__(256) void recur_x3p_kernel(const float* __restrict__ W, const float* __restrict__ bias,
                                                        float* hid, int T, int B) {
    __shared__ __attribute__((aligned(16))) __bf16 hs[2][3][RPIECE];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c15 = lane & 15, g = lane >> 4;
    const int r0 = blockIdx.x * 16;
    bf16x8 bh[XCT][8], bm[XCT][8], bl[XCT][8];
    int n[XCT];
    float bb[XCT];
#pragma unroll
    for (int ct = 0; ct < XCT; ct++) {
        n[ct] = 64 * w + 16 * ct + c15;
        bb[ct] = bias[n[ct]];
#pragma unroll
        for (int c = 0; c < 8; c++)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                __bf16 h, m, l;
                split3(W[(long)(32 * c + 8 * g + j) * RH + n[ct]], h, m, l);
                bh[ct][c][j] = h;
                bm[ct][c][j] = m;
                bl[ct][c][j] = l;
            }
    }
    for (int x = tid; x < 3 * RPIECE; x += 256) (&hs[0][0][0])[x] = (__bf16)0.f;
    const long ts = (long)B * RH;
    const int rbase = (r0 + 4 * g) * RH;
    float pn[XCT][4];
#pragma unroll
    for (int ct = 0; ct < XCT; ct++)
#pragma unroll
        for (int j = 0; j < 4; j++) pn[ct][j] = hid[rbase + j * RH + n[ct]];
    __syncthreads();
    int cur = 0;
    for (int t = 0; t < T; t++) {
        float p[XCT][4];
#pragma unroll
        for (int ct = 0; ct < XCT; ct++)
#pragma unroll
            for (int j = 0; j < 4; j++) p[ct][j] = pn[ct][j];
        const long tn = (t + 1 < T ? t + 1 : t) * ts;
#pragma unroll
        for (int ct = 0; ct < XCT; ct++)
#pragma unroll
            for (int j = 0; j < 4; j++) pn[ct][j] = hid[tn + rbase + j * RH + n[ct]];
        f32x4 acc[XCT];
#pragma unroll
        for (int ct = 0; ct < XCT; ct++) acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
        const __bf16* pb = &hs[cur][0][0];
        __bf16* hn = &hs[cur ^ 1][0][0];
        float* hrow = hid + t * ts + rbase;
        auto epi = [&](int ct) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float h = tanh_nb((p[ct][j] + acc[ct][j]) + bb[ct]);
                __bf16 a, b2, c2;
                split3(h, a, b2, c2);
                const int o = (4 * g + j) * RAS + n[ct];
                hn[o] = a;
                hn[RPIECE + o] = b2;
                hn[2 * RPIECE + o] = c2;
                hrow[j * RH + n[ct]] = h;
            }
        };
#pragma unroll
        for (int half = 0; half < 2; half++) {
#pragma unroll
            for (int c = 0; c < 8; c++) {
                const int off = c15 * RAS + 32 * c + 8 * g;
                const bf16x8 ah = *reinterpret_cast<const bf16x8*>(pb + off);
                const bf16x8 am = *reinterpret_cast<const bf16x8*>(pb + RPIECE + off);
                const bf16x8 al = *reinterpret_cast<const bf16x8*>(pb + 2 * RPIECE + off);
#define X3Q(A_, B_)                                                                                   \
    _Pragma("unroll") for (int cc = 0; cc < 2; cc++) acc[2 * half + cc] =                             \
        __builtin_amdgcn_mfma_f32_16x16x32_bf16(A_, B_[2 * half + cc][c], acc[2 * half + cc], 0, 0, 0);
                X3Q(al, bh) X3Q(am, bm) X3Q(ah, bl) X3Q(am, bh) X3Q(ah, bm) X3Q(ah, bh)
#undef X3Q
            }
            if (half == 1) {
#if X3_SGB
                // tiles 0, 1's epilogue VALU between the tiles 2, 3 MFMAs
                for (int i = 0; i < 96; i++) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
                }
#endif
            }
            if (half == 0) {
                epi(0);
                epi(1);
            }
        }
        epi(2);
        epi(3);
        cur ^= 1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    }
}

// tanh to ~2 ulp without branches: the polynomial of ocml's tanhf below
// 0.625, 1 - 2 / (1 + 2^(2|x| log2 e)) above (the exponential's argument
// error, <= 2^-24 |arg|, is damped by 2 / (1 + y) there)
__device__ __forceinline__ float tanh_fast(float x) {
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
}

__global__ void tanh_fast_kernel(const float* x, float* a, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = tanh_fast(x[i]);
}

// v4: 8 waves (two per SIMD: the VALU of one issues beside the MFMAs of the
// other), wave w owns columns 32w .. 32w + 31 (W pieces: 192 registers);
// P loads / h stores as buffer ops (rows past B fall outside the resource:
// loads return 0, stores are dropped), branch-free epilogue.
constexpr int W4_CT = 2;
__global__ __launch_bounds__(512) void recur_x3w_kernel(const float* __restrict__ W, const float* __restrict__ bias,
                                                        float* hid, int T, int B) {
    __shared__ __attribute__((aligned(16))) __bf16 hs[2][3][RPIECE];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c15 = lane & 15, g = lane >> 4;
    const int r0 = blockIdx.x * 16;
    bf16x8 bh[W4_CT][8], bm[W4_CT][8], bl[W4_CT][8];
    int voff[W4_CT];
    float bb[W4_CT];
#pragma unroll
    for (int ct = 0; ct < W4_CT; ct++) {
        const int n = 32 * w + 16 * ct + c15;
        bb[ct] = bias[n];
        voff[ct] = ((r0 + 4 * g) * RH + n) * 4;
#pragma unroll
        for (int c = 0; c < 8; c++)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                __bf16 h, m, l;
                split3(W[(long)(32 * c + 8 * g + j) * RH + n], h, m, l);
                bh[ct][c][j] = h;
                bm[ct][c][j] = m;
                bl[ct][c][j] = l;
            }
    }
    for (int x = tid; x < 3 * RPIECE; x += 512) (&hs[0][0][0])[x] = (__bf16)0.f;
    const long ts = (long)B * RH;
    const int nrec = B * RH * 4;
    auto rsrc_at = [&](int t) { return __builtin_amdgcn_make_buffer_rsrc(hid + t * ts, (short)0, nrec, 0x00020000); };
    float pn[W4_CT][4];
    {
        const auto rs = rsrc_at(0);
#pragma unroll
        for (int ct = 0; ct < W4_CT; ct++)
#pragma unroll
            for (int j = 0; j < 4; j++)
                pn[ct][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff[ct] + j * RH * 4, 0, 0));
    }
    __syncthreads();
    int cur = 0;
    for (int t = 0; t < T; t++) {
        float p[W4_CT][4];
#pragma unroll
        for (int ct = 0; ct < W4_CT; ct++)
#pragma unroll
            for (int j = 0; j < 4; j++) p[ct][j] = pn[ct][j];
        const auto rs = rsrc_at(t);
        const auto rn = rsrc_at(t + 1 < T ? t + 1 : t);
#if X3_NOLOAD
#pragma unroll
        for (int ct = 0; ct < W4_CT; ct++)
#pragma unroll
            for (int j = 0; j < 4; j++) pn[ct][j] = p[ct][j] * 0.5f;
#else
#pragma unroll
        for (int ct = 0; ct < W4_CT; ct++)
#pragma unroll
            for (int j = 0; j < 4; j++)
                pn[ct][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rn, voff[ct] + j * RH * 4, 0, 0));
#endif
        f32x4 acc[W4_CT];
#pragma unroll
        for (int ct = 0; ct < W4_CT; ct++) acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
        const __bf16* pb = &hs[cur][0][0];
        __bf16* hn = &hs[cur ^ 1][0][0];
#if X3_CTMAJOR
#pragma unroll
        for (int ct = 0; ct < W4_CT; ct++) {
#pragma unroll
            for (int c = 0; c < 8; c++) {
                const int off = c15 * RAS + 32 * c + 8 * g;
                const bf16x8 ah = *reinterpret_cast<const bf16x8*>(pb + off);
                const bf16x8 am = *reinterpret_cast<const bf16x8*>(pb + RPIECE + off);
                const bf16x8 al = *reinterpret_cast<const bf16x8*>(pb + 2 * RPIECE + off);
                acc[ct] = mma6(ah, am, al, bh[ct][c], bm[ct][c], bl[ct][c], acc[ct]);
            }
        }
#else
#pragma unroll
        for (int c = 0; c < 8; c++) {
            const int off = c15 * RAS + 32 * c + 8 * g;
            const bf16x8 ah = *reinterpret_cast<const bf16x8*>(pb + off);
            const bf16x8 am = *reinterpret_cast<const bf16x8*>(pb + RPIECE + off);
            const bf16x8 al = *reinterpret_cast<const bf16x8*>(pb + 2 * RPIECE + off);
#if X3_NOMFMA
#pragma unroll
            for (int ct = 0; ct < W4_CT; ct++) acc[ct][0] += (float)ah[0] + (float)am[1] + (float)al[2];
#else
#define X3Q(A_, B_)                                                                                   \
    _Pragma("unroll") for (int ct = 0; ct < W4_CT; ct++) acc[ct] =                                    \
        __builtin_amdgcn_mfma_f32_16x16x32_bf16(A_, B_[ct][c], acc[ct], 0, 0, 0);
            X3Q(al, bh) X3Q(am, bm) X3Q(ah, bl) X3Q(am, bh) X3Q(ah, bm) X3Q(ah, bh)
#undef X3Q
#endif
        }
#endif
#pragma unroll
        for (int ct = 0; ct < W4_CT; ct++) {
            const int n = 32 * w + 16 * ct + c15;
#pragma unroll
            for (int j = 0; j < 4; j++) {
#if X3_NOEPI
                const float h = (p[ct][j] + acc[ct][j]) * 0.001f;
#else
                const float h = tanh_fast((p[ct][j] + acc[ct][j]) + bb[ct]);
#endif
                __bf16 a, b2, c2;
                split3(h, a, b2, c2);
                const int o = (4 * g + j) * RAS + n;
                hn[o] = a;
                hn[RPIECE + o] = b2;
                hn[2 * RPIECE + o] = c2;
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, h), rs, voff[ct] + j * RH * 4, 0, 0);
            }
        }
        cur ^= 1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    }
}

// plain fp32: one workgroup per utterance, thread n, sequential k
__global__ __launch_bounds__(256) void recur_f32_kernel(const float* W, const float* bias, float* hid, int T, int B,
                                                        int nutt) {
    __shared__ float h[RH];
    const int b = blockIdx.x, n = threadIdx.x;
    if (b >= nutt) return;
    h[n] = 0.f;
    __syncthreads();
    const long ts = (long)B * RH;
    for (int t = 0; t < T; t++) {
        float s = 0.f;
        for (int k = 0; k < RH; k++) s = fmaf(h[k], W[k * RH + n], s);
        const float v = tanhf((hid[t * ts + (long)b * RH + n] + s) + bias[n]);
        __syncthreads();
        h[n] = v;
        hid[t * ts + (long)b * RH + n] = v;
        __syncthreads();
    }
}

static uint64_t rng = 88172645463325252ull;
static float urand() {   // uniform [-1, 1)
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (float)((rng >> 11) * (1.0 / 9007199254740992.0)) * 2.f - 1.f;
}

static void probe_gemm(long M) {
    const int K = 256, N = 256;
    std::vector<float> hA(M * K), hB(K * N), hb(N);
    for (auto& x : hA) x = urand();
    for (auto& x : hB) x = urand() * 0.0625f;
    for (auto& x : hb) x = urand() * 0.1f;
    float *dA, *dB, *db, *dC, *dR;
    CK(hipMalloc(&dA, M * K * 4));
    CK(hipMalloc(&dB, K * N * 4));
    CK(hipMalloc(&db, N * 4));
    CK(hipMalloc(&dC, M * N * 4));
    CK(hipMalloc(&dR, 4096L * N * 4));
    CK(hipMemcpy(dA, hA.data(), M * K * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, hB.data(), K * N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), N * 4, hipMemcpyHostToDevice));
    const size_t lds = 2 * 3 * XPIECE * 2;
    CK(hipFuncSetAttribute((const void*)gemm_x3_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    int ncu = 256;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int ntile = (int)((M + XR - 1) / XR);
    for (int grid : {ncu, 2 * ncu}) {
        const int gr = grid < ntile ? grid : ntile;
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        hipLaunchKernelGGL(gemm_x3_kernel<8>, dim3(gr), dim3(256), lds, 0, dA, dB, db, dC, (int)M, N, K);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        const int reps = 10;
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; i++)
            hipLaunchKernelGGL(gemm_x3_kernel<8>, dim3(gr), dim3(256), lds, 0, dA, dB, db, dC, (int)M, N, K);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        const double fl = 2.0 * M * N * K;
        printf("{\"probe\": \"gemm_x3\", \"M\": %ld, \"K\": %d, \"N\": %d, \"grid\": %d, \"ms\": %.4f, "
               "\"fp32_equiv_tflops\": %.1f, \"bf16_mfma_tflops\": %.1f}\n",
               M, K, N, gr, ms, fl / ms / 1e9, 6 * fl / ms / 1e9);
    }
    // accuracy on 4096 sampled rows (the first 4096) against fp64
    const int S = 4096 < M ? 4096 : (int)M;
    hipLaunchKernelGGL(gemm_f32_kernel, dim3(S), dim3(256), 0, 0, dA, dB, db, dR, S, N, K);
    CK(hipDeviceSynchronize());
    std::vector<float> hC((size_t)S * N), hR((size_t)S * N);
    CK(hipMemcpy(hC.data(), dC, (size_t)S * N * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hR.data(), dR, (size_t)S * N * 4, hipMemcpyDeviceToHost));
    double ex = 0, ef = 0, sx = 0, sf = 0;
    for (int r = 0; r < S; r++)
        for (int n = 0; n < N; n++) {
            double s = 0, sa = 0;
            for (int k = 0; k < K; k++) {
                s += (double)hA[(long)r * K + k] * hB[k * N + n];
                sa += fabs((double)hA[(long)r * K + k] * hB[k * N + n]);
            }
            s += hb[n];
            sa += fabs(hb[n]);
            const double dx = fabs(hC[(size_t)r * N + n] - s) / sa, df = fabs(hR[(size_t)r * N + n] - s) / sa;
            ex = dx > ex ? dx : ex;
            ef = df > ef ? df : ef;
            sx += dx;
            sf += df;
        }
    printf("{\"probe\": \"gemm_x3_error\", \"rows\": %d, \"max_err_over_abs_sum_x3\": %.3e, \"fp32\": %.3e, "
           "\"mean_x3\": %.3e, \"mean_fp32\": %.3e}\n",
           S, ex, ef, sx / ((double)S * N), sf / ((double)S * N));
    CK(hipFree(dA));
    CK(hipFree(dB));
    CK(hipFree(db));
    CK(hipFree(dC));
    CK(hipFree(dR));
}

static void probe_recur(int T, int B) {
    const long n = (long)T * B * RH;
    std::vector<float> hP(n), hW(RH * RH), hb(RH);
    for (auto& x : hP) x = urand() * 0.5f;
    for (auto& x : hW) x = urand() * 0.0625f;
    for (auto& x : hb) x = urand() * 0.1f;
    float *dP, *dH, *dW, *db, *dR;
    CK(hipMalloc(&dP, n * 4));
    CK(hipMalloc(&dH, n * 4));
    CK(hipMalloc(&dR, n * 4));
    CK(hipMalloc(&dW, RH * RH * 4));
    CK(hipMalloc(&db, RH * 4));
    CK(hipMemcpy(dP, hP.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dW, hW.data(), RH * RH * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), RH * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grid = (B + 15) / 16;
    CK(hipMemcpy(dH, dP, n * 4, hipMemcpyDeviceToDevice));
    hipLaunchKernelGGL(recur_x3_kernel, dim3(grid), dim3(256), 0, 0, dW, db, dH, T, B);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        CK(hipMemcpy(dH, dP, n * 4, hipMemcpyDeviceToDevice));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(recur_x3_kernel, dim3(grid), dim3(256), 0, 0, dW, db, dH, T, B);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    printf("{\"probe\": \"recur_x3\", \"T\": %d, \"B\": %d, \"H\": %d, \"workgroups\": %d, \"ms\": %.4f, "
           "\"us_per_step\": %.3f}\n",
           T, B, RH, grid, best, 1000.0 * best / T);
    {
        float bp = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            CK(hipMemcpy(dR, dP, n * 4, hipMemcpyDeviceToDevice));
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(recur_x3p_kernel, dim3(grid), dim3(256), 0, 0, dW, db, dR, T, B);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            bp = ms < bp ? ms : bp;
        }
        std::vector<float> a(n), b(n);
        CK(hipMemcpy(a.data(), dH, n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), dR, n * 4, hipMemcpyDeviceToHost));
        long diff = 0;
        for (long i = 0; i < n; i++) diff += a[i] != b[i];
        printf("{\"probe\": \"recur_x3p\", \"ms\": %.4f, \"us_per_step\": %.3f, \"values_differing_from_v2\": %ld}\n",
               bp, 1000.0 * bp / T, diff);
        float bw = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            CK(hipMemcpy(dR, dP, n * 4, hipMemcpyDeviceToDevice));
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(recur_x3w_kernel, dim3(grid), dim3(512), 0, 0, dW, db, dR, T, B);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            bw = ms < bw ? ms : bw;
        }
        {   // error of v4 against fp64 on 8 utterances, first 200 steps
            std::vector<float> c(n);
            CK(hipMemcpy(c.data(), dR, n * 4, hipMemcpyDeviceToHost));
            double ew = 0;
            for (int b = 0; b < 8; b++) {
                std::vector<double> h(RH, 0.0), hn2(RH);
                for (int t = 0; t < 200 && t < T; t++) {
                    for (int j = 0; j < RH; j++) {
                        double sacc = 0;
                        for (int k = 0; k < RH; k++) sacc += h[k] * hW[k * RH + j];
                        hn2[j] = tanh(((double)hP[(long)t * B * RH + (long)b * RH + j] + sacc) + hb[j]);
                    }
                    h = hn2;
                    for (int j = 0; j < RH; j++) {
                        const double d = fabs(c[(long)t * B * RH + (long)b * RH + j] - h[j]);
                        ew = d > ew ? d : ew;
                    }
                }
            }
            printf("{\"probe\": \"recur_x3w\", \"ms\": %.4f, \"us_per_step\": %.3f, \"max_abs_err_first_200\": %.3e}\n",
                   bw, 1000.0 * bw / T, ew);
        }
        {   // tanh_fast against fp64 tanh, in ulps of the float result
            const int nt = 1 << 22;
            std::vector<float> hx(nt);
            for (int i = 0; i < nt; i++) hx[i] = (float)((i - nt / 2) * (24.0 / nt));
            float *dx, *da;
            CK(hipMalloc(&dx, nt * 4));
            CK(hipMalloc(&da, nt * 4));
            CK(hipMemcpy(dx, hx.data(), nt * 4, hipMemcpyHostToDevice));
            hipLaunchKernelGGL(tanh_fast_kernel, dim3(nt / 256), dim3(256), 0, 0, dx, da, nt);
            CK(hipDeviceSynchronize());
            std::vector<float> ha(nt);
            CK(hipMemcpy(ha.data(), da, nt * 4, hipMemcpyDeviceToHost));
            double mu = 0;
            for (int i = 0; i < nt; i++) {
                const double r = tanh((double)hx[i]);
                const float rf = (float)r;
                const double ulp = fabs((double)nextafterf(rf, 2.f) - rf);
                const double u = fabs(ha[i] - r) / (ulp > 0 ? ulp : 1e-45);
                mu = u > mu ? u : mu;
            }
            printf("{\"probe\": \"tanh_fast\", \"points\": %d, \"max_ulp\": %.2f}\n", nt, mu);
            CK(hipFree(dx));
            CK(hipFree(da));
        }
        // branch-free tanh against tanhf on a sweep
        const int nt = 1 << 22;
        std::vector<float> hx(nt);
        for (int i = 0; i < nt; i++) hx[i] = (float)((i - nt / 2) * (24.0 / nt));
        float *dx, *da, *db2;
        CK(hipMalloc(&dx, nt * 4));
        CK(hipMalloc(&da, nt * 4));
        CK(hipMalloc(&db2, nt * 4));
        CK(hipMemcpy(dx, hx.data(), nt * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(tanh_check_kernel, dim3(nt / 256), dim3(256), 0, 0, dx, da, db2, nt);
        CK(hipDeviceSynchronize());
        std::vector<float> ha(nt), hb2(nt);
        CK(hipMemcpy(ha.data(), da, nt * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hb2.data(), db2, nt * 4, hipMemcpyDeviceToHost));
        long td = 0;
        for (int i = 0; i < nt; i++) td += memcmp(&ha[i], &hb2[i], 4) != 0;
        printf("{\"probe\": \"tanh_nb\", \"points\": %d, \"differing_from_tanhf\": %ld}\n", nt, td);
        CK(hipFree(dx));
        CK(hipFree(da));
        CK(hipFree(db2));
    }
    const int S = 8;
    CK(hipMemcpy(dR, dP, n * 4, hipMemcpyDeviceToDevice));
    hipLaunchKernelGGL(recur_f32_kernel, dim3(S), dim3(256), 0, 0, dW, db, dR, T, B, S);
    CK(hipDeviceSynchronize());
    std::vector<float> hX(n), hF(n);
    CK(hipMemcpy(hX.data(), dH, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hF.data(), dR, n * 4, hipMemcpyDeviceToHost));
    double ex = 0, ef = 0;
    int tmax = T < 200 ? T : 200;   // before chaos grows rounding differences
    double ex_all = 0, ef_all = 0;
    for (int b = 0; b < S; b++) {
        std::vector<double> h(RH, 0.0), hn(RH);
        for (int t = 0; t < T; t++) {
            for (int j = 0; j < RH; j++) {
                double s = 0;
                for (int k = 0; k < RH; k++) s += h[k] * hW[k * RH + j];
                hn[j] = tanh(((double)hP[(long)t * B * RH + (long)b * RH + j] + s) + hb[j]);
            }
            h = hn;
            for (int j = 0; j < RH; j++) {
                const long o = (long)t * B * RH + (long)b * RH + j;
                const double dx = fabs(hX[o] - h[j]), df = fabs(hF[o] - h[j]);
                if (t < tmax) {
                    ex = dx > ex ? dx : ex;
                    ef = df > ef ? df : ef;
                }
                ex_all = dx > ex_all ? dx : ex_all;
                ef_all = df > ef_all ? df : ef_all;
            }
        }
    }
    printf("{\"probe\": \"recur_x3_error\", \"utterances\": %d, \"max_abs_err_first_%d_x3\": %.3e, \"fp32\": %.3e, "
           "\"max_abs_err_all_x3\": %.3e, \"fp32_all\": %.3e}\n",
           S, tmax, ex, ef, ex_all, ef_all);
    CK(hipFree(dP));
    CK(hipFree(dH));
    CK(hipFree(dR));
    CK(hipFree(dW));
    CK(hipFree(db));
}

int main(int argc, char** argv) {
    const char* what = argc > 1 ? argv[1] : "all";
    const long M = argc > 2 ? atol(argv[2]) : 2048000L;
    const int T = argc > 3 ? atoi(argv[3]) : 1000;
    const int B = argc > 4 ? atoi(argv[4]) : 2048;
    if (!strcmp(what, "gemm") || !strcmp(what, "all")) probe_gemm(M);
    if (!strcmp(what, "recur") || !strcmp(what, "all")) probe_recur(T, B);
    return 0;
}
