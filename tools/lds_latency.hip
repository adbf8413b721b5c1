// Microbenchmark: latency of s_memtime, dependent LDS reads / atomics, and
// block barriers on gfx950, with 1..8 waves in the workgroup.  Diagnostic
// tool for the decoder design; not part of the product.
//   hipcc --offload-arch=gfx950 -O3 tools/lds_latency.hip -o build/lds_latency
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int N = 256;

__global__ void lat(uint64_t* out, int mode, int active_waves) {
    __shared__ uint32_t buf[4096];
    __shared__ uint64_t b64[1024];
    const int tid = threadIdx.x, w = tid >> 6;
    for (int i = tid; i < 4096; i += blockDim.x) buf[i] = (uint32_t)((i * 7 + 1) & 4095);
    for (int i = tid; i < 1024; i += blockDim.x) b64[i] = 0;
    __syncthreads();
    uint64_t t0 = 0, t1 = 0;
    uint32_t x = (uint32_t)tid & 63;
    if (w < active_waves) {
        t0 = __builtin_amdgcn_s_memtime();
        if (mode == 0) {            // empty: s_memtime pair
        } else if (mode == 1) {     // dependent ds_read_b32 chain
            for (int i = 0; i < N; i++) x = buf[x];
        } else if (mode == 2) {     // dependent ds_cmpst_rtn_b64 chain (always fails)
            for (int i = 0; i < N; i++) {
                const unsigned long long p =
                    atomicCAS((unsigned long long*)&b64[x & 1023], 1ull, 2ull);
                x = (uint32_t)(p + x + 1) & 1023;
            }
        } else if (mode == 3) {     // __syncthreads only
            for (int i = 0; i < N; i++) __syncthreads();
        } else if (mode == 4) {     // dependent ds_read_b32 + __shfl (bpermute)
            for (int i = 0; i < N; i++) x = (uint32_t)__shfl((int)x, (int)(x + 1) & 63);
        } else if (mode == 5) {     // dependent DPP row_shr + readlane
            for (int i = 0; i < N; i++) {
                x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
                x = (uint32_t)__builtin_amdgcn_readlane((int)x, 15) & 63;
            }
        } else if (mode == 7) {     // ds_add_rtn_u32, all lanes one address
            for (int i = 0; i < N; i++) x = atomicAdd(&buf[x & 0x1000], 1u) & 63;
        } else if (mode == 8) {     // ds_add_rtn_u32, distinct addresses
            for (int i = 0; i < N; i++) x = atomicAdd(&buf[(x & 0) + (tid & 63) * 1], 1u) & 63;
        } else if (mode == 9) {     // ds_or_b64 no return, all lanes one address, then one read
            for (int i = 0; i < N; i++) atomicOr((unsigned long long*)&b64[0], 1ull << (tid & 63));
            x = (uint32_t)b64[1];
        } else if (mode == 10) {    // ds_cmpst_rtn_b64 all lanes one address (always fails)
            for (int i = 0; i < N; i++) {
                const unsigned long long p = atomicCAS((unsigned long long*)&b64[x & 0x400], 1ull, 2ull);
                x = (uint32_t)p & 63;
            }
        } else if (mode == 11) {    // ds_or_b32 no return, all lanes one address
            for (int i = 0; i < N; i++) atomicOr(&buf[0], 1u << (tid & 31));
            x = buf[1];
        } else if (mode == 12) {    // ds_or_b64 no return, distinct addresses
            for (int i = 0; i < N; i++) atomicOr((unsigned long long*)&b64[tid & 63], 1ull << (tid & 63));
            x = (uint32_t)b64[1];
        } else if (mode == 13) {    // ds_max_u64 no return, all lanes one address
            for (int i = 0; i < N; i++) atomicMax((unsigned long long*)&b64[0], (unsigned long long)(tid + i));
            x = (uint32_t)b64[1];
        } else if (mode == 14) {    // ds_max_u32 no return, all lanes one address
            for (int i = 0; i < N; i++) atomicMax(&buf[0], (uint32_t)(tid + i));
            x = buf[1];
        } else if (mode == 15) {    // ds_or_b64 no return, 4 lanes per address
            for (int i = 0; i < N; i++) atomicOr((unsigned long long*)&b64[(tid & 63) >> 2], 1ull << (tid & 63));
            x = (uint32_t)b64[1];
        } else if (mode == 16) {    // ds_add_u64 no return, all lanes one address
            for (int i = 0; i < N; i++) atomicAdd((unsigned long long*)&b64[0], 1ull << (tid & 63));
            x = (uint32_t)b64[1];
        } else if (mode == 17) {    // ds_add_u32 no return, all lanes one address
            for (int i = 0; i < N; i++) atomicAdd(&buf[0], 1u);
            x = buf[1];
        } else if (mode == 18) {    // ds_add_u32 no return, 16 addresses (histogram-like)
            for (int i = 0; i < N; i++) atomicAdd(&buf[(tid * 7) & 15], 1u);
            x = buf[1];
        } else if (mode == 19) {    // ds_add_u32, 2 addresses x 32 lanes
            for (int i = 0; i < N; i++) atomicAdd(&buf[tid & 1], 1u);
            x = buf[1];
        } else if (mode == 20) {    // ds_add_u32, 48 lanes one address + 16 distinct
            for (int i = 0; i < N; i++) atomicAdd(&buf[(tid & 63) < 48 ? 0 : (tid & 63)], 1u);
            x = buf[1];
        } else if (mode == 21) {    // ds_add_u32, 20 active lanes, one address
            if ((tid & 63) < 20)
                for (int i = 0; i < N; i++) atomicAdd(&buf[0], 1u);
            x = buf[1];
        } else if (mode == 22) {    // ds_add_u32, 64 lanes, 8 addresses skewed (geometric)
            const int a = __builtin_ctz((tid & 63) | 64);   // 0:32 lanes, 1:16, 2:8, ...
            for (int i = 0; i < N; i++) atomicAdd(&buf[a], 1u);
            x = buf[1];
        } else if (mode == 23) {    // exchange: ds_write_b32 + barrier + dependent ds_read_b32
            for (int i = 0; i < N; i++) {
                buf[2048 + (i & 1) * 1024 + tid] = x;
                __syncthreads();
                x = buf[2048 + (i & 1) * 1024 + ((tid + 64) & (blockDim.x - 1))] & 63;
            }
        } else if (mode == 24) {    // ds_write_b64 x4 + barrier (write drain) + read
            for (int i = 0; i < N; i++) {
                b64[(i & 1) * 512 + (tid & 63)] = x;
                b64[(i & 1) * 512 + 64 + (tid & 63)] = x + 1;
                b64[(i & 1) * 512 + 128 + (tid & 63)] = x + 2;
                b64[(i & 1) * 512 + 192 + (tid & 63)] = x + 3;
                __syncthreads();
                x = (uint32_t)b64[(i & 1) * 512 + ((tid + 1) & 63)] & 63;
            }
        } else if (mode == 6) {     // dependent ds_read_b64
            uint64_t y = x;
            for (int i = 0; i < N; i++) y = b64[y & 1023] + (y & 1023);
            x = (uint32_t)y;
        }
        t1 = __builtin_amdgcn_s_memtime();
    }
    if ((mode == 3 || mode == 23 || mode == 24) && w >= active_waves)
        for (int i = 0; i < N; i++) __syncthreads();
    if ((tid & 63) == 0) out[blockIdx.x * 16 + w] = (t1 - t0) + (x == 0xFFFFFFFFu ? 1 : 0);
}

int main() {
    uint64_t* d;
    hipMalloc(&d, sizeof(uint64_t) * 16 * 64);
    uint64_t h[16 * 64];
    const char* names[] = {"memtime pair", "ds_read_b32 chain", "ds_cmpst_b64 chain", "barrier",
                           "shfl chain", "dpp+readlane chain", "ds_read_b64 chain",
                           "ds_add_rtn same addr", "ds_add_rtn distinct", "ds_or_b64 same addr",
                           "ds_cmpst same addr", "ds_or_b32 same addr", "ds_or_b64 distinct",
                           "ds_max_u64 same addr", "ds_max_u32 same addr", "ds_or_b64 4/addr",
                           "ds_add_u64 same addr", "ds_add_u32 same addr", "ds_add_u32 16 addrs",
                           "ds_add_u32 2x32", "ds_add_u32 48+16", "ds_add_u32 20 lanes 1 addr",
                           "ds_add_u32 geometric", "write+barrier+read", "4x write_b64+barrier+read"};
    for (int mode : {0, 1, 6, 3, 23, 24})
        for (int nw : {1, 2, 4, 8}) {
            for (int rep = 0; rep < 2; rep++) {
                hipLaunchKernelGGL(lat, dim3(64), dim3(64 * nw), 0, 0, d, mode,
                                   (mode == 3 || mode == 23 || mode == 24) ? nw : 1);
                hipDeviceSynchronize();
            }
            hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
            const double per = mode == 0 ? (double)h[0] : (double)h[0] / N;
            printf("%-20s waves=%d  cycles%s = %.1f\n", names[mode], nw, mode == 0 ? "" : "/op",
                   per);
        }
    return 0;
}
