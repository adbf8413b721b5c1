#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}
__global__ void k(const uint32_t* in, uint32_t* out) { out[threadIdx.x] = wave_incl_scan(in[threadIdx.x]); }
int main() {
    uint32_t h[64], o[64]; for (int i = 0; i < 64; i++) h[i] = (i * 7 + 3) % 11;
    uint32_t *di, *dout; hipMalloc(&di, 256); hipMalloc(&dout, 256);
    hipMemcpy(di, h, 256, hipMemcpyHostToDevice);
    k<<<1, 64>>>(di, dout); hipMemcpy(o, dout, 256, hipMemcpyDeviceToHost);
    uint32_t s = 0; int bad = 0;
    for (int i = 0; i < 64; i++) { s += h[i]; if (o[i] != s) bad++; }
    printf("scan mismatches: %d\n", bad); return bad != 0;
}
