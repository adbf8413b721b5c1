// Test helper (never part of the product): fills every CU's LDS with
// 0xFFFFFFFF (a NaN as fp32) so that a kernel launched next on the same
// stream that reads LDS it did not write shows up as NaN output
// (gemm_wide_kernel's B^T slice past K).
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(1024) void lds_poison_kernel(unsigned n_words) {
    extern __shared__ unsigned lds_words[];
    for (unsigned i = threadIdx.x; i < n_words; i += blockDim.x) lds_words[i] = 0xFFFFFFFFu;
    __syncthreads();
}

extern "C" int lds_poison(void* stream) {
    const size_t bytes = 160 * 1024;
    if (hipFuncSetAttribute((const void*)lds_poison_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)bytes) != hipSuccess)
        return 1;
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 1;
    hipLaunchKernelGGL(lds_poison_kernel, dim3(4 * ncu), dim3(1024), bytes, (hipStream_t)stream,
                       (unsigned)(bytes / 4));
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
