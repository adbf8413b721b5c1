// Probe: accuracy of the decoder's fp64 lse (csrc/ctc_beam_kernel.inc: lse2 =
// max + lse_log1p01(lse_exp_neg(-|a - b|))) against a long-double reference
// and against glibc's double log1p(exp(.)), over random pairs whose gap
// covers the folds' range (0 .. 40 nats, and a tail to 745).
//   hipcc --offload-arch=gfx950 -O3 -I gpu-accelerated-speech-recognition_amd/csrc \
//         -I include -o tools/lse_probe tools/lse_probe.hip && tools/lse_probe [N]
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "ctc_beam_kernel.inc"

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

__global__ void lse_kernel(const double* a, const double* b, double* out, double* sp, long n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = asr::lse2(a[i], b[i]);
    sp[i] = asr::lse_log1p01(asr::lse_exp_neg(-fabs(a[i] - b[i])));   // the softplus term alone
}

static double ulp_of(double x) { return std::nextafter(std::fabs(x), INFINITY) - std::fabs(x); }

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1L << 24;
    std::mt19937_64 rng(20261018);
    std::uniform_real_distribution<double> base(-3000.0, 0.0), gap(0.0, 40.0), tail(40.0, 745.0);
    std::vector<double> a(n), b(n);
    for (long i = 0; i < n; i++) {
        a[i] = base(rng);
        const double d = (i % 16 == 0) ? tail(rng) : gap(rng);
        b[i] = (i & 1) ? a[i] - d : a[i] + d;
    }
    double *da, *db, *dout, *dsp;
    CK(hipMalloc(&da, n * 8));
    CK(hipMalloc(&db, n * 8));
    CK(hipMalloc(&dout, n * 8));
    CK(hipMalloc(&dsp, n * 8));
    CK(hipMemcpy(da, a.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, b.data(), n * 8, hipMemcpyHostToDevice));
    lse_kernel<<<(unsigned)((n + 255) / 256), 256>>>(da, db, dout, dsp, n);
    CK(hipGetLastError());
    std::vector<double> out(n), sp(n);
    CK(hipMemcpy(out.data(), dout, n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sp.data(), dsp, n * 8, hipMemcpyDeviceToHost));
    double max_sp_ulp = 0, max_lse_ulp = 0, max_glibc_sp_ulp = 0;
    long eq_glibc = 0;
    for (long i = 0; i < n; i++) {
        const double d = std::fabs(a[i] - b[i]);
        const long double ref_sp = log1pl(expl(-(long double)d));
        const double ref_spd = (double)ref_sp;
        if (ref_spd > 0) {
            max_sp_ulp = std::max(max_sp_ulp, (double)(std::fabs((long double)sp[i] - ref_sp) / ulp_of(ref_spd)));
            const double g = std::log1p(std::exp(-d));
            max_glibc_sp_ulp = std::max(max_glibc_sp_ulp, (double)(std::fabs((long double)g - ref_sp) / ulp_of(ref_spd)));
        }
        const double m = std::max(a[i], b[i]);
        const long double ref = (long double)m + ref_sp;
        max_lse_ulp = std::max(max_lse_ulp, (double)(std::fabs((long double)out[i] - ref) / ulp_of((double)ref)));
        const double gl = m + std::log1p(std::exp(-d));
        if (gl == out[i]) eq_glibc++;
    }
    printf("{\"pairs\": %ld, \"softplus_max_ulp\": %.3f, \"glibc_softplus_max_ulp\": %.3f, "
           "\"lse_max_ulp\": %.3f, \"lse_bit_equal_to_glibc\": %.5f}\n",
           n, max_sp_ulp, max_glibc_sp_ulp, max_lse_ulp, (double)eq_glibc / n);
    return 0;
}
