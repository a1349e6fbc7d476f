// Accuracy and dependent latency of the FP64 reciprocal square roots a Cholesky pivot can use
// (k_solve_dmx's diag_factor): the library rsqrt (ocml), the hardware v_rsq_f64 alone, and
// v_rsq_f64 + one / two Newton steps.  Errors in ulps against 1/sqrt in x87 long double on the
// host; latency in shader cycles per dependent call (s_memtime over a chain of 1024).
// Build: hipcc --offload-arch=gfx950 -O3 bench/rsq_probe.hip -o build/rsq_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__device__ __forceinline__ double rsq_nr1(double d) {
    double y = __builtin_amdgcn_rsq(d);
    const double h = 0.5 * d;
    const double e = __builtin_fma(-h * y, y, 0.5);  // 0.5 - d y^2 / 2
    return __builtin_fma(y, e, y);
}
__device__ __forceinline__ double rsq_nr2(double d) {
    double y = rsq_nr1(d);
    const double h = 0.5 * d;
    const double e = __builtin_fma(-h * y, y, 0.5);
    return __builtin_fma(y, e, y);
}

__global__ void k_acc(const double* d, double* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = d[i];
    out[4 * i] = rsqrt(x);
    out[4 * i + 1] = __builtin_amdgcn_rsq(x);
    out[4 * i + 2] = rsq_nr1(x);
    out[4 * i + 3] = rsq_nr2(x);
}

template <int K>
__global__ void k_lat(double* out, long long* cyc, double seed) {
    double x = seed + threadIdx.x * 1e-9;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 1024; i++) {
        double y;
        if (K == 0) y = rsqrt(x);
        else if (K == 1) y = __builtin_amdgcn_rsq(x);
        else if (K == 2) y = rsq_nr1(x);
        else if (K == 3) y = rsq_nr2(x);
        else y = __builtin_fma(x, 1.0000001, 1e-300);  // one dependent FMA
        x = y * 0.5 + 0.75;  // keep x in (0.75, 1.5]: the chain's next input depends on y
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[0] = x;
        cyc[0] = t1 - t0;
    }
}

int main() {
    const int n = 1 << 20;
    std::vector<double> h(n);
    unsigned long long s = 88172645463325252ull;
    for (int i = 0; i < n; i++) {  // pivots of a normalised SPD matrix: (1e-8, 4], log-uniform
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const double u = (double)(s >> 11) / 9007199254740992.0;
        h[i] = std::exp(std::log(1e-8) + u * (std::log(4.0) - std::log(1e-8)));
    }
    double *dd, *dout, *dl;
    long long* dc;
    hipMalloc(&dd, sizeof(double) * n);
    hipMalloc(&dout, sizeof(double) * 4 * n);
    hipMalloc(&dl, sizeof(double));
    hipMalloc(&dc, sizeof(long long));
    hipMemcpy(dd, h.data(), sizeof(double) * n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_acc, dim3(n / 256), dim3(256), 0, 0, dd, dout, n);
    std::vector<double> o(4 * n);
    hipMemcpy(o.data(), dout, sizeof(double) * 4 * n, hipMemcpyDeviceToHost);
    const char* names[4] = {"ocml rsqrt", "v_rsq_f64", "v_rsq_f64 + 1 Newton", "v_rsq_f64 + 2 Newton"};
    for (int k = 0; k < 4; k++) {
        double worst = 0;
        for (int i = 0; i < n; i++) {
            const long double ref = 1.0L / std::sqrt((long double)h[i]);
            const double ulp = std::nextafter((double)ref, 1e300) - (double)ref;
            const double e = (double)std::fabs((long double)o[4 * i + k] - ref) / ulp;
            if (e > worst) worst = e;
        }
        printf("%-24s max error %.3g ulp\n", names[k], worst);
    }
    long long c = 0;
    double x = 0;
#define LAT(K, NAME)                                                               \
    hipLaunchKernelGGL(k_lat<K>, dim3(1), dim3(64), 0, 0, dl, dc, 1.1);           \
    hipMemcpy(&c, dc, sizeof(c), hipMemcpyDeviceToHost);                         \
    hipMemcpy(&x, dl, sizeof(x), hipMemcpyDeviceToHost);                          \
    printf("%-24s %.1f cycles per dependent call (+ the mul-add of the chain)\n", NAME, c / 1024.0);
    for (int rep = 0; rep < 2; rep++) {  // the first launch warms the code object
        LAT(0, "ocml rsqrt")
        LAT(1, "v_rsq_f64")
        LAT(2, "v_rsq_f64 + 1 Newton")
        LAT(3, "v_rsq_f64 + 2 Newton")
        LAT(4, "fma")
    }
    return 0;
}
