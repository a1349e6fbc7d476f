// Microbenchmarks for the roofline peaks used by bench.py (MI355X, gfx950):
//   f64 MFMA  v_mfma_f64_16x16x4f64, 4 independent accumulators per wave, all CUs
//   f64 FMA   v_fma_f64 vector rate
//   HBM       read+write streaming copy (16 B per lane)
// Build: hipcc --offload-arch=gfx950 -O3 bench/peaks.hip -o build/peaks
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double double4_t __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_mfma64(double* out, int iters) {
    double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
    double4_t c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < iters; i++) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    double s = c0[0] + c1[1] + c2[2] + c3[3];
    if (s == 12345.0) out[0] = s;
}

__global__ __launch_bounds__(256) void k_fma64(double* out, int iters) {
    double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    const double m = 0.999999, a = 1e-7;
    for (int i = 0; i < iters; i++) {
        x0 = fma(x0, m, a); x1 = fma(x1, m, a); x2 = fma(x2, m, a); x3 = fma(x3, m, a);
        x4 = fma(x4, m, a); x5 = fma(x5, m, a); x6 = fma(x6, m, a); x7 = fma(x7, m, a);
    }
    double s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
    if (s == 12345.0) out[0] = s;
}

__global__ __launch_bounds__(256) void k_copy(const double4_t* __restrict__ in, double4_t* __restrict__ out, long n) {
    long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    long stride = (long)gridDim.x * blockDim.x;
    for (; i < n; i += stride) out[i] = in[i];
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    int cus = p.multiProcessorCount;
    double* d;
    hipMalloc(&d, 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float ms;
    // MFMA f64: 4 waves/block x (8 blocks per CU) ; flops per mfma = 16*16*4*2
    int blocks = cus * 8, iters = 4000;
    k_mfma64<<<blocks, 256>>>(d, 10);
    hipEventRecord(e0);
    k_mfma64<<<blocks, 256>>>(d, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    double fl = (double)blocks * 4 * iters * 4 * 2048.0;
    printf("{\"f64_mfma_tflops\": %.2f, ", fl / (ms * 1e-3) / 1e12);
    k_fma64<<<blocks, 256>>>(d, 10);
    hipEventRecord(e0);
    k_fma64<<<blocks, 256>>>(d, iters * 4);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    fl = (double)blocks * 256 * iters * 4 * 8 * 2.0;
    printf("\"f64_fma_tflops\": %.2f, ", fl / (ms * 1e-3) / 1e12);
    long n = 1L << 27;  // 4 GiB of double4 per buffer
    double4_t *a, *b;
    hipMalloc(&a, n * sizeof(double4_t));
    hipMalloc(&b, n * sizeof(double4_t));
    hipMemset(a, 0, n * sizeof(double4_t));
    k_copy<<<cus * 16, 256>>>(a, b, n);
    hipEventRecord(e0);
    for (int r = 0; r < 5; r++) k_copy<<<cus * 16, 256>>>(a, b, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("\"hbm_copy_gbs\": %.1f, \"cus\": %d, \"clock_mhz\": %d}\n", 5.0 * 2 * n * sizeof(double4_t) / (ms * 1e-3) / 1e9,
           cus, p.clockRate / 1000);
    return 0;
}
