// Cycles per v_mfma_f64_16x16x4f64 on one SIMD (s_memtime, shader clock) and the chip-wide
// rate at 1..8 waves per SIMD with 8 independent accumulators per wave: separates the
// instruction's issue cost from the clock the chip holds under FP64 MFMA load.
// Build: hipcc --offload-arch=gfx950 -O3 bench/mfma_probe.hip -o build/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double double4_t __attribute__((ext_vector_type(4)));

__global__ void k_mfma(double* out, long long* cyc, int iters) {
    double a = (threadIdx.x + 1) * 1.0000001e-3, b = (blockIdx.x + 3) * 0.999999e-3;
    double4_t c[8];
#pragma unroll
    for (int k = 0; k < 8; k++) c[k] = (double4_t){0.1 * k, 0.2, 0.3, 0.4};
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[k], 0, 0, 0);
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) s += c[k][0] + c[k][3];
    if (threadIdx.x == 0) {
        out[blockIdx.x] = s;
        cyc[blockIdx.x] = t1 - t0;
    }
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    double* d;
    long long* cyc;
    hipMalloc(&d, sizeof(double) * cus * 64);
    hipMalloc(&cyc, sizeof(long long) * cus * 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("{\"cus\": %d, \"rows\": [", cus);
    const int iters = 2000;
    for (int wps = 1; wps <= 8; wps *= 2) {  // waves per SIMD: blocks of 256 threads = 4 waves (one per SIMD)
        const int blocks = cus * wps;
        k_mfma<<<blocks, 256>>>(d, cyc, 10);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        k_mfma<<<blocks, 256>>>(d, cyc, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        long long c0;
        hipMemcpy(&c0, cyc, sizeof(long long), hipMemcpyDeviceToHost);
        const double nm = (double)blocks * 4 * iters * 8;  // MFMA instructions (waves x per wave)
        const double tf = nm * 2048.0 / (ms * 1e-3) / 1e12;
        // per SIMD: wps waves x iters x 8 MFMAs in c0 shader cycles (memtime counts shader clocks)
        printf("%s{\"waves_per_simd\": %d, \"tflops\": %.2f, \"cycles_per_mfma_per_simd\": %.2f, \"implied_clock_ghz\": %.3f}",
               wps == 1 ? "" : ", ", wps, tf, (double)c0 / (wps * (double)iters * 8),
               (double)c0 / (ms * 1e-3) / 1e9);
    }
    printf("]}\n");
    return 0;
}
