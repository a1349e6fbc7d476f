// FP64 vector FMA issue rate on one SIMD: 1 or 2 waves per SIMD, NCH independent chains
// per wave (s_memtime cycles per v_fma_f64).
// Build: hipcc --offload-arch=gfx950 -O3 bench/valu_probe.hip -o build/valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>

template <int NCH>
__global__ __launch_bounds__(512) void k_valu(double* out, long long* cyc, int iters, int nwaves) {
    const int wave = threadIdx.x >> 6;
    if (wave >= nwaves) return;
    double x[NCH];
    const double m = 1.0000001, a = threadIdx.x * 1e-7;
#pragma unroll
    for (int k = 0; k < NCH; k++) x[k] = k + threadIdx.x;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < NCH; k++) x[k] = x[k] * m + a;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int k = 0; k < NCH; k++) s += x[k];
    if ((threadIdx.x & 63) == 0) {
        out[blockIdx.x * 8 + wave] = s;
        cyc[blockIdx.x * 8 + wave] = t1 - t0;
    }
}

template <int NCH>
void run(int cus, double* d, long long* cyc) {
    for (int nw = 4; nw <= 8; nw += 4) {
        const int iters = 32768 / NCH;
        k_valu<NCH><<<cus, 512>>>(d, cyc, 10, nw);
        hipDeviceSynchronize();
        k_valu<NCH><<<cus, 512>>>(d, cyc, iters, nw);
        hipDeviceSynchronize();
        long long h[8];
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        printf("chains %2d waves/SIMD %d: %.2f cycles per v_fma_f64 per wave\n", NCH, nw / 4,
               (double)h[0] / (iters * (double)NCH));
    }
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    double* d;
    long long* cyc;
    hipMalloc(&d, sizeof(double) * cus * 8);
    hipMalloc(&cyc, sizeof(long long) * cus * 8);
    run<1>(cus, d, cyc);
    run<2>(cus, d, cyc);
    run<4>(cus, d, cyc);
    run<8>(cus, d, cyc);
    run<16>(cus, d, cyc);
    run<32>(cus, d, cyc);
    return 0;
}
