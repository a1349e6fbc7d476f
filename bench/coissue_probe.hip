// Does FP64 vector work on one SIMD run while that SIMD's matrix core runs FP64 MFMAs?
// 512-thread blocks, one per CU: waves 0-3 (one per SIMD) issue v_mfma_f64_16x16x4f64 on 8
// independent accumulators, waves 4-7 (the SIMD's second wave) run 8 independent FMA chains
// of the given kind.  Cycles of each role alone and together (s_memtime): both ~= max means
// the two pipes overlap, ~= sum means they share.
// Build: hipcc --offload-arch=gfx950 -O3 bench/coissue_probe.hip -o build/coissue_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double double4_t __attribute__((ext_vector_type(4)));

template <typename T, int MODE>
__global__ __launch_bounds__(512) void k_co(double* out, long long* cyc, int miters, int viters) {
    // MODE 0: plain; 1: the vector waves at s_setprio 3; 2: s_nop padding after each MFMA;
    // 3: both
    const int wave = threadIdx.x >> 6;
    if ((MODE & 1) && wave >= 4) __builtin_amdgcn_s_setprio(3);
    long long t0 = __builtin_amdgcn_s_memtime();
    double s = 0;
    if (wave < 4) {
        double a = (threadIdx.x + 1) * 1.0000001e-3, b = (blockIdx.x + 3) * 0.999999e-3;
        double4_t c[8];
#pragma unroll
        for (int k = 0; k < 8; k++) c[k] = (double4_t){0.1 * k, 0.2, 0.3, 0.4};
        for (int i = 0; i < miters; i++) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[k], 0, 0, 0);
                if (MODE & 2) {
                    asm volatile("s_nop 15");
                    asm volatile("s_nop 15");
                    asm volatile("s_nop 15");
                }
            }
        }
#pragma unroll
        for (int k = 0; k < 8; k++) s += c[k][0] + c[k][3];
    } else {
        T x[8];
        const T m = (T)1.0000001, a = (T)(threadIdx.x * 1e-7);
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = (T)(k + threadIdx.x);
        for (int i = 0; i < viters; i++) {
#pragma unroll
            for (int k = 0; k < 8; k++) x[k] = x[k] * m + a;
        }
#pragma unroll
        for (int k = 0; k < 8; k++) s += (double)x[k];
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) {
        out[blockIdx.x * 8 + wave] = s;
        cyc[blockIdx.x * 8 + wave] = t1 - t0;
    }
}

template <typename T, int MODE>
void run(const char* name, int cus, double* d, long long* cyc) {
    const int M = 2000, V = 8000;
    const int cases[3][2] = {{M, 0}, {0, V}, {M, V}};
    const char* cn[3] = {"mfma_only", "valu_only", "both"};
    for (int c = 0; c < 3; c++) {
        k_co<T, MODE><<<cus, 512>>>(d, cyc, 10, 10);
        hipDeviceSynchronize();
        k_co<T, MODE><<<cus, 512>>>(d, cyc, cases[c][0], cases[c][1]);
        hipDeviceSynchronize();
        long long h[16];
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        printf("%s mode %d %s: mfma-wave cycles %lld (%.1f per MFMA), valu-wave cycles %lld (%.2f per instr)\n", name, MODE, cn[c],
               h[0], cases[c][0] ? (double)h[0] / (cases[c][0] * 8.0) : 0.0, h[4],
               cases[c][1] ? (double)h[4] / (cases[c][1] * 8.0) : 0.0);
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
    run<double, 0>("f64", cus, d, cyc);
    run<double, 1>("f64", cus, d, cyc);
    run<double, 2>("f64", cus, d, cyc);
    run<double, 3>("f64", cus, d, cyc);
    run<int, 0>("i32", cus, d, cyc);
    run<int, 1>("i32", cus, d, cyc);
    run<int, 2>("i32", cus, d, cyc);
    return 0;
}
