// The 16x16 diagonal-block factor of the blocked Cholesky (k_solve_dmx's diag_factor): one
// wave factors a symmetric positive-definite 16x16 block held in LDS and overwrites it with
// L^-1.  Variants:
//   0  as in pint_hip.hip (row per lane, readlane broadcasts; the compiler hoists the
//      readlanes of several pivots and spills SGPRs to VGPR lanes),
//   1  the same arithmetic with a scheduling barrier after each pivot (no cross-pivot
//      hoisting: the broadcasts of one pivot live in SGPRs at a time),
//   2  variant 1 with one Newton step on v_rsq_f64 instead of two,
//   3  the pivot column broadcast through LDS (VGPR operands), 4: that with one Newton step,
//   5  variant 3 with a scheduling barrier after each pivot,
//   6  two waves: the factorisation (readlane) and the inverse (LDS columns) one pivot apart,
//   7  variant 0 with the lane index opaque per pivot (no hoisted lane-mask SGPR pairs),
//   8  readlane broadcasts, every lane scaling its entry (a[j] *= il: no lane masks; the rows
//      above the pivot hold values no later pivot reads), a scheduling barrier per pivot,
//   9  variant 8 with the pivot column through LDS, 10: that without the barrier.
// The kernel is compiled with the register budget of -DLB threads per workgroup (default
// 1024, the 16-wave solves' 128 VGPRs; 512: the 8-wave solve's 256).
// Prints the max error of L^-1 against a long-double Cholesky inverse on the host (relative
// to max |L^-1|) and the cycles per factor (s_memtime, 64 dependent factors in one wave).
// Build: hipcc --offload-arch=gfx950 -O3 bench/diag_probe.hip -o build/diag_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__device__ __forceinline__ double rdlane(double v, int l) {
    long long b = __double_as_longlong(v);
    int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
    int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ int swz(int r, int c) { return (c << 4) + (r ^ (c & 14)); }

template <int NEWTON>
__device__ __forceinline__ double rsqn(double d) {
    double y = __builtin_amdgcn_rsq(d);
    const double h = 0.5 * d;
#pragma unroll
    for (int k = 0; k < NEWTON; k++) y = __builtin_fma(y, __builtin_fma(-h * y, y, 0.5), y);
    return y;
}

template <int V>
__device__ __forceinline__ bool diag_factor(double* Akk, int lane) {
    const int r = lane & 15;
    double a[16], x[16];
#pragma unroll
    for (int c = 0; c < 16; c++) {
        a[c] = Akk[swz(r, c)];
        x[c] = (r == c) ? 1.0 : 0.0;
    }
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const double djj = rdlane(a[j], j);
        ok = ok && (djj > 0.0);
        const double il = V == 2 ? rsqn<1>(djj) : rsqn<2>(djj);
        a[j] = (r == j) ? djj * il : (r > j ? a[j] * il : 0.0);
        x[j] *= il;
#pragma unroll
        for (int c = j + 1; c < 16; c++) {
            const double Lcj = rdlane(a[j], c);
            a[c] -= a[j] * Lcj;
            x[c] -= Lcj * x[j];
        }
        if (V >= 1) __builtin_amdgcn_sched_barrier(0);
    }
    if (lane < 16) {
#pragma unroll
        for (int t = 0; t < 16; t++) Akk[swz(t, r)] = x[t];
    }
    return ok;
}

// variant 7: as variant 0, with the lane's row index made opaque in every pivot, so the
// compiler cannot hoist the sixteen pivots' lane-mask compares (SGPR pairs kept live, spilled
// to VGPR lanes); for lane r == j the scaled pivot a[j] * il is djj * il exactly
__device__ __forceinline__ bool diag_factor_c4(double* Akk, int lane) {
    int r = lane & 15;
    double a[16], x[16];
#pragma unroll
    for (int c = 0; c < 16; c++) {
        a[c] = Akk[swz(r, c)];
        x[c] = (r == c) ? 1.0 : 0.0;
    }
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        __asm__ volatile("" : "+v"(r));
        const double djj = rdlane(a[j], j);
        ok = ok && (djj > 0.0);
        const double il = rsqn<2>(djj);
        a[j] = (r >= j) ? a[j] * il : 0.0;
        x[j] *= il;
#pragma unroll
        for (int c = j + 1; c < 16; c++) {
            const double Lcj = rdlane(a[j], c);
            a[c] -= a[j] * Lcj;
            x[c] -= Lcj * x[j];
        }
    }
    if (lane < 16) {
#pragma unroll
        for (int t = 0; t < 16; t++) Akk[swz(t, r)] = x[t];
    }
    return ok;
}

// variants 8-10: no lane masks (every lane scales its own entry), readlane or LDS columns
template <bool LDSC, bool SB>
__device__ __forceinline__ bool diag_factor_nm(double* Akk, double* colbuf, int lane) {
    const int r = lane & 15;
    double a[16], x[16];
#pragma unroll
    for (int c = 0; c < 16; c++) {
        a[c] = Akk[swz(r, c)];
        x[c] = (r == c) ? 1.0 : 0.0;
    }
    bool ok = true;
    typedef __attribute__((address_space(3))) double ldsd;
    typedef double dv2 __attribute__((ext_vector_type(2)));
    typedef __attribute__((address_space(3))) dv2 ldsd2;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const double djj = rdlane(a[j], j);
        ok = ok && (djj > 0.0);
        const double il = rsqn<2>(djj);
        a[j] *= il;
        x[j] *= il;
        if constexpr (LDSC) {
            if (lane < 16) ((ldsd*)colbuf)[lane] = a[j];
            __builtin_amdgcn_wave_barrier();
            double Lc[16];
#pragma unroll
            for (int c2 = (j + 1) / 2; c2 < 8; c2++) {
                const dv2 v = ((ldsd2*)colbuf)[c2];
                Lc[2 * c2] = v.x;
                Lc[2 * c2 + 1] = v.y;
            }
#pragma unroll
            for (int c = j + 1; c < 16; c++) {
                a[c] -= a[j] * Lc[c];
                x[c] -= Lc[c] * x[j];
            }
            __builtin_amdgcn_wave_barrier();
        } else {
#pragma unroll
            for (int c = j + 1; c < 16; c++) {
                const double Lcj = rdlane(a[j], c);
                a[c] -= a[j] * Lcj;
                x[c] -= Lcj * x[j];
            }
        }
        if (SB) __builtin_amdgcn_sched_barrier(0);
    }
    if (lane < 16) {
#pragma unroll
        for (int t = 0; t < 16; t++) Akk[swz(t, r)] = x[t];
    }
    return ok;
}

// variant 3: the scaled pivot column goes through LDS (one ds_write by lanes 0..15, then
// uniform-address reads: every lane gets L_cj in VGPRs, no SGPR broadcasts)
template <int NEWTON, bool SB = false>
__device__ __forceinline__ bool diag_factor_lds(double* Akk, double* colbuf, int lane) {
    const int r = lane & 15;
    double a[16], x[16];
#pragma unroll
    for (int c = 0; c < 16; c++) {
        a[c] = Akk[swz(r, c)];
        x[c] = (r == c) ? 1.0 : 0.0;
    }
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const double djj = rdlane(a[j], j);
        ok = ok && (djj > 0.0);
        const double il = rsqn<NEWTON>(djj);
        a[j] = (r == j) ? djj * il : (r > j ? a[j] * il : 0.0);
        x[j] *= il;
        typedef __attribute__((address_space(3))) double ldsd;
        typedef double dv2 __attribute__((ext_vector_type(2)));
        typedef __attribute__((address_space(3))) dv2 ldsd2;
        if (lane < 16) ((ldsd*)colbuf)[lane] = a[j];
        __builtin_amdgcn_wave_barrier();
        double Lc[16];
#pragma unroll
        for (int c2 = (j + 1) / 2; c2 < 8; c2++) {
            const dv2 v = ((ldsd2*)colbuf)[c2];
            Lc[2 * c2] = v.x;
            Lc[2 * c2 + 1] = v.y;
        }
#pragma unroll
        for (int c = j + 1; c < 16; c++) {
            a[c] -= a[j] * Lc[c];
            x[c] -= Lc[c] * x[j];
        }
        __builtin_amdgcn_wave_barrier();
        if (SB) __builtin_amdgcn_sched_barrier(0);
    }
    if (lane < 16) {
#pragma unroll
        for (int t = 0; t < 16; t++) Akk[swz(t, r)] = x[t];
    }
    return ok;
}

// variant 6: two waves.  Wave 0 factors (lane r holds row r of A, readlane broadcasts of the
// scaled pivot column, as variant 1 without the x updates) and publishes each scaled column
// L[.][j] in LDS with a counter; wave 1 forms X = L^-1 (lane r holds column r of X) from the
// published columns as they arrive (uniform-address LDS loads), one pivot behind.
__device__ __forceinline__ bool diag_factor2(double* Akk, double* colbuf, volatile int* cnt, int wave, int lane) {
    const int r = lane & 15;
    typedef double dv2 __attribute__((ext_vector_type(2)));
    typedef __attribute__((address_space(3))) double ldsd;
    typedef __attribute__((address_space(3))) dv2 ldsd2;
    bool ok = true;
    if (wave == 0) {
        double a[16];
#pragma unroll
        for (int c = 0; c < 16; c++) a[c] = Akk[swz(r, c)];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const double djj = rdlane(a[j], j);
            ok = ok && (djj > 0.0);
            const double il = rsqn<2>(djj);
            a[j] = (r == j) ? djj * il : (r > j ? a[j] * il : 0.0);
            if (lane < 16) ((ldsd*)colbuf)[16 * j + lane] = a[j];
            colbuf[256 + j] = il;  // (uniform) the pivot's 1/L_jj for wave 1
            __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) *cnt = j + 1;
#pragma unroll
            for (int c = j + 1; c < 16; c++) {
                const double Lcj = rdlane(a[j], c);
                a[c] -= a[j] * Lcj;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    } else if (wave == 1) {
        double x[16];
#pragma unroll
        for (int c = 0; c < 16; c++) x[c] = (r == c) ? 1.0 : 0.0;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            while (*cnt < j + 1) __builtin_amdgcn_s_sleep(1);
            __asm__ volatile("" ::: "memory");
            const double il = colbuf[256 + j];
            x[j] *= il;
            double Lc[16];
#pragma unroll
            for (int c2 = (j + 1) / 2; c2 < 8; c2++) {
                const dv2 v = ((ldsd2*)colbuf)[8 * j + c2];
                Lc[2 * c2] = v.x;
                Lc[2 * c2 + 1] = v.y;
            }
#pragma unroll
            for (int c = j + 1; c < 16; c++) x[c] -= Lc[c] * x[j];
            __builtin_amdgcn_sched_barrier(0);
        }
        if (lane < 16) {
#pragma unroll
            for (int t = 0; t < 16; t++) Akk[swz(t, r)] = x[t];
        }
    }
    return ok;
}

template <int V>
__device__ __forceinline__ bool factor_v(double* Akk, double* colbuf, int lane) {
    if constexpr (V == 8) return diag_factor_nm<false, true>(Akk, colbuf, lane);
    else if constexpr (V == 9) return diag_factor_nm<true, true>(Akk, colbuf, lane);
    else if constexpr (V == 10) return diag_factor_nm<true, false>(Akk, colbuf, lane);
    else if constexpr (V == 7) return diag_factor_c4(Akk, lane);
    else if constexpr (V >= 5) return diag_factor_lds<2, true>(Akk, colbuf, lane);
    else if constexpr (V >= 3) return diag_factor_lds<V == 3 ? 2 : 1>(Akk, colbuf, lane);
    else return diag_factor<V>(Akk, lane);
}

#ifndef LB
#define LB 1024
#endif
template <int V>
__global__ __launch_bounds__(LB) void k_diag(const double* __restrict__ in, double* __restrict__ out,
                                             long long* __restrict__ cyc, int reps) {
    __shared__ double blk[256];
    __shared__ double colbuf[16 * 16 + 16];
    __shared__ int cnt;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if constexpr (V == 6) {  // two waves (128 threads); the other variants run on one
        for (int e = threadIdx.x; e < 256; e += blockDim.x) blk[e] = in[e];
        if (threadIdx.x == 0) cnt = 0;
        __syncthreads();
        bool ok6 = diag_factor2(blk, colbuf, &cnt, wave, lane);
        __syncthreads();
        for (int e = threadIdx.x; e < 256; e += blockDim.x) out[e] = blk[e];
        __syncthreads();
        long long t0 = __builtin_amdgcn_s_memtime();
        for (int k = 0; k < reps; k++) {
            for (int e = threadIdx.x; e < 256; e += blockDim.x) blk[e] = in[e] + (ok6 ? 0.0 : 1.0) * blk[e];
            if (threadIdx.x == 0) cnt = 0;
            __syncthreads();
            ok6 &= diag_factor2(blk, colbuf, &cnt, wave, lane);
            __syncthreads();
        }
        long long t1 = __builtin_amdgcn_s_memtime();
        if (threadIdx.x == 0) cyc[0] = (t1 - t0) / reps;
        return;
    }
    for (int e = lane; e < 256; e += 64) blk[e] = in[e];
    __syncthreads();
    bool ok = factor_v<V>(blk, colbuf, lane);
    __syncthreads();
    for (int e = lane; e < 256; e += 64) out[e] = blk[e];
    // timing: reps dependent factors of the same block (restaged from registers each time)
    __syncthreads();
    for (int e = lane; e < 256; e += 64) blk[e] = in[e];
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < reps; k++) {
        ok &= factor_v<V>(blk, colbuf, lane);
        __syncthreads();
        for (int e = lane; e < 256; e += 64) blk[e] = in[e] + (ok ? 0.0 : 1.0) * blk[e];
        __syncthreads();
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[0] = (t1 - t0) / reps;
}

int main() {
    // a normalised SPD block like the solve's: unit-ish diagonal, correlated off-diagonals
    std::vector<double> A(256), M(256);
    unsigned long long s = 88172645463325252ull;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (double)(s >> 11) / 9007199254740992.0 - 0.5; };
    for (int i = 0; i < 16; i++)
        for (int k = 0; k < 24; k++) M[i * 16 + (k % 16)] += rnd();
    std::vector<long double> S(256, 0.0L);
    for (int i = 0; i < 16; i++)
        for (int j = 0; j < 16; j++) {
            long double v = (i == j) ? 0.05L : 0.0L;
            for (int k = 0; k < 16; k++) v += (long double)M[i * 16 + k] * M[j * 16 + k];
            S[i * 16 + j] = v;
        }
    for (int i = 0; i < 16; i++)
        for (int j = 0; j < 16; j++) A[((j << 4) + (i ^ (j & 14)))] = (double)S[i * 16 + j];
    // host: L (long double) from the double input, then L^-1
    std::vector<long double> L(256, 0.0L), X(256, 0.0L);
    for (int i = 0; i < 16; i++)
        for (int j = 0; j < 16; j++) S[i * 16 + j] = (long double)A[((j << 4) + (i ^ (j & 14)))];
    for (int j = 0; j < 16; j++) {
        long double d = S[j * 16 + j];
        for (int k = 0; k < j; k++) d -= L[j * 16 + k] * L[j * 16 + k];
        L[j * 16 + j] = sqrtl(d);
        for (int i = j + 1; i < 16; i++) {
            long double v = S[i * 16 + j];
            for (int k = 0; k < j; k++) v -= L[i * 16 + k] * L[j * 16 + k];
            L[i * 16 + j] = v / L[j * 16 + j];
        }
    }
    for (int c = 0; c < 16; c++)
        for (int i = 0; i < 16; i++) {
            long double v = (i == c) ? 1.0L : 0.0L;
            for (int k = 0; k < i; k++) v -= L[i * 16 + k] * X[k * 16 + c];
            X[i * 16 + c] = v / L[i * 16 + i];
        }
    long double xmax = 0;
    for (auto v : X) xmax = fmaxl(xmax, fabsl(v));
    double *din, *dout;
    long long* dc;
    hipMalloc(&din, 256 * 8);
    hipMalloc(&dout, 256 * 8);
    hipMalloc(&dc, 8);
    hipMemcpy(din, A.data(), 256 * 8, hipMemcpyHostToDevice);
    printf("register budget of %d-thread workgroups\n", LB);
    for (int v = 0; v < 11; v++) {
        if (v == 0) hipLaunchKernelGGL(k_diag<0>, dim3(1), dim3(64), 0, 0, din, dout, dc, 64);
        if (v == 1) hipLaunchKernelGGL(k_diag<1>, dim3(1), dim3(64), 0, 0, din, dout, dc, 64);
        if (v == 2) hipLaunchKernelGGL(k_diag<2>, dim3(1), dim3(64), 0, 0, din, dout, dc, 64);
        if (v == 3) hipLaunchKernelGGL(k_diag<3>, dim3(1), dim3(64), 0, 0, din, dout, dc, 64);
        if (v == 4) hipLaunchKernelGGL(k_diag<4>, dim3(1), dim3(64), 0, 0, din, dout, dc, 64);
        if (v == 5) hipLaunchKernelGGL(k_diag<5>, dim3(1), dim3(64), 0, 0, din, dout, dc, 64);
        if (v == 6) hipLaunchKernelGGL(k_diag<6>, dim3(1), dim3(128), 0, 0, din, dout, dc, 64);
        if (v == 7) hipLaunchKernelGGL(k_diag<7>, dim3(1), dim3(64), 0, 0, din, dout, dc, 64);
        if (v == 8) hipLaunchKernelGGL(k_diag<8>, dim3(1), dim3(64), 0, 0, din, dout, dc, 64);
        if (v == 9) hipLaunchKernelGGL(k_diag<9>, dim3(1), dim3(64), 0, 0, din, dout, dc, 64);
        if (v == 10) hipLaunchKernelGGL(k_diag<10>, dim3(1), dim3(64), 0, 0, din, dout, dc, 64);
        std::vector<double> o(256);
        long long c;
        hipMemcpy(o.data(), dout, 256 * 8, hipMemcpyDeviceToHost);
        hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
        long double err = 0;
        for (int i = 0; i < 16; i++)
            for (int j = 0; j < 16; j++) {
                const long double ref = j <= i ? X[i * 16 + j] : 0.0L;
                err = fmaxl(err, fabsl((long double)o[(j << 4) + (i ^ (j & 14))] - ref));
            }
        printf("variant %d: max |X - X_ref| / max|X| = %.3Le, %lld cycles per factor (s_memtime)\n", v,
               err / xmax, c);
    }
    return 0;
}
