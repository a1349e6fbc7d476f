// pint_hip.hip — gfx950 kernels and the C-ABI of libpint_hip.so.
//
// Launch sequence per fit iteration (all instances of a batch in each launch):
//   k_eval      one thread per TOA row: delays, dd phase, design-matrix row, red-noise
//               Fourier columns (HBM-streaming; timing_model.py:1515/1548/2073)
//   k_resid1/2  1024-row blocks of every instance: TZR subtraction, track mode, weighted
//               mean, time residuals, WLS chi2 (residuals.py:314-667) — wave-shuffle
//               reductions, block partials summed in a fixed order
//   k_gram      FP64 MFMA (v_mfma_f64_16x16x4f64) Gram [T|r]^T W [T|r] over TOA chunks
//               staged in LDS, split over N (fitter.py:2187-2192, :1425-1470)
//   k_solve     one workgroup per instance: normalisation, Cholesky in LDS, xhat, inverse
//               (covariance), Woodbury Sigma factor for the GLS chi2 (utils.py:3074)
//   k_apply     parameter update in double-double (fitter.py:957, :2073-2080)
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <string>
#include <vector>
#include <cstring>
#include <cstdio>
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>
#include <type_traits>
#include <mutex>
#include <functional>
#include <chrono>
#include "physics.hpp"

using namespace pint;

typedef double double4_t __attribute__((ext_vector_type(4)));

// e^{i theta} rotation: (c, s) <- (c, s) * (c1, s1)
__device__ __forceinline__ void rot(double& c, double& s, double c1, double s1) {
    const double cn = c * c1 - s * s1;
    s = s * c1 + c * s1;
    c = cn;
}

// a pointer in the global address space (loads through it are global_load, not flat_load)
template <typename T>
using gptr = const T __attribute__((address_space(1)))*;

__device__ __forceinline__ double rdlane(double v, int l) {  // v_readlane of a double, l uniform
    long long b = __double_as_longlong(v);
    int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
    int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// ---------------------------------------------------------------------------------
// device-side descriptors
// ---------------------------------------------------------------------------------
struct PsrDev {
    const double *tdb_hi, *tdb_lo, *freq, *sigma, *isig, *pos, *vel, *sun, *pn, *dpn;
    const double* planet;    // (n+1) x 15 observatory -> planet vectors (spec shapiro == 2), else null
    const uint32_t* flags;
    const uint64_t* jmask;
    const int32_t *dmx_a, *dmx_b;
    const int32_t* dmx_x;    // bins beyond the first two: n+2 offsets, then indices (null: none)
    const pint_spec_t* spec;
    const double* red_freq;  // 2 nred: the frequencies as double-double, hi[nred] then lo[nred]
    const double* red_phi;   // 2*nred
    const double* red_cs;    // n x 4: (cos, sin) of theta and of 8 theta, theta = 2 pi t f_1 (k_trig_setup)
    const double* trigU;     // 2 x 64: U_m = sum_i cos m theta_i, V_m = sum_i sin m theta_i (k_trig_setup)
    const double* trigW;     // 2 x 64: C_m, S_m = sum_i w_i (cos, sin) m theta_i, w = 1/sigma^2 (k_trig_setup):
                             // TOA-only at fixed sigma, formed at upload and by pint_set_sigma
    const int32_t* ep_ptr;   // ECORR epochs, CSR (nep+1)
    const int32_t* ep_idx;
    const double* ep_phi;    // nep prior variances (s^2)
    const int32_t* toa_ep;   // n: the ECORR epoch of each TOA (-1: none)
    // compact layout with ECORR: every epoch's TOAs lie in at most one DMX column, so the
    // epoch block couples to one bin and its elimination keeps the DMX block diagonal
    const int32_t* ep_bin;   // nep: the DMX column of each epoch's TOAs (-1: none)
    const int32_t* bep_ptr;  // ndc+1: CSR of the epochs of each DMX column
    const int32_t* bep_idx;
    // white-noise classes for noise-parameter fits (pint_set_noise_classes): TOAs grouped by
    // the set of EFAC/EQUAD masks selecting them, CSR; raw TOA errors (us)
    const int32_t *cls_ptr, *cls_idx, *toa_cls;
    const double* sigma0;
    // wideband DM data (pint_set_wideband): measured DMs, raw and scaled errors, DMJUMP masks
    const double *pp_dm, *pp_dme, *dm_sig;
    const uint64_t* dmjmask;
    int wb;
    int ncls;
    int ep_overlap;          // some TOA lies in two ECORR epochs (no per-epoch Sherman-Morrison)
    const ColRun* runs;      // design-matrix column runs
    int nrun;
    // sparse-DMX fit layout: the DMX columns (one nonzero value per TOA, in its bin) are
    // kept out of M and out of the dense Gram; their Gram rows are bin sums (k_dmx)
    const int32_t* cmap;     // K+1: compact column (>= 0) or -(a+1) for DMX column a
    const int32_t* dptr;     // ndc+1: CSR of the TOAs of each DMX column
    const int32_t* didx;
    const int32_t* drow;     // n: DMX column of each TOA (-1: none)
    const int32_t* dslot;    // n: its k_gram_v slot, drow % vns (-1: none); vg pulsars only
    const int32_t* dorig;    // Kd: original column of each compact dense column
    const int32_t* xorig;    // ndc: original column of each DMX column
    int dsplit;              // compact layout applies (>= 8 DMX columns, no overlapping bins, every ECORR
                             // epoch within one DMX column)
    int dcontig;             // every DMX column's TOAs are one contiguous row range (k_gram fuses the bin sums)
    int ndc, Kd, Kpd, red0c; // DMX columns; compact width (excl. residual), padded, first red column
    int n;
    int K;   // ncol + 2*nred
    int Kp;  // padded K+1 (residual column) to 16
    int nep; // ECORR epochs (eliminated by Schur complement)
    int vg;  // compact fit layout on the k_gram_v path (DMX slots as MFMA rows, F^T W F from trig sums)
    int vns; // k_gram_v DMX slots (bins of an N-split are distinct mod vns)
    int vkp; // k_gram_v LDS width: [T | r | slots | F] padded to 16
    int vb;  // k_gram_v binned DMX x Fourier tile (VB) for this pulsar
    double logsig;  // sum_i log sigma_i (s): the WLS likelihood normalisation (residuals.py:665)
    double sumw;    // sum_i 1/sigma_i^2 (s^-2)
};

struct InstDev {
    int psr;
    int n;
    int K;
    int Kp;
    long toff;   // table offset (doubles)
    long roff;   // eval-row offset (n+1 rows)
    long moff;   // design-matrix offset (n*K)
    long goff;   // Gram offset (Kp*Kp per split)
    long soff;   // solve outputs offset (K*K)
    long coff;   // per-instance K vectors offset
    long cvoff;  // compact timing covariance offset (ncol*ncol)
    long eoff;   // ECORR epoch sums offset (nep*Kp) and per-epoch scalars (eoff/Kp)
    long epoff;  // per-epoch scalar offset (nep)
    long ooff;   // residual output offset (n per instance)
    long sdoff;  // DMX cross-sum offset (ndc*Kpd) / per-column sums offset (ndc)
    long ddoff;
    long vgoff;  // k_gram_v DMX slot partials offset (nsplit * vns * (Kd+3))
    long vboff;  // k_gram_v binned DMX x Fourier partials offset (nsplit * GW * vns * 128)
    long xwoff;  // k_solve_dmx -> k_cov_dmx export offset (X, U blocks and the scalings)
    int self;    // index of this instance in the batch
    int nrb;     // k_resid row blocks of this instance (RES_RB rows each)
    long rb0;    // first k_resid row block
    int neb;     // evaluation blocks with the fused residual pass (EF_ROWS rows each; 0: not fused)
    long eb0;    // their first weighted-sum partial (d_epart, 2 per block)
    // the pulsar's model structure and column runs (copies of its PsrDev fields: the evaluation
    // blocks' LDS staging starts from the instance record, two dependent loads sooner)
    const pint_spec_t* spec;
    const ColRun* runs;
    int ts;            // spec->tstride
    int nrun;
};

// Symmetric view of an instance's Gram [T|r]^T W [T|r] in the original column order:
// full layout (cmap == nullptr), or the compact layout's dense Gram plus the DMX bin sums.
struct GramView {
    const double* Gp;
    int Kp;
    const int32_t* cmap;
    const double* Sd;  // ndc x Kp: sum_{i in bin a} w_i x_i [T|r]_i (compact columns)
    const double* DD;  // ndc: sum_{i in bin a} w_i x_i^2
    __device__ __forceinline__ double operator()(int i, int j) const {
        if (!cmap) {
            if (i > j) { int t = i; i = j; j = t; }
            return Gp[(long)i * Kp + j];
        }
        int a = cmap[i], b = cmap[j];
        if (a >= 0 && b >= 0) {
            if (a > b) { int t = a; a = b; b = t; }
            return Gp[(long)a * Kp + b];
        }
        if (a < 0 && b < 0) return a == b ? DD[-a - 1] : 0.0;
        if (a < 0) return Sd[(long)(-a - 1) * Kp + b];
        return Sd[(long)(-b - 1) * Kp + a];
    }
};

__device__ __forceinline__ GramView gram_view(const PsrDev& Pd, const InstDev& I, const double* Gpart, bool cmp,
                                              const double* Sd, const double* DD) {
    GramView g;
    g.Gp = Gpart + I.goff;
    g.Kp = cmp ? Pd.Kpd : I.Kp;
    g.cmap = cmp ? Pd.cmap : nullptr;
    g.Sd = Sd + I.sdoff;
    g.DD = DD + I.ddoff;
    return g;
}
// unweighted column sum of squares (normalize_designmatrix) in the original order
__device__ __forceinline__ double colsq_of(const PsrDev& Pd, const InstDev& I, const double* colsq, int nsplit,
                                           bool cmp, const double* DCS, int j) {
    if (!cmp) return colsq[(I.coff + j) * nsplit];
    int a = Pd.cmap[j];
    return a >= 0 ? colsq[(I.coff + a) * nsplit] : DCS[I.ddoff - a - 1];
}

struct KpGroup {  // instances sharing k_gram's tiles-per-wave T (launched together)
    int T, first, count, maxKp;
};

#define HIPCHK(x)                                                                    \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            ctx->err = std::string(#x) + ": " + hipGetErrorString(e_);               \
            return PINT_E_HIP;                                                       \
        }                                                                            \
    } while (0)

// ---------------------------------------------------------------------------------
// Per-workgroup timeline of the fit step's kernels (diagnostic: pint_debug_read 7 reads it,
// 8 switches it on or off and clears it; scripts/diag/wg_timeline.py): workgroup b of
// kernel k stores its first stamp (s_memrealtime, 100 MHz) from thread 0, and every wave
// raises its exit stamp with an atomic max when it leaves.  Off: one scalar flag load per
// workgroup.
// ---------------------------------------------------------------------------------
constexpr int WGT_K = 12, WGT_B = 2048;
enum { WGT_EVAL = 0, WGT_GRAMV, WGT_GRED, WGT_SCHUR, WGT_SOLVE, WGT_RES1, WGT_RES2, WGT_WSOLVE, WGT_COV, WGT_NOISE,
       WGT_EXPORT, WGT_OTHER };
__device__ int g_wgt_on;
__device__ unsigned long long g_wgt[WGT_K * WGT_B * 2];
// evaluation blocks' phase stamps (pint_debug_read 9): end of the LDS staging prologue
// (thread 0), end of the rows' evaluation (atomic max over the waves)
__device__ unsigned long long g_wgp[WGT_B * 2];
__device__ __forceinline__ void wgp_stamp(int which, bool first_only) {
    const int b = blockIdx.x;
    if (!__builtin_amdgcn_readfirstlane(g_wgt_on) || b >= WGT_B) return;
    if (first_only ? threadIdx.x == 0 : (threadIdx.x & 63) == 0)
        atomicMax(&g_wgp[2 * b + which], __builtin_amdgcn_s_memrealtime());
}
struct WgTimer {
    int slot;  // (k * WGT_B + b) * 2, or -1 when off / beyond WGT_B
    __device__ __forceinline__ explicit WgTimer(int k) {
        const int b = blockIdx.y * gridDim.x + blockIdx.x;
        slot = (__builtin_amdgcn_readfirstlane(g_wgt_on) && b < WGT_B) ? (k * WGT_B + b) * 2 : -1;
        if (slot >= 0 && threadIdx.x == 0) g_wgt[slot] = __builtin_amdgcn_s_memrealtime();
    }
    __device__ __forceinline__ ~WgTimer() {
        if (slot >= 0 && (threadIdx.x & 63) == 0) atomicMax(&g_wgt[slot + 1], __builtin_amdgcn_s_memrealtime());
    }
};

// ---------------------------------------------------------------------------------
// wave / block reductions (64-wide waves)
// ---------------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// a workgroup barrier, or with NW == 1 (one wave per instance, several instances per
// workgroup) the wave's own: its LDS writes visible to its other lanes, no cross-wave wait
template <int NW>
__device__ __forceinline__ void bsync() {
    if constexpr (NW == 1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
}
template <int NW>
__device__ double block_sum(double v, double* sh) {
    v = wave_sum(v);
    if constexpr (NW == 1) return 0.0 + v;  // (the NW-wave form's order with one wave)
    int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) sh[w] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < NW; i++) t += sh[i];
    return t;
}
// block_sum of V values at once (one barrier pair; each value reduced in block_sum's order,
// so the same bits); sh holds V * NW doubles
template <int NW, int V>
__device__ void block_sums(double* v, double* sh) {
#pragma unroll
    for (int k = 0; k < V; k++) v[k] = wave_sum(v[k]);
    if constexpr (NW == 1) {  // (the NW-wave form's order with one wave)
#pragma unroll
        for (int k = 0; k < V; k++) v[k] = 0.0 + v[k];
        return;
    }
    int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) {
#pragma unroll
        for (int k = 0; k < V; k++) sh[k * NW + w] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < V; k++) {
        double t = 0.0;
#pragma unroll
        for (int i = 0; i < NW; i++) t += sh[k * NW + i];
        v[k] = t;
    }
}

// dst[e] = src[e], e < n, by NT threads, U loads per thread in flight before their stores:
// a copy loop of one load per iteration waits on each load in turn (a 100 KB LDS stage of
// the solve took ~5 us that way)
template <int NT, int U, typename D>
__device__ __forceinline__ void copy_in(D* __restrict__ dst, const double* __restrict__ src, int n, int tid) {
    for (int base = 0; base < n; base += NT * U) {
        double t[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int e = base + tid + u * NT;
            t[u] = e < n ? src[e] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int e = base + tid + u * NT;
            if (e < n) dst[e] = t[u];
        }
    }
}

// ---------------------------------------------------------------------------------
// k_eval: one thread per TOA row (row n = TZR TOA)
// ---------------------------------------------------------------------------------
// k_prep: per-instance constants of the evaluation (astrometry/starpm state, 1/F0), one
// thread per instance, so k_eval's threads only do per-TOA work.
// The setup is one thread's serial code over a dozen parameters; its global loads would be
// a chain of dependent round trips, so the block first stages the spec header (everything
// before the column arrays, all that inst_setup reads) and the table in LDS, coalesced.
constexpr int PREP_T = 64;
constexpr int PREP_MAXTAB = 1024;  // doubles of a staged table (larger ones read in place)
constexpr int PREP_HDR = (int)(offsetof(pint_spec_t, col_kind) + 7) / 8;  // spec header, doubles
__device__ __forceinline__ void prep_one(const pint_spec_t* Sg, const double* Pg, int tstride, InstConst* out) {
    __shared__ double sS[PREP_HDR];
    __shared__ double sP[PREP_MAXTAB];
    const double* hg = reinterpret_cast<const double*>(Sg);
    for (int i = threadIdx.x; i < PREP_HDR; i += blockDim.x) sS[i] = hg[i];
    const bool staged = tstride <= PREP_MAXTAB;
    if (staged)
        for (int i = threadIdx.x; i < tstride; i += blockDim.x) sP[i] = Pg[i];
    __syncthreads();
    // the wave's lanes share the independent transcendental calls (inst_setup_wave)
    __shared__ double sx[16];
    __shared__ InstConst sC;
    inst_setup_wave(*reinterpret_cast<const pint_spec_t*>(sS), staged ? sP : Pg, sC, sx, threadIdx.x);
    __syncthreads();
    if (threadIdx.x == 0) *out = sC;
}

// k_prep / k_apply, lane per instance (PREP_LANES: batches whose tables all fit
// PREP_LANE_TAB doubles, i.e. grid points of a small model): every thread sets up its own
// instance with inst_setup_seq (inst_setup_wave's operations in one thread: the same values),
// 64 instances per wave instead of one instance's serial code on one lane of a wave
constexpr int PREP_LANE_TAB = 64;
__global__ __launch_bounds__(64) void k_prep_lanes(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                   int ninst, double* __restrict__ tables,
                                                   const double* __restrict__ tables0, InstConst* __restrict__ ic) {
    const int q = blockIdx.x * 64 + threadIdx.x;
    if (q >= ninst) return;
    const InstDev I = insts[q];
    const pint_spec_t& S = *psrs[I.psr].spec;
    const double* P = tables + I.toff;
    if (tables0) {
        const int ts = S.tstride;
        for (int i = 0; i < ts; i++) tables[I.toff + i] = tables0[I.toff + i];
        P = tables0 + I.toff;
    }
    InstConst C;
    inst_setup_seq(S, P, C);
    ic[q] = C;
}
__global__ __launch_bounds__(64) void k_apply_lanes(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                    int ninst, double* __restrict__ tables,
                                                    const double* __restrict__ dpars, const double* __restrict__ lam,
                                                    InstConst* __restrict__ ic, double lam_u) {
    const int q = blockIdx.x * 64 + threadIdx.x;
    if (q >= ninst) return;
    const InstDev I = insts[q];
    const pint_spec_t& S = *psrs[I.psr].spec;
    double* P = tables + I.toff;
    const double li = lam ? lam[q] : lam_u;
    if (li != 0.0) {  // (decided instances: a non-finite step must not touch them)
        for (int c = 0; c < S.ncol; c++) {
            const int o = S.col_toff[c];
            if (o < 0) continue;
            const dd v = dd_add_d(dd_make(P[o], P[o + 1]), li * dpars[I.coff + c]);
            P[o] = v.hi;
            P[o + 1] = v.lo;
        }
    }
    InstConst C;
    inst_setup_seq(S, P, C);
    ic[q] = C;
}

// k_prep: the per-instance constants of the tables; with tables0 (pint_restore_tables
// pending) the instance's table is first put back from the device snapshot, in the same
// launch (the constants are formed from the snapshot, which is what the table then holds)
__global__ __launch_bounds__(PREP_T) void k_prep(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                 double* __restrict__ tables, const double* __restrict__ tables0,
                                                 InstConst* __restrict__ ic) {
    const InstDev I = insts[blockIdx.x];
    const PsrDev& Pd = psrs[I.psr];
    const int ts = Pd.spec->tstride;
    if (tables0) {
        for (int i = threadIdx.x; i < ts; i += PREP_T) tables[I.toff + i] = tables0[I.toff + i];
        prep_one(Pd.spec, tables0 + I.toff, ts, ic + blockIdx.x);
        return;
    }
    prep_one(Pd.spec, tables + I.toff, ts, ic + blockIdx.x);
}

constexpr int EVAL_MAXTAB = 512;  // doubles of a parameter table staged in LDS (larger ones read in place)
constexpr int EVAL_MAXRUN = 64;   // column runs staged in LDS
struct alignas(16) EvalLds {  // (16-byte aligned: the staging stores 16-byte words)
    pint_spec_t S;
    InstConst C;
    ColRun R[EVAL_MAXRUN];
    double P[EVAL_MAXTAB];
    double X[4];    // fused residual pass: the TZR row's and row 0's phase (hi, lo)
    double red[8];  // fused residual pass: block_sums<4, 2>
};
// The residual pass's first half (k_resid1) fused into the evaluation (EvalRestore::epart):
// each 256-thread block evaluates EF_ROWS rows of its instance plus, on its last two lanes,
// row 0 and the TZR row (row n) -- 2 of 256 lanes of extra work -- so it forms its rows'
// phase residuals and their weighted sums itself instead of a k_resid1 launch after the
// evaluation (k_resid1's operations per row; the sums per block of EF_ROWS rows).
constexpr int EF_ROWS = 254;

// restore targets of an evaluation that reads the parameter snapshot (pint_restore_tables): the
// first block of each instance writes the snapshot's table and constants back (k_prep's work
// on the restore path, without its launch); null otherwise
struct EvalRestore {
    double* tables;
    InstConst* ic;
    double* rph;    // fused residual pass (null: k_resid1 follows): phase residuals (output rows)
    double* epart;  // ... and the blocks' (sum w, sum w x) partials
};

// the TOA inputs of row r (row n: the TZR TOA)
__device__ __forceinline__ void load_toa_row(const PsrDev& Pd, const pint_spec_t& S, unsigned r, ToaRow& t) {
    t.tdb = dd_make(Pd.tdb_hi[r], Pd.tdb_lo[r]);
    t.freq = Pd.freq[r];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        t.pos[k] = Pd.pos[3 * r + k];
        t.vel[k] = Pd.vel[3 * r + k];
        t.sun[k] = Pd.sun[3 * r + k];
    }
    t.planet = S.shapiro == 2 ? Pd.planet + 15 * r : nullptr;
    t.flags = Pd.flags[r];
    t.jmask = Pd.jmask[r];
    t.dmx_a = Pd.dmx_a[r];
    t.dmx_b = Pd.dmx_b[r];
    t.dmx_x = Pd.dmx_x;
    t.dmx_x0 = Pd.dmx_x ? Pd.dmx_x[r] : 0;
    t.dmx_x1 = Pd.dmx_x ? Pd.dmx_x[r + 1] : 0;
}

// one row of eval_block: the row's evaluation and its outputs (own: this lane writes them)
template <int WANT_M, int BIN>
__device__ __forceinline__ void eval_row(const pint_spec_t& S, EvalLds& L, const PsrDev& Pd, const InstDev& I, bool stP,
                                         bool stR, int nrun, const double* __restrict__ tables, unsigned r, int n,
                                         bool own, double* __restrict__ Mout, double* __restrict__ dmxv, int compact,
                                         int write_red, int* __restrict__ status, int* __restrict__ istatus, int ii,
                                         double* __restrict__ ph_hi, double* __restrict__ ph_lo,
                                         double* __restrict__ ftay, double* __restrict__ delay_out,
                                         double* __restrict__ dfac, EvalOut& o) {
    const double* P = stP ? L.P : tables + I.toff;
    ToaRow t;
    load_toa_row(Pd, S, r, t);
    double* Mb = WANT_M ? (Mout + I.moff) : nullptr;  // wave-uniform column base
    const bool rowM = WANT_M && own && r < (unsigned)n;
    const bool cmp = WANT_M && compact && Pd.dsplit;
    eval_toa<BIN>(S, P, L.C, t, o, rowM ? Mb : nullptr, r, n, stR ? L.R : Pd.runs, nrun, cmp);
    if (!own) return;
    if (rowM && cmp) dmxv[I.ooff + r] = o.dmc;
    if (o.status) {  // the batch's status word and this instance's own (pint_inst_status)
        atomicOr(status, 1 << o.status);
        atomicOr(istatus + ii, 1 << o.status);
    }
    ph_hi[I.roff + r] = o.phase.hi;
    ph_lo[I.roff + r] = o.phase.lo;
    ftay[I.roff + r] = o.ftaylor;
    delay_out[I.roff + r] = o.delay;
    const bool dmn = S.dmn0 < S.nred;  // PLDMNoise modes: rescaled per TOA, rewritten every time
    const double Dfac = 1400.0 * 1400.0 * o.inv_f2;
    if (WANT_M && rowM && dmn) dfac[I.ooff + r] = Dfac;
    if (WANT_M && rowM && S.nred > 0 && (write_red || dmn) && !(cmp && Pd.vg)) {  // vg: generated where used
        // PLRedNoise Fourier basis (noise_model.py:861-880): F[:,2k]=sin(2pi t f_k),
        // F[:,2k+1]=cos(...), t = tdbld*86400 s.  Argument reduced exactly in dd.  The basis
        // does not depend on the timing parameters: it is written once per instance and
        // layout (write_red) and stays resident in M across fit iterations.
        dd ts = dd_mul_d(t.tdb, DAYSEC);
        double* colp = Mb + (long)(cmp ? Pd.red0c : S.ncol) * n;
        for (int k = write_red ? 0 : S.dmn0; k < S.nred; k++) {
            dd x = dd_mul(ts, dd_make(Pd.red_freq[k], Pd.red_freq[S.nred + k]));
            double fr = dd_to_d(dd_sub(x, dd_floor(x)));
            double sn, cs;
            sincos(TWO_PI * fr, &sn, &cs);
            const double sc = k >= S.dmn0 ? Dfac : 1.0;
            colp[2L * k * n + r] = sn * sc;
            colp[2L * k * n + r + n] = cs * sc;
        }
    }
}

template <int WANT_M, int BIN>
__device__ __forceinline__ void eval_block(int b, const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                           const int* __restrict__ blk_inst, const int* __restrict__ blk_row0,
                                           const double* __restrict__ tables, const InstConst* __restrict__ ic,
                                           double* __restrict__ ph_hi, double* __restrict__ ph_lo,
                                           double* __restrict__ ftay, double* __restrict__ delay_out,
                                           double* __restrict__ Mout, double* __restrict__ dmxv, int compact,
                                           int write_red, int* __restrict__ status, int* __restrict__ istatus,
                                           double* __restrict__ dfac, EvalLds& L, EvalRestore rs) {
    int ii = blk_inst[b];
    const InstDev I = insts[ii];
    const PsrDev& Pd = psrs[I.psr];
    // the block's instance -- model structure, parameter table, per-instance constants and
    // column runs -- staged in LDS: every row reads them, and an LDS read returns in a
    // fraction of a global (cache) load's latency and needs no address registers
    const int ts = I.ts, nrun = I.nrun;
    const bool stP = ts <= EVAL_MAXTAB, stR = nrun <= EVAL_MAXRUN;
    {
        // every load of the staging issued before any LDS store, in 16-byte words: one load
        // latency per block instead of one per strided round (the 4 KB spec alone took five
        // dependent rounds of 4-byte loads and stores, ~2 us of a block's 14-23 us)
        static_assert(sizeof(pint_spec_t) % 16 == 0 && sizeof(InstConst) % 16 == 0 && sizeof(ColRun) % 16 == 0,
                      "eval staging: 16-byte words");
        constexpr int NS = (int)(sizeof(pint_spec_t) / 16), NC = (int)(sizeof(InstConst) / 16);
        constexpr int RW = (int)(sizeof(ColRun) / 16);
        static_assert(NS <= 512 && NC + EVAL_MAXRUN * RW <= 256 && EVAL_MAXTAB <= 512, "eval staging: two rounds of 256");
        const int t = threadIdx.x;  // (256 threads: every eval_block launch)
        const int NR = stR ? nrun * RW : 0;
        const uint4* sg = reinterpret_cast<const uint4*>(I.spec);
        const uint4* cg = reinterpret_cast<const uint4*>(ic + ii);
        const uint4* rg = reinterpret_cast<const uint4*>(I.runs);
        const double* pg = tables + I.toff;
        const bool hs0 = t < NS, hs1 = t + 256 < NS, hc = t < NC, hr = !hc && t < NC + NR;
        const bool hp0 = stP && t < ts, hp1 = stP && t + 256 < ts;
        uint4 s0 = {}, s1 = {}, cr = {};
        double p0 = 0.0, p1 = 0.0;
        if (hs0) s0 = sg[t];
        if (hs1) s1 = sg[t + 256];
        if (hc) cr = cg[t];
        else if (hr) cr = rg[t - NC];
        if (hp0) p0 = pg[t];
        if (hp1) p1 = pg[t + 256];
        uint4* sd = reinterpret_cast<uint4*>(&L.S);
        if (hs0) sd[t] = s0;
        if (hs1) sd[t + 256] = s1;
        if (hc) reinterpret_cast<uint4*>(&L.C)[t] = cr;
        else if (hr) reinterpret_cast<uint4*>(L.R)[t - NC] = cr;
        if (hp0) L.P[t] = p0;
        if (hp1) L.P[t + 256] = p1;
    }
    __syncthreads();
    wgp_stamp(0, true);
    if (rs.tables && blk_row0[b] == 0) {  // the instance's first block puts the snapshot back
        for (int k = threadIdx.x; k < ts; k += blockDim.x) rs.tables[I.toff + k] = stP ? L.P[k] : tables[I.toff + k];
        const int* cs = reinterpret_cast<const int*>(&L.C);
        int* cd = reinterpret_cast<int*>(rs.ic + ii);
        for (int k = threadIdx.x; k < (int)(sizeof(InstConst) / 4); k += blockDim.x) cd[k] = cs[k];
    }
    const pint_spec_t& S = L.S;
    const int n = I.n;
    const bool ef = rs.epart != nullptr;  // (launch-uniform) the fused residual pass
    const int lt = threadIdx.x;
    unsigned r;
    bool own;  // the row's outputs are this lane's to write
    if (ef) {
        r = lt < EF_ROWS ? (unsigned)(blk_row0[b] + lt) : (lt == EF_ROWS ? 0u : (unsigned)n);
        own = lt < EF_ROWS ? r < (unsigned)n : (lt == EF_ROWS + 1 && blk_row0[b] == 0);
        if (lt < EF_ROWS && r >= (unsigned)n) r = 0;  // (an idle lane of the last block: evaluates row 0, writes nothing)
    } else {
        r = (unsigned)(blk_row0[b] + lt);
        own = r <= (unsigned)n;
        if (!own) return;
    }
    EvalOut o;
    eval_row<WANT_M, BIN>(S, L, Pd, I, stP, stR, nrun, tables, r, n, own, Mout, dmxv, compact, write_red, status, istatus,
                          ii, ph_hi, ph_lo, ftay, delay_out, dfac, o);
    wgp_stamp(1, false);
    if (!ef) return;
    // ---- the fused k_resid1 (residuals.py:314-425): tz and d0 from the block's own TZR and
    //      row-0 lanes, then k_resid1's per-row operations and the block's weighted sums ----
    if (lt == EF_ROWS) {
        L.X[2] = o.phase.hi;
        L.X[3] = o.phase.lo;
    } else if (lt == EF_ROWS + 1) {
        L.X[0] = o.phase.hi;
        L.X[1] = o.phase.lo;
    }
    __syncthreads();
    const dd tz = dd_make(L.X[0], L.X[1]);
    dd d0 = dd_make(0.0);
    if (!S.track_pn && S.subtract_mean) d0 = dd_add_d(dd_sub(dd_make(L.X[2], L.X[3]), tz), Pd.dpn[0]);
    double sw = 0.0, swx = 0.0;
    if (lt < EF_ROWS && own) {
        const dd d = dd_add_d(dd_sub(dd_make(o.phase.hi, o.phase.lo), tz), Pd.dpn[r]);
        double full;
        if (S.track_pn) {
            full = dd_to_d(dd_add_d(d, -Pd.pn[r]));
        } else {
            const dd x = dd_sub(d, d0);
            full = dd_to_d(dd_sub(x, dd_round_half_up(x)));
        }
        rs.rph[I.roff - ii + r] = full;
        const double lw = Pd.isig[r];
        const double w = S.weighted_mean ? lw * lw : 1.0;
        sw += w;
        swx += w * full;
    }
    if (S.subtract_mean) {
        double v[2] = {swx, sw};
        block_sums<4, 2>(v, L.red);
        if (lt == 0) {
            const long eb = I.eb0 + blk_row0[b] / EF_ROWS;
            rs.epart[2 * eb] = v[1];
            rs.epart[2 * eb + 1] = v[0];
        }
    }
}

// Spin-only grids (pint_set_grid's variables all spin frequencies, isolated model, no
// red-noise basis, the full layout): before the first fit step every point shares its
// delays, astrometric geometry and dispersion factors (they depend on the TOAs and the
// non-spin parameters only), so k_eval_head evaluates them once, on the batch's first
// point, with eval_toa's own operations (eval_pre), and k_eval_spin gives each point only
// eval_toa's spin part (eval_spin_a/b: spin phase and frequencies, the chain factor, the
// design-matrix row).  The same operations on the same values as the full evaluation of
// each point: the same bits (test_spin_grid_eval_matches_full).
__global__ __launch_bounds__(256) void k_eval_head(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                   const double* __restrict__ tables, const InstConst* __restrict__ ic,
                                                   double* __restrict__ shr) {
    const InstDev I = insts[0];
    const PsrDev& Pd = psrs[I.psr];
    const pint_spec_t& S = *Pd.spec;
    const unsigned r = blockIdx.x * 256 + threadIdx.x;
    if (r > (unsigned)I.n) return;
    ToaRow t;
    load_toa_row(Pd, S, r, t);
    EvalHead h;
    eval_head(S, tables + I.toff, ic[0], t, h);
    double* o = shr + (long)r * EVAL_HEAD_W;
    o[0] = h.delay;
    o[1] = h.gLON;
    o[2] = h.gLAT;
    o[3] = h.gPMLON;
    o[4] = h.gPMLAT;
    o[5] = h.gPX;
    o[6] = h.inv_f2;
    o[7] = h.dt_yr_dm;
    o[8] = h.logf;
}

// a wave per point, lanes over its rows
__global__ __launch_bounds__(256) void k_eval_spin(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                   int ninst, const double* __restrict__ tables,
                                                   const InstConst* __restrict__ ic, const double* __restrict__ shr,
                                                   double* __restrict__ ph_hi, double* __restrict__ ph_lo,
                                                   double* __restrict__ ftay, double* __restrict__ delay_out,
                                                   double* __restrict__ Mout) {
    const int ii = blockIdx.x * 4 + (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (ii >= ninst) return;  // (wave-uniform)
    const InstDev I = insts[ii];
    const PsrDev& Pd = psrs[I.psr];
    const pint_spec_t& S = *Pd.spec;
    const InstConst C = ic[ii];
    const double* P = tables + I.toff;
    const int n = I.n;
    double* Mb = Mout + I.moff;
    for (int r = threadIdx.x & 63; r <= n; r += 64) {
        ToaRow t;
        t.tdb = dd_make(Pd.tdb_hi[r], Pd.tdb_lo[r]);
        t.jmask = Pd.jmask[r];
        t.dmx_a = Pd.dmx_a[r];
        t.dmx_b = Pd.dmx_b[r];
        t.dmx_x = Pd.dmx_x;
        t.dmx_x0 = Pd.dmx_x ? Pd.dmx_x[r] : 0;
        t.dmx_x1 = Pd.dmx_x ? Pd.dmx_x[r + 1] : 0;
        const double* q = shr + (long)r * EVAL_HEAD_W;
        const EvalHead h = {q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7], q[8]};
        EvalOut o;
        o.status = 0;
        o.dmc = 0.0;
        o.inv_f2 = h.inv_f2;
        EvalSpin sp;
        eval_spin_a(S, P, C, t, h.delay, o, sp);
        eval_spin_b<0>(S, P, C, t, h, sp, o, r < n ? Mb : nullptr, (unsigned)r, n, Pd.runs, Pd.nrun, false);
        ph_hi[I.roff + r] = o.phase.hi;
        ph_lo[I.roff + r] = o.phase.lo;
        ftay[I.roff + r] = o.ftaylor;
        delay_out[I.roff + r] = o.delay;
    }
}

// k_eval: one thread per TOA row; one launch per binary model (blocks of the isolated,
// ELL1 or DD instances), so each instantiation carries only its own registers.
template <int WANT_M, int BIN, int W = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W > 0 ? W : 1, W > 0 ? W : 10)))
void k_eval(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                              const int* __restrict__ blk_inst, const int* __restrict__ blk_row0,
                                              const double* __restrict__ tables, const InstConst* __restrict__ ic,
                                              double* __restrict__ ph_hi, double* __restrict__ ph_lo,
                                              double* __restrict__ ftay, double* __restrict__ delay_out,
                                              double* __restrict__ Mout, double* __restrict__ dmxv, int compact,
                                              int write_red, int* __restrict__ status, int* __restrict__ istatus,
                                              double* __restrict__ dfac, EvalRestore rs) {
    __shared__ EvalLds L;
    eval_block<WANT_M, BIN>(blockIdx.x, psrs, insts, blk_inst, blk_row0, tables, ic, ph_hi, ph_lo, ftay, delay_out,
                            Mout, dmxv, compact, write_red, status, istatus, dfac, L, rs);
}

// k_eval_mix: all binary models in one launch (heaviest first: DD, ELL1, isolated blocks),
// each block running its own instantiation; the kernel carries the largest register set,
// and saves the two launch tails of the per-model launches.
template <int WANT_M>
__device__ __forceinline__ void eval_mix_body(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                  const int* __restrict__ blk_inst, const int* __restrict__ blk_row0,
                                                  int off1, int off2, int off3,
                                                  const double* __restrict__ tables, const InstConst* __restrict__ ic,
                                                  double* __restrict__ ph_hi, double* __restrict__ ph_lo,
                                                  double* __restrict__ ftay, double* __restrict__ delay_out,
                                                  double* __restrict__ Mout, double* __restrict__ dmxv, int compact,
                                                  int write_red, int* __restrict__ status, int* __restrict__ istatus,
                                                  double* __restrict__ dfac, EvalRestore rs) {
    const int n2 = off3 - off2, n1 = off2 - off1;
    const int b = blockIdx.x;
    __shared__ EvalLds L;
    if (b < n2)
        eval_block<WANT_M, 2>(off2 + b, psrs, insts, blk_inst, blk_row0, tables, ic, ph_hi, ph_lo, ftay, delay_out,
                              Mout, dmxv, compact, write_red, status, istatus, dfac, L, rs);
    else if (b < n2 + n1)
        eval_block<WANT_M, 1>(off1 + b - n2, psrs, insts, blk_inst, blk_row0, tables, ic, ph_hi, ph_lo, ftay,
                              delay_out, Mout, dmxv, compact, write_red, status, istatus, dfac, L, rs);
    else
        eval_block<WANT_M, 0>(b - n2 - n1, psrs, insts, blk_inst, blk_row0, tables, ic, ph_hi, ph_lo, ftay, delay_out,
                              Mout, dmxv, compact, write_red, status, istatus, dfac, L, rs);
}
#define PINT_EVAL_MIX_ARGS                                                                                      \
    const PsrDev *__restrict__ psrs, const InstDev *__restrict__ insts, const int *__restrict__ blk_inst,        \
        const int *__restrict__ blk_row0, int off1, int off2, int off3, const double *__restrict__ tables,      \
        const InstConst *__restrict__ ic, double *__restrict__ ph_hi, double *__restrict__ ph_lo,               \
        double *__restrict__ ftay, double *__restrict__ delay_out, double *__restrict__ Mout,                   \
        double *__restrict__ dmxv, int compact, int write_red, int *__restrict__ status,                        \
        int *__restrict__ istatus, double *__restrict__ dfac, EvalRestore rs
#define PINT_EVAL_MIX_PASS                                                                                      \
    psrs, insts, blk_inst, blk_row0, off1, off2, off3, tables, ic, ph_hi, ph_lo, ftay, delay_out, Mout, dmxv,  \
        compact, write_red, status, istatus, dfac, rs
template <int WANT_M>
__global__ __launch_bounds__(256) void k_eval_mix(PINT_EVAL_MIX_ARGS) {
    WgTimer wgt_(WGT_EVAL);
    eval_mix_body<WANT_M>(PINT_EVAL_MIX_PASS);
}
// the same with the register budget of W resident waves per SIMD: the evaluation with the
// design matrix is latency-bound (dependent FP64 / double-double chains, ~40 cycles each),
// so a third wave per SIMD hides more than its 108 B of spills cost (PINT_EVAL_WPE)
template <int WANT_M, int W>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, W))) void k_eval_mix_w(PINT_EVAL_MIX_ARGS) {
    WgTimer wgt_(WGT_EVAL);
    eval_mix_body<WANT_M>(PINT_EVAL_MIX_PASS);
}

// ---------------------------------------------------------------------------------
// k_resid1/k_resid2 — residuals.py:314-425, :483-538, :638-667
// ---------------------------------------------------------------------------------
// The residual pass split over RES_RB-row blocks of every instance,
// so a batch of a few large pulsars still fills the CUs.  k_resid1 forms the phase
// residuals and each block's weighted sums; k_resid2 sums the instance's block partials in
// a fixed order (deterministic), subtracts the weighted mean, converts to time and
// accumulates chi2 partials, which k_rsum adds per instance.
constexpr int RES_BT = 256;
constexpr int RES_RB = 1024;  // rows per block (4 per thread)
constexpr int RES_RPT = RES_RB / RES_BT;  // rows per thread
// BT = threads per residual block: RES_BT, or 64 when every instance has at most 256 rows
// (a grid's points): a wave per block, four blocks per workgroup, no workgroup barrier
// (the 256-thread form gave a 62-row instance one busy wave, three idle ones and the
// barriers of the block sums)
constexpr int RES_SMALLN = 64 * RES_RPT;
template <int BT>
__global__ __launch_bounds__(RES_BT) void k_resid1(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                   const int* __restrict__ rblk_inst, int nrblk,
                                                   const double* __restrict__ ph_hi, const double* __restrict__ ph_lo,
                                                   double* __restrict__ rphase, double* __restrict__ rpart) {
    WgTimer wgt_(WGT_RES1);
    constexpr int NW = BT / 64;
    __shared__ double sh[2 * (RES_BT / 64)];
    const int rb = blockIdx.x * (RES_BT / BT) + (BT == RES_BT ? 0 : (int)__builtin_amdgcn_readfirstlane(threadIdx.x / BT));
    if (BT != RES_BT && rb >= nrblk) return;  // (wave-uniform)
    const int tid = threadIdx.x % BT;
    const int ii = rblk_inst[rb];
    const InstDev I = insts[ii];
    const PsrDev& Pd = psrs[I.psr];
    const pint_spec_t& S = *Pd.spec;
    const int n = I.n;
    const long ro = I.roff;
    const long oo = I.roff - ii;  // output rows: n per instance (roff counts n+1)
    const int r0 = (int)(rb - I.rb0) * RES_RB;
    const int r1 = min(n, r0 + RES_RB);
    const dd tz = dd_make(ph_hi[ro + n], ph_lo[ro + n]);
    dd d0 = dd_make(0.0);
    if (!S.track_pn && S.subtract_mean) d0 = dd_add_d(dd_sub(dd_make(ph_hi[ro], ph_lo[ro]), tz), Pd.dpn[0]);
    double sw = 0.0, swx = 0.0;
    // the thread's RES_RPT rows: every load issued before the arithmetic (one load latency per
    // block, not one per row: a small batch's pass is latency-bound)
    double lh[RES_RPT], ll[RES_RPT], lp[RES_RPT], lpn[RES_RPT], lw[RES_RPT];
#pragma unroll
    for (int u = 0; u < RES_RPT; u++) {
        const int i = r0 + tid + u * BT;
        const bool in = i < r1;
        lh[u] = in ? ph_hi[ro + i] : 0.0;
        ll[u] = in ? ph_lo[ro + i] : 0.0;
        lp[u] = in ? Pd.dpn[i] : 0.0;
        lpn[u] = (in && S.track_pn) ? Pd.pn[i] : 0.0;
        lw[u] = (in && S.weighted_mean) ? Pd.isig[i] : 1.0;
    }
#pragma unroll
    for (int u = 0; u < RES_RPT; u++) {
        const int i = r0 + tid + u * BT;
        if (i >= r1) break;
        dd d = dd_add_d(dd_sub(dd_make(lh[u], ll[u]), tz), lp[u]);
        double full;
        if (S.track_pn) {
            full = dd_to_d(dd_add_d(d, -lpn[u]));
        } else {
            dd x = dd_sub(d, d0);
            full = dd_to_d(dd_sub(x, dd_round_half_up(x)));
        }
        rphase[oo + i] = full;
        double w = S.weighted_mean ? lw[u] * lw[u] : 1.0;
        sw += w;
        swx += w * full;
    }
    if (S.subtract_mean) {
        double v[2] = {swx, sw};
        block_sums<NW, 2>(v, sh);
        swx = v[0];
        sw = v[1];
        if (tid == 0) {
            rpart[3 * rb] = sw;
            rpart[3 * rb + 1] = swx;
        }
    }
}

// k_resid2 with wtile: the Woodbury dot products of the post-fit chi2 (k_wdot's F^T W r and
// 1^T W r, residuals.py:567-589 via utils.py:3074) come out of the same pass.  The PLRedNoise
// basis is the harmonic series e^{i k theta} (k_trig_setup), and e^{i (a + 8b) theta} =
// e^{i a theta} e^{i 8b theta}: one 16x16 v_mfma_f64_16x16x4f64 tile D = A^T B per block with
// A = w r [cos a theta | sin a theta] and B = [cos 8b theta | sin 8b theta] (a, b < 8) holds
// every sum_i w_i r_i e^{i k theta_i}, k < 64 (k_rsum combines: cos k = D[a][b] - D[8+a][8+b],
// sin k = D[8+a][b] + D[a][8+b]; 1^T W r = D[0][0]).  Wave w of the block holds rows r0 + 64w
// + 256j + lane (j < 4): four contiguous 64-row chunks, staged one at a time in the wave's own
// LDS columns and contracted by 16 k-steps of 4 rows.
constexpr int WT_CS = 66;  // k_wdot tile staging: column stride (doubles), 64 rows + 2
constexpr int WT_CS2 = 34;  // k_resid2 tile staging: 32-row halves of the wave's 64 rows, stride 32 + 2
template <int BT>
__global__ __launch_bounds__(RES_BT) void k_resid2(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                   const int* __restrict__ rblk_inst, int nrblk,
                                                   const double* __restrict__ ftay,
                                                   double* __restrict__ rtime, double* __restrict__ rphase,
                                                   double* __restrict__ rpart, double* __restrict__ wtile,
                                                   const double* __restrict__ epart) {
    WgTimer wgt_(WGT_RES2);
    constexpr int NW = BT / 64;
    __shared__ double sh[2 * (RES_BT / 64)];
    extern __shared__ double xs[];  // with wtile, per wave 32 * WT_CS2: A (columns 0-15), B (16-31)
    const int rb = blockIdx.x * (RES_BT / BT) + (BT == RES_BT ? 0 : (int)__builtin_amdgcn_readfirstlane(threadIdx.x / BT));
    if (BT != RES_BT && rb >= nrblk) return;  // (wave-uniform)
    const int tid = threadIdx.x % BT;
    const int ii = rblk_inst[rb];
    const InstDev I = insts[ii];
    const PsrDev& Pd = psrs[I.psr];
    const pint_spec_t& S = *Pd.spec;
    const int n = I.n;
    const long ro = I.roff;
    const long oo = I.roff - ii;
    const int r0 = (int)(rb - I.rb0) * RES_RB;
    const int r1 = min(n, r0 + RES_RB);
    const bool tile = wtile != nullptr;
    const bool harm = tile && __builtin_amdgcn_readfirstlane(S.nred) > 0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;  // (the workgroup's wave: its LDS columns)
    // the thread's RES_RPT rows loaded up front (one load latency per block, not one per row),
    // before the weighted mean's partial sums and barriers, so the two latencies overlap
    double lr[RES_RPT], lf[RES_RPT], ls[RES_RPT];
    double4_t lz[RES_RPT];
#pragma unroll
    for (int j = 0; j < RES_RPT; j++) {
        const int i = r0 + tid + j * BT;
        const bool in = i < r1;
        lr[j] = in ? rphase[oo + i] : 0.0;
        lf[j] = in ? ftay[ro + i] : 1.0;
        ls[j] = in ? Pd.isig[i] : 0.0;
        lz[j] = (harm && in) ? ((gptr<double4_t>)Pd.red_cs)[i] : double4_t{1.0, 0.0, 1.0, 0.0};
    }
    double mean = 0.0;
    if (S.subtract_mean) {  // residuals.py:314-425 weighted mean (utils.py:2002), fixed tree order
        double a = 0.0, b = 0.0;
        if (epart) {  // the evaluation's fused residual pass: its blocks' partials
            for (int k = tid; k < I.neb; k += BT) {
                b += epart[2 * (I.eb0 + k)];
                a += epart[2 * (I.eb0 + k) + 1];
            }
        } else {
            for (int k = tid; k < I.nrb; k += BT) {
                b += rpart[3 * (I.rb0 + k)];
                a += rpart[3 * (I.rb0 + k) + 1];
            }
        }
        double v[2] = {a, b};
        block_sums<NW, 2>(v, sh);
        mean = v[0] / v[1];
    }
    double4_t acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};  // independent chains
    typedef double __attribute__((address_space(3))) ldsd;
    ldsd* X = (ldsd*)(xs + wave * 32 * WT_CS2);
    double c2 = 0.0;
#pragma unroll
    for (int j = 0; j < RES_RPT; j++) {
        const int i = r0 + tid + j * BT;
        double wr = 0.0;
        if (i < r1) {
            double p = lr[j] - mean;
            rphase[oo + i] = p;
            double rt = p / lf[j];  // calc_time_resids (residuals.py:483-538)
            rtime[oo + i] = rt;
            const double is = ls[j];
            double z = rt * is;
            c2 += z * z;
            wr = z * is;
        }
        if (tile) {  // (block-uniform)
            // the row's 32 tile values, then two 32-row halves staged and contracted in turn
            // (half the LDS of one 64-row stage: 4 workgroups per CU instead of 2; the k-steps
            // keep their chains and order -- k-step ks of half h is the 64-row form's 8h + ks)
            const double c1 = lz[j][0], s1 = lz[j][1], c8 = lz[j][2], s8 = lz[j][3];
            double ca = wr, sa = 0.0, cb = 1.0, sb = 0.0;
            double va[8], vs[8], vc[8], vd[8];
#pragma unroll
            for (int a = 0; a < 8; a++) {
                va[a] = ca;
                vs[a] = sa;
                vc[a] = cb;
                vd[a] = sb;
                rot(ca, sa, c1, s1);
                rot(cb, sb, c8, s8);
            }
#pragma unroll
            for (int h = 0; h < 2; h++) {
                if ((lane >> 5) == h) {
                    const int lr_ = lane & 31;
#pragma unroll
                    for (int a = 0; a < 8; a++) {
                        X[a * WT_CS2 + lr_] = va[a];
                        X[(8 + a) * WT_CS2 + lr_] = vs[a];
                        X[(16 + a) * WT_CS2 + lr_] = vc[a];
                        X[(24 + a) * WT_CS2 + lr_] = vd[a];
                    }
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's stores before its reads
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int ks = 0; ks < 8; ks++) {
                    const int row = 4 * ks + (lane >> 4);
                    const double av = X[(lane & 15) * WT_CS2 + row], bv = X[(16 + (lane & 15)) * WT_CS2 + row];
                    acc[ks & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[ks & 3], 0, 0, 0);
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
    c2 = block_sum<NW>(c2, sh);
    if (tid == 0) rpart[3 * rb + 2] = c2;
    if (tile && NW == 1) {  // the wave's own tile (D[4q + lane/16][lane%16])
#pragma unroll
        for (int q = 0; q < 4; q++)
            wtile[(long)rb * 256 + (4 * q + (lane >> 4)) * 16 + (lane & 15)] = (acc[0][q] + acc[1][q]) + (acc[2][q] + acc[3][q]);
    } else if (tile) {
        // the waves' tiles summed in a fixed order through LDS (acc[q]: D[4q + lane/16][lane%16])
        __syncthreads();
        double* red = xs;
#pragma unroll
        for (int q = 0; q < 4; q++)
            red[wave * 256 + (4 * q + (lane >> 4)) * 16 + (lane & 15)] = (acc[0][q] + acc[1][q]) + (acc[2][q] + acc[3][q]);
        __syncthreads();
        for (int e = threadIdx.x; e < 256; e += RES_BT)
            wtile[(long)rb * 256 + e] = (red[e] + red[256 + e]) + (red[512 + e] + red[768 + e]);
    }
}

// k_resid12: k_resid1 and k_resid2 in one launch when every instance is one residual block
// of <= 256 rows (a grid's points) and no trig tiles are formed: a wave per instance forms the
// phase residuals, its weighted sums and -- from those sums, which are the instance's only
// block partial, so k_resid2's read-back would give the same values -- the mean, the time
// residuals and the chi2 partial, the phase residuals kept in registers in between.  The same
// operations in the same order as the two kernels, so the same bits.
__global__ __launch_bounds__(RES_BT) void k_resid12(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                    const int* __restrict__ rblk_inst, int nrblk,
                                                    const double* __restrict__ ph_hi, const double* __restrict__ ph_lo,
                                                    const double* __restrict__ ftay, double* __restrict__ rtime,
                                                    double* __restrict__ rphase, double* __restrict__ rpart) {
    const int rb = blockIdx.x * 4 + (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (rb >= nrblk) return;  // (wave-uniform)
    const int tid = threadIdx.x & 63;
    const int ii = rblk_inst[rb];
    const InstDev I = insts[ii];
    const PsrDev& Pd = psrs[I.psr];
    const pint_spec_t& S = *Pd.spec;
    const int n = I.n;
    const long ro = I.roff;
    const long oo = I.roff - ii;
    const int r0 = (int)(rb - I.rb0) * RES_RB;
    const int r1 = min(n, r0 + RES_RB);
    const dd tz = dd_make(ph_hi[ro + n], ph_lo[ro + n]);
    dd d0 = dd_make(0.0);
    if (!S.track_pn && S.subtract_mean) d0 = dd_add_d(dd_sub(dd_make(ph_hi[ro], ph_lo[ro]), tz), Pd.dpn[0]);
    double sw = 0.0, swx = 0.0;
    double lh[RES_RPT], ll[RES_RPT], lp[RES_RPT], lpn[RES_RPT], lw[RES_RPT], lf[RES_RPT], ls[RES_RPT], full[RES_RPT];
#pragma unroll
    for (int u = 0; u < RES_RPT; u++) {
        const int i = r0 + tid + u * 64;
        const bool in = i < r1;
        lh[u] = in ? ph_hi[ro + i] : 0.0;
        ll[u] = in ? ph_lo[ro + i] : 0.0;
        lp[u] = in ? Pd.dpn[i] : 0.0;
        lpn[u] = (in && S.track_pn) ? Pd.pn[i] : 0.0;
        lw[u] = (in && S.weighted_mean) ? Pd.isig[i] : 1.0;
        lf[u] = in ? ftay[ro + i] : 1.0;
        ls[u] = in ? Pd.isig[i] : 0.0;
        full[u] = 0.0;
    }
#pragma unroll
    for (int u = 0; u < RES_RPT; u++) {  // (k_resid1)
        const int i = r0 + tid + u * 64;
        if (i >= r1) break;
        dd d = dd_add_d(dd_sub(dd_make(lh[u], ll[u]), tz), lp[u]);
        if (S.track_pn) {
            full[u] = dd_to_d(dd_add_d(d, -lpn[u]));
        } else {
            dd x = dd_sub(d, d0);
            full[u] = dd_to_d(dd_sub(x, dd_round_half_up(x)));
        }
        double w = S.weighted_mean ? lw[u] * lw[u] : 1.0;
        sw += w;
        swx += w * full[u];
    }
    double mean = 0.0;
    if (S.subtract_mean) {
        double v[2] = {swx, sw};
        block_sums<1, 2>(v, nullptr);
        if (tid == 0) {
            rpart[3 * rb] = v[1];
            rpart[3 * rb + 1] = v[0];
        }
        // (k_resid2: 0.0 + each partial, the wave's sum of the one partial, 0.0 + that)
        const double a = 0.0 + (0.0 + v[0]), b = 0.0 + (0.0 + v[1]);
        mean = a / b;
    }
    double c2 = 0.0;
#pragma unroll
    for (int u = 0; u < RES_RPT; u++) {  // (k_resid2)
        const int i = r0 + tid + u * 64;
        if (i < r1) {
            double p = full[u] - mean;
            rphase[oo + i] = p;
            double rt = p / lf[u];
            rtime[oo + i] = rt;
            const double z = rt * ls[u];
            c2 += z * z;
        }
    }
    c2 = block_sum<1>(c2, nullptr);
    if (tid == 0) rpart[3 * rb + 2] = c2;
}

// _calc_wls_chi2 (residuals.py:638-667): one wave per instance sums its blocks' chi2
// partials in a fixed tree order (a kernel boundary, not a device-wide fence, orders them)
__global__ __launch_bounds__(64) void k_rsum(const InstDev* __restrict__ insts, const double* __restrict__ rpart,
                                             double* __restrict__ chi2) {
    const InstDev I = insts[blockIdx.x];
    double t = 0.0;
    for (int k = threadIdx.x; k < I.nrb; k += 64) t += rpart[3 * (I.rb0 + k) + 2];
    t = wave_sum(t);
    if (threadIdx.x == 0) chi2[blockIdx.x] = t;
}

// ---------------------------------------------------------------------------------
// k_gram: FP64 MFMA Gram of [T | r] with weights w = 1/sigma^2, one workgroup computes
// the whole (upper-triangular tiles of the) Kp x Kp Gram for one N-split of one instance.
// Also accumulates the unweighted column sums of squares (normalize_designmatrix).
// ---------------------------------------------------------------------------------
constexpr int GCH = 32;       // TOA rows per LDS chunk at the widest Gram (multiple of 4)
constexpr int GMAXKP = 256;   // max padded columns
constexpr int GWAVES = 16;
constexpr int GTHREADS = GWAVES * 64;
constexpr int GMAXT_ALL = 9;  // max upper 16x16 tiles per wave = ceil(136 / 16) at Kp = 256
// rows per chunk for a tiles-per-wave T: narrow Grams (the compact fit layout) stage more
// rows per chunk so each CU keeps enough bytes in flight; the staging registers per thread
// (gram_q) stay <= 10 so the 1024-thread workgroup fits 128 VGPRs without spilling.
__host__ __device__ constexpr int gram_ch(int T) { return T == 1 ? 128 : (T <= 3 ? 64 : 32); }
__host__ __device__ constexpr int gram_maxkp(int T) {  // widest Kp whose upper tiles need T per wave
    return T == 1 ? 80 : T == 2 ? 112 : T == 3 ? 144 : T == 4 ? 160 : T == 5 ? 192 : T == 6 ? 208 : T == 7 ? 224 : T == 8 ? 240 : 256;
}
__host__ __device__ constexpr int gram_q(int T) { return (gram_maxkp(T) * gram_ch(T) + GTHREADS - 1) / GTHREADS; }

// ECORR epoch sums (one wave per epoch, lanes over columns): s_e = sum_{i in e} w_i [T|r]_i,
// W_e = sum w_i, D_e = W_e + 1/phi_e.  The quantisation-matrix block of the GLS normal
// matrix is diagonal (disjoint epochs), so eliminating it is the rank-nep update
// G' = G - sum_e s_e s_e^T / D_e, folded into k_gram as nep extra rows of weight -1/D_e.
// Compact layout: s_e over the dense compact columns (stride Kpd), and the epoch's DMX entry
// c_e = sum_{i in e} w_i x_i of its one bin (ep_bin) into eC (k_ecorr_dmx reduces DD, Sd).
__global__ __launch_bounds__(256) void k_ecorr(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                               const double* __restrict__ M, const double* __restrict__ rtime,
                                               double* __restrict__ esum, double* __restrict__ eD,
                                               double* __restrict__ eW, int compact, const double* __restrict__ dmxv,
                                               double* __restrict__ eC) {
    const int inst = blockIdx.y;
    const InstDev I = insts[inst];
    const PsrDev& Pd = psrs[I.psr];
    const int e = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (e >= Pd.nep) return;
    const bool cmp = compact && Pd.dsplit;
    const int n = I.n, K = cmp ? Pd.Kd : I.K, Kp = cmp ? Pd.Kpd : I.Kp;
    const double* Mi = M + I.moff;
    const double* ri = rtime + (I.roff - inst);
    const int a = Pd.ep_ptr[e], b = Pd.ep_ptr[e + 1];
    double* out = esum + I.eoff + (long)e * Kp;
    // lanes over columns, the epoch's rows 64 at a time: lane j holds row k0 + j's weight,
    // broadcast with readlane (uniform); four independent accumulators keep four row loads in
    // flight (fixed order: deterministic).  Every loop is wave-uniform, so the broadcast never
    // reads a lane that skipped the weight.  (Lanes over 16 rows x 4 columns per load were
    // slower: 0.66 vs 0.49 ms on the C2 batch, whose M -- 0.9 GB -- this pass streams once.)
    for (int c0 = 0; c0 < Kp; c0 += 64) {
        const int c = c0 + lane;
        double acc[4] = {0.0, 0.0, 0.0, 0.0};
        const double* col = (c < K) ? Mi + (long)c * n : ri;  // c > K: read and discarded
        for (int k0 = a; k0 < b; k0 += 64) {
            const int m = min(64, b - k0);
            double wl = 0.0;
            if (lane < m) {
                const double is = Pd.isig[Pd.ep_idx[k0 + lane]];
                wl = is * is;
            }
            int j = 0;
            for (; j + 4 <= m; j += 4) {
#pragma unroll
                for (int u = 0; u < 4; u++) acc[u] += col[Pd.ep_idx[k0 + j + u]] * rdlane(wl, j + u);
            }
            for (; j < m; j++) acc[0] += col[Pd.ep_idx[k0 + j]] * rdlane(wl, j);
        }
        if (c < Kp) out[c] = c <= K ? (acc[0] + acc[1]) + (acc[2] + acc[3]) : 0.0;
    }
    if (lane == 0) {
        double W = 0.0;
        for (int k = a; k < b; k++) {
            double sg = Pd.sigma[Pd.ep_idx[k]];
            W += 1.0 / (sg * sg);
        }
        eW[I.epoff + e] = W;
        eD[I.epoff + e] = W + 1.0 / Pd.ep_phi[e];
        if (cmp) {
            double c = 0.0;
            if (Pd.ep_bin[e] >= 0) {
                const double* xv = dmxv + I.ooff;
                for (int k = a; k < b; k++) {
                    const int i = Pd.ep_idx[k];
                    if (Pd.drow[i] >= 0) c += xv[i] / (Pd.sigma[i] * Pd.sigma[i]);
                }
            }
            eC[I.epoff + e] = c;
        }
    }
}

// k_ecorr_dmx: the ECORR elimination's share of the DMX rows in the compact layout.  With
// every epoch in one DMX column a(e), eliminating the epochs leaves the DMX block diagonal:
//   DD[a] -= sum_{e: a(e)=a} c_e^2 / D_e,   Sd[a][c] -= sum_{e: a(e)=a} c_e s_e[c] / D_e
// (c over the dense compact columns and the residual).  One wave per (DMX column,
// instance), lanes over columns; epochs summed in index order (deterministic).
__global__ __launch_bounds__(64) void k_ecorr_dmx(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                  const double* __restrict__ esum, const double* __restrict__ eD,
                                                  const double* __restrict__ eC, double* __restrict__ Sd,
                                                  double* __restrict__ DD) {
    const InstDev I = insts[blockIdx.y];
    const PsrDev& Pd = psrs[I.psr];
    const int a = blockIdx.x, lane = threadIdx.x;
    if (!Pd.dsplit || Pd.nep == 0 || a >= Pd.ndc) return;
    const int k0 = Pd.bep_ptr[a], k1 = Pd.bep_ptr[a + 1];
    if (k0 == k1) return;
    const int Kd = Pd.Kd, Kpd = Pd.Kpd;
    double* out = Sd + I.sdoff + (long)a * Kpd;
    double dd_ = 0.0;
    for (int k0b = k0; k0b < k1; k0b += 64) {  // the bin's epochs 64 at a time: c_e / D_e per lane
        const int m = min(64, k1 - k0b);
        int el = 0;
        double fl = 0.0;
        if (lane < m) {
            el = Pd.bep_idx[k0b + lane];
            const double ce = eC[I.epoff + el], De = eD[I.epoff + el];
            fl = ce / De;
            dd_ += ce * ce / De;
        }
        for (int c0 = 0; c0 <= Kd; c0 += 64) {  // wave-uniform (the broadcasts read every lane)
            const int c = min(c0 + lane, Kd);
            double acc[4] = {0.0, 0.0, 0.0, 0.0};
            int j = 0;
            for (; j + 4 <= m; j += 4) {
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int e = __builtin_amdgcn_readlane(el, j + u);
                    acc[u] += rdlane(fl, j + u) * esum[I.eoff + (long)e * Kpd + c];
                }
            }
            for (; j < m; j++) acc[0] += rdlane(fl, j) * esum[I.eoff + (long)__builtin_amdgcn_readlane(el, j) * Kpd + c];
            if (c0 + lane <= Kd) out[c] -= (acc[0] + acc[1]) + (acc[2] + acc[3]);
        }
    }
    dd_ = wave_sum(dd_);
    if (lane == 0) DD[I.ddoff + a] -= dd_;
}

// s_e of original column j (j = K: the residual) whatever the layout: the compact layout's
// dense columns through cmap, its DMX columns as the epoch's bin entry c_e
__device__ __forceinline__ double esum_col(const PsrDev& Pd, const InstDev& I, const double* esum,
                                           const double* eC, bool cmp, int e, int j) {
    if (!cmp) return esum[I.eoff + (long)e * I.Kp + j];
    const int c = Pd.cmap[j];
    if (c >= 0) return esum[I.eoff + (long)e * Pd.Kpd + c];
    return Pd.ep_bin[e] == -c - 1 ? eC[I.epoff + e] : 0.0;
}

// k_gram: FP64 MFMA Gram of the whitened rows [T | r] / sigma, one 16-wave workgroup per
// (N-split, instance).  The row-major list of upper 16x16 tiles is cut into 16 contiguous
// runs of T or T-1 tiles (T = ceil(ntiles/16), a template parameter so the first T-1
// tiles are unconditional and the operand reads can be hoisted).  Chunks of CH rows are
// staged global -> registers (prefetched one chunk ahead, branch-free clamped loads) ->
// LDS; every wave then issues CH/4 x T v_mfma_f64_16x16x4f64 with operands from LDS.
// VIRT: the ECORR Schur rows s_e / sqrt(D_e) of k_ecorr, stored negated in the extra
// partial slot, so the sum over partials is G - sum_e s_e s_e^T / D_e.
// Also accumulates the unweighted column sums of squares (normalize_designmatrix).
template <int T, int CH, bool VIRT>
__global__ __launch_bounds__(GTHREADS) void k_gram(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                   const double* __restrict__ M, const double* __restrict__ rtime,
                                                   const double* __restrict__ esum, const double* __restrict__ eD,
                                                   int nsplit, int compact, double* __restrict__ Gpart,
                                                   double* __restrict__ colsq) {
    extern __shared__ double lds[];
    const InstDev I = insts[blockIdx.y];
    const int split = VIRT ? nsplit : blockIdx.x;
    const PsrDev& Pd = psrs[I.psr];
    const bool cmp = compact && Pd.dsplit;
    const int n = I.n, K = cmp ? Pd.Kd : I.K, Kp = cmp ? Pd.Kpd : I.Kp;
    // the staged chunk is column-major, column stride CS = CH + 2 (= 2 mod 32 doubles): the
    // staging stores (lanes over consecutive rows) and the MFMA operand reads (16 columns x
    // 4 rows per wave) both hit distinct bank pairs within each half-wave
    constexpr int CS = CH + 2;
    double* Ts = lds;                    // [Kp][CS] whitened rows, column-major
    double* Sg = lds + Kp * CS;          // [CH] sigma of the staged rows (colsq)
    const double* Mi = M + I.moff;
    const double* ri = rtime + I.ooff;
    const double* Ei = esum + I.eoff;
    const double* eDi = eD + I.epoff;
    long i0, i1;
    if (VIRT) {
        i0 = 0;
        i1 = Pd.nep;
    } else {
        long per = (n + nsplit - 1) / nsplit;
        per = (per + 3) / 4 * 4;
        i0 = split * per;
        i1 = i0 + per;
        if (i1 > n) i1 = n;
        if (i0 > n) i0 = n;
    }
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nt = Kp / 16;
    const int ntiles = nt * (nt + 1) / 2;
    const int t_lo = (ntiles * wave) / GWAVES, t_hi = (ntiles * (wave + 1)) / GWAVES;
    const bool full = (t_hi - t_lo) == T;  // else T-1 tiles
    int tI[T], tJ[T];
    {
        int ti = 0, rem = t_lo;
        while (rem >= nt - ti) { rem -= nt - ti; ti++; }
        int tj = ti + rem;
#pragma unroll
        for (int t = 0; t < T; t++) {
            tI[t] = ti;
            tJ[t] = tj;
            if (t + 2 < T || (t + 1 < T && full)) {
                if (++tj == nt) { ti++; tj = ti; }
            }
        }
    }
    double4_t acc[T];
#pragma unroll
    for (int t = 0; t < T; t++) acc[t] = (double4_t){0, 0, 0, 0};
    // column sums of squares: every thread takes column tid % Kp of rows tid / Kp (mod CG2)
    // of each chunk; the CG2 partials are summed through LDS at the end of the split
    const int ccol = tid % Kp, cgrp = tid / Kp, CG2 = GTHREADS / Kp;
    double csq = 0.0;
    // staging: thread -> (row ii = tid % CH, columns c_base + (1024/CH) q)
    constexpr int CG = GTHREADS / CH;
    const int ii = tid % CH, c_base = tid / CH;
    const int nq = (Kp + CG - 1) / CG;  // uniform
    // the prefetch only issues loads (raw values into registers, clamped addresses, no
    // arithmetic on the results), so the waits land at the LDS store of the next chunk
    constexpr int QN = gram_q(T);
    double st[QN];
    double sg_next = 1.0, w_next = 0.0, r_next = 0.0;
    bool ok_next = false;
    auto load = [&](long c0) {
        long row = c0 + ii;
        ok_next = row < i1;
        if (!ok_next) row = i1 - 1;  // clamped, valid address; zero weight at the store
        if (VIRT) {
            w_next = eDi[row];
        } else {
            sg_next = Pd.sigma[row];
            w_next = Pd.isig[row];
            r_next = ri[row];
        }
#pragma unroll
        for (int q = 0; q < QN; q++) {
            if (q < nq) {
                const int c = c_base + CG * q;
                if (VIRT) st[q] = Ei[row * Kp + (c < Kp ? c : Kp - 1)];
                else st[q] = Mi[(long)(c < K ? c : K - 1) * n + row];
            }
        }
    };
    if (i0 < i1) load(i0);
    for (long c0 = i0; c0 < i1; c0 += CH) {
        __syncthreads();  // previous chunk's MFMAs are done with the LDS tile
        {
            double iw = VIRT ? 1.0 / sqrt(w_next) : w_next;
            iw = ok_next ? iw : 0.0;
#pragma unroll
            for (int q = 0; q < QN; q++) {
                const int c = c_base + CG * q;
                if (q < nq && c < Kp) {
                    double v = st[q];
                    if (!VIRT) v = c < K ? v : (c == K ? r_next : 0.0);
                    Ts[c * CS + ii] = v * iw;
                }
            }
            if (!VIRT && c_base == 0) Sg[ii] = sg_next;
        }
        __syncthreads();
        if (c0 + CH < i1) load(c0 + CH);  // prefetch next chunk (overlaps the MFMAs)
        if (!VIRT && cgrp < CG2) {
            const int nr = (i1 - c0 < CH) ? (int)(i1 - c0) : CH;
            for (int r = cgrp; r < nr; r += CG2) {
                const double u = Ts[ccol * CS + r] * Sg[r];
                csq += u * u;
            }
        }
#pragma unroll
        for (int kk = 0; kk < CH / 4; kk++) {
            const double* Tr = Ts + (lane & 15) * CS + kk * 4 + (lane >> 4);
            double a[T], b[T];
#pragma unroll
            for (int t = 0; t < T; t++) {
                a[t] = Tr[tI[t] * 16 * CS];
                b[t] = Tr[tJ[t] * 16 * CS];
            }
#pragma unroll
            for (int t = 0; t < T - 1; t++) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[t], b[t], acc[t], 0, 0, 0);
            if (full) acc[T - 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[T - 1], b[T - 1], acc[T - 1], 0, 0, 0);
        }
    }
    // write partial tiles: D[row=(lane>>4)+4*r][col=lane&15]
    double* G = Gpart + I.goff + (long)split * Kp * Kp;
    const double sgn = VIRT ? -1.0 : 1.0;
#pragma unroll
    for (int t = 0; t < T; t++) {
        if (t < T - 1 || full) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                int row = tI[t] * 16 + (lane >> 4) + 4 * q;
                int col = tJ[t] * 16 + (lane & 15);
                G[(long)row * Kp + col] = sgn * acc[t][q];
            }
        }
    }
    if (!VIRT) {
        __syncthreads();  // done with the LDS tile: reuse it for the colsq partials
        if (cgrp < CG2) lds[cgrp * Kp + ccol] = csq;
        __syncthreads();
        if (tid < K) {
            double v = 0.0;
            for (int g = 0; g < CG2; g++) v += lds[g * Kp + tid];
            colsq[(I.coff + tid) * nsplit + split] = v;
        }
    }
}

// k_gram_s: k_gram's output (Gram partial of [T | r] / sigma, column sums of squares) for
// small instances -- Kp <= 32, at most GS_MAXN rows per split (a grid's points: 62-row
// NGC6440E fits by the 10^5).  One wave per (N-split, instance), four instances per
// workgroup, no LDS and no barrier: lane l loads the MFMA operand it contributes directly,
// row 4 kk + l / 16 of column l % 16 (and l % 16 + 16), weighted as it arrives, so a k-step
// is one v_mfma_f64_16x16x4f64 per upper tile ((0,0); with Kp = 32 also (0,1), (1,1)).
// The 16-wave k_gram gave such an instance one tile on one wave and 15 idle waves.
constexpr int GS_MAXN = 512;
__global__ __launch_bounds__(256) void k_gram_s(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                int count, const double* __restrict__ M,
                                                const double* __restrict__ rtime, int nsplit, int compact,
                                                double* __restrict__ Gpart, double* __restrict__ colsq) {
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.y * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (q >= count) return;  // (wave-uniform)
    const InstDev I = insts[q];
    const PsrDev& Pd = psrs[I.psr];
    const bool cmp = compact && Pd.dsplit;
    const int n = I.n, K = cmp ? Pd.Kd : I.K, Kp = cmp ? Pd.Kpd : I.Kp;
    const bool two = Kp > 16;
    const int split = blockIdx.x;
    long per = (n + nsplit - 1) / nsplit;
    per = (per + 3) / 4 * 4;
    const long i0 = min((long)n, split * per), i1 = min((long)n, i0 + per);
    const double* Mi = M + I.moff;
    const double* ri = rtime + I.ooff;
    const int c0 = lane & 15, c1 = c0 + 16, kr = lane >> 4;
    // the lane's two columns: a design-matrix column, the residual (column K) or padding
    const double* p0 = c0 < K ? Mi + (long)c0 * n : ri;
    const double* p1 = c1 < K ? Mi + (long)c1 * n : ri;
    const bool z0 = c0 > K, z1 = c1 > K || !two;
    double4_t a00 = {0, 0, 0, 0}, a01 = {0, 0, 0, 0}, a11 = {0, 0, 0, 0};
    double s0 = 0.0, s1 = 0.0;  // unweighted sums of squares of the lane's columns
    constexpr int U = 4;        // k-steps per iteration: every load of the 16 rows issued first
    for (long r0 = i0; r0 < i1; r0 += 4 * U) {
        double v0[U], v1[U], w[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long row = r0 + 4 * u + kr;
            ok[u] = row < i1;
            const long rc = ok[u] ? row : i0;  // clamped, valid address
            w[u] = ok[u] ? Pd.isig[rc] : 0.0;
            v0[u] = z0 ? 0.0 : p0[rc];
            v1[u] = z1 ? 0.0 : p1[rc];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const double x0 = v0[u] * w[u], x1 = v1[u] * w[u];
            if (ok[u]) {
                s0 += v0[u] * v0[u];
                s1 += v1[u] * v1[u];
            }
            a00 = __builtin_amdgcn_mfma_f64_16x16x4f64(x0, x0, a00, 0, 0, 0);
            if (two) {
                a01 = __builtin_amdgcn_mfma_f64_16x16x4f64(x0, x1, a01, 0, 0, 0);
                a11 = __builtin_amdgcn_mfma_f64_16x16x4f64(x1, x1, a11, 0, 0, 0);
            }
        }
    }
    // only the (K+1) x (K+1) entries the solves read (a 62-row grid point's 16 x 16 tile was
    // 2 KB of writes, ~90 % padding)
    double* G = Gpart + I.goff + (long)split * Kp * Kp;
#pragma unroll
    for (int e = 0; e < 4; e++) {  // D[row = lane / 16 + 4 e][col = lane % 16]
        const int row = kr + 4 * e;
        if (row <= K && c0 <= K) G[(long)row * Kp + c0] = a00[e];
        if (two) {
            if (row <= K && c1 <= K) G[(long)row * Kp + c1] = a01[e];
            if (row + 16 <= K && c1 <= K) G[(long)(row + 16) * Kp + c1] = a11[e];
        }
    }
    // column sums of squares: the four lanes of a column (kr = 0..3) summed in a fixed order
    s0 += __shfl_xor(s0, 16);
    s0 += __shfl_xor(s0, 32);
    s1 += __shfl_xor(s1, 16);
    s1 += __shfl_xor(s1, 32);
    if (kr == 0) {
        if (c0 < K) colsq[(I.coff + c0) * nsplit + split] = s0;
        if (two && c1 < K) colsq[(I.coff + c1) * nsplit + split] = s1;
    }
}


// k_dmx: Gram rows of the DMX columns in the compact fit layout when a bin's TOAs are not
// one contiguous row range (otherwise k_gram accumulates them).  A DMX column is x_i on
// the TOAs of its bin (d_dm_d_DMX, dispersion_model.py:684, times DMconst/f^2 and the
// phase chain) and 0 elsewhere, so its Gram row is a sum over the bin's TOAs:
//   Sd[a][c] = sum_{i in bin a} w_i x_i [T|r]_ic (c over the compact columns + residual),
//   DD[a] = sum w_i x_i^2 (bins do not overlap in this layout), DCS[a] = sum x_i^2.
// One workgroup per (bin, instance); a wave per column, lanes over the bin's TOAs.
__global__ __launch_bounds__(256) void k_dmx(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                             const double* __restrict__ M, const double* __restrict__ rtime,
                                             const double* __restrict__ dmxv, double* __restrict__ Sd,
                                             double* __restrict__ DD, double* __restrict__ DCS) {
    const InstDev I = insts[blockIdx.y];
    const PsrDev& Pd = psrs[I.psr];
    const int a = blockIdx.x;
    if (!Pd.dsplit || Pd.dcontig || Pd.vg || a >= Pd.ndc) return;  // dcontig: k_dmx_rows
    const int n = I.n, Kd = Pd.Kd, Kpd = Pd.Kpd;
    const double* Mi = M + I.moff;
    const double* ri = rtime + I.ooff;
    const double* xv = dmxv + I.ooff;
    const int k0 = Pd.dptr[a], k1 = Pd.dptr[a + 1];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double* out = Sd + I.sdoff + (long)a * Kpd;
    if (k1 - k0 <= 4 * 64) {
        // the bin's rows and weights w_i x_i held in registers (lane l: rows k0 + l + 64 u), so
        // each column costs its own loads only, four of them in flight per lane
        int ir[4];
        double wx[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int k = k0 + lane + 64 * u;
            ir[u] = k < k1 ? Pd.didx[k] : Pd.didx[k0];
            const double is = Pd.isig[ir[u]];
            wx[u] = k < k1 ? is * is * xv[ir[u]] : 0.0;
        }
        const int nu = (k1 - k0 + 63) >> 6;
        // four columns per iteration (c = wave + 4 v + 16 j): their loads and reductions interleave
        for (int cb = wave; cb <= Kd; cb += 16) {
            double acc[4];
#pragma unroll
            for (int v = 0; v < 4; v++) {
                const int c = min(cb + 4 * v, Kd);
                const double* col = c < Kd ? Mi + (long)c * n : ri;
                double t = 0.0;
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (u < nu) t += wx[u] * col[ir[u]];
                acc[v] = t;
            }
#pragma unroll
            for (int v = 0; v < 4; v++) acc[v] = wave_sum(acc[v]);
            if (lane == 0) {
#pragma unroll
                for (int v = 0; v < 4; v++)
                    if (cb + 4 * v <= Kd) out[cb + 4 * v] = acc[v];
            }
        }
    } else {
        for (int c = wave; c <= Kd; c += 4) {
            const double* col = c < Kd ? Mi + (long)c * n : ri;
            double acc = 0.0;
            for (int k = k0 + lane; k < k1; k += 64) {
                const int i = Pd.didx[k];
                const double is = Pd.isig[i];
                acc += is * is * xv[i] * col[i];
            }
            acc = wave_sum(acc);
            if (lane == 0) out[c] = acc;
        }
    }
    if (wave == 0) {
        double d = 0.0, q = 0.0;
        for (int k = k0 + lane; k < k1; k += 64) {
            const int i = Pd.didx[k];
            const double x = xv[i], is = Pd.isig[i];
            d += is * is * x * x;
            q += x * x;
        }
        d = wave_sum(d);
        q = wave_sum(q);
        if (lane == 0) {
            DD[I.ddoff + a] = d;
            DCS[I.ddoff + a] = q;
        }
    }
}

// k_dmx_rows: the same bin sums when every bin is one contiguous row range (time-sorted
// TOAs).  One workgroup per (bin, instance): 64-row slices of [T|r] are staged through LDS
// with coalesced column reads (a wave reads 64 consecutive rows of one column), then
// thread c sums column c down the slice; thread Kd+1 forms DD/DCS.
constexpr int DMX_RS = 64;
__global__ __launch_bounds__(256) void k_dmx_rows(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                  const double* __restrict__ M, const double* __restrict__ rtime,
                                                  const double* __restrict__ dmxv, double* __restrict__ Sd,
                                                  double* __restrict__ DD, double* __restrict__ DCS) {
    extern __shared__ double lds[];
    const InstDev I = insts[blockIdx.y];
    const PsrDev& Pd = psrs[I.psr];
    const int a = blockIdx.x;
    if (!Pd.dsplit || !Pd.dcontig || Pd.vg || a >= Pd.ndc) return;  // vg: fused into k_gram_v
    const int n = I.n, Kd = Pd.Kd, Kpd = Pd.Kpd;
    const int W = Kd + 2;               // columns + residual + the DD/DCS slot
    const int str = W | 1;              // odd stride
    double* Ts = lds;                   // [DMX_RS][str]
    double* wx = lds + DMX_RS * str;    // [DMX_RS] w_i x_i
    double* xx = wx + DMX_RS;           // [DMX_RS] x_i
    const double* Mi = M + I.moff;
    const double* ri = rtime + I.ooff;
    const double* xv = dmxv + I.ooff;
    const int cnt = Pd.dptr[a + 1] - Pd.dptr[a];
    const int lo = cnt > 0 ? Pd.didx[Pd.dptr[a]] : 0, hi = lo + cnt;
    const int t = threadIdx.x, row = t & 63, g = t >> 6;
    // summing threads: column sc = t % W of rows t / W (mod SG)
    const int sc = t % W, sg = t / W, SG = (256 / W < DMX_RS) ? 256 / W : DMX_RS;
    double acc = 0.0, qacc = 0.0;
    for (int r0 = lo; r0 < hi; r0 += DMX_RS) {
        const int nr = hi - r0 < DMX_RS ? hi - r0 : DMX_RS;
        const int i = r0 + (row < nr ? row : nr - 1);
        for (int cb = g; cb <= Kd; cb += 32) {  // 8 independent loads in flight per thread
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int c = cb + 4 * u;
                v[u] = c < Kd ? Mi[(long)c * n + i] : ri[i];
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int c = cb + 4 * u;
                if (c <= Kd && row < nr) Ts[row * str + c] = v[u];
            }
        }
        if (g == 0 && row < nr) {
            const double is = Pd.isig[i], x = xv[i];
            wx[row] = is * is * x;
            xx[row] = x;
        }
        __syncthreads();
        if (sg < SG) {
            for (int r = sg; r < nr; r += SG) {
                if (sc <= Kd) acc += Ts[r * str + sc] * wx[r];
                else {
                    acc += wx[r] * xx[r];
                    qacc += xx[r] * xx[r];
                }
            }
        }
        __syncthreads();
    }
    // sum the SG row-group partials
    if (sg < SG) {
        Ts[sg * str + sc] = acc;
        if (sc == Kd + 1) wx[sg] = qacc;
    }
    __syncthreads();
    if (t < W) {
        double v = 0.0;
        for (int q = 0; q < SG; q++) v += Ts[q * str + t];
        if (t <= Kd) Sd[I.sdoff + (long)a * Kpd + t] = v;
        else {
            double qv = 0.0;
            for (int q = 0; q < SG; q++) qv += wx[q];
            DD[I.ddoff + a] = v;
            DCS[I.ddoff + a] = qv;
        }
    }
}

// ---------------------------------------------------------------------------------
// Compact fit layout, "vg" path (PsrDev::vg, PINT_OPT_VGRAM), one fused kernel k_gram_v.
// The PLRedNoise basis (noise_model.py:861-880, frequencies :847-858) is a harmonic
// series: F[:,2h] = sin((h+1) theta_i), F[:,2h+1] = cos((h+1) theta_i), theta_i =
// 2 pi t_i f_1, t = tdbld * 86400 s, f_k = k f_1.  Hence
//  - F is generated in the kernel by rotations of the per-TOA fundamental (k_trig_setup),
//    never stored in M;
//  - its Gram block F^T W F follows from the weighted trig sums C_m = sum_i w_i cos(m
//    theta_i), S_m = sum_i w_i sin(m theta_i), m <= 2 nred, by the product-to-sum
//    identities (k_greduce), and every C_m, S_m (m < 64) is one 16x16 MFMA tile A^T B of
//    A = [cos a theta | sin a theta], B = [cos 8b theta | sin 8b theta] (a, b < 8), since
//    e^{i(a + 8b) theta} = e^{i a theta} e^{i 8b theta}: O(N) MFMA work instead of the
//    O(N nred^2) of F^T W F;
//  - the MFMA row tiles are [T | r | DMX slots] (compact timing columns, residual, and the
//    DMX bins of the N-split in bin % vns slots: bins are contiguous row ranges, so each
//    slot holds one bin per split) against every column [T | r | slots | F]: the DMX bin
//    rows of the normal matrix come out of the same tiles.
// ---------------------------------------------------------------------------------
constexpr int VTRIG = 64;   // trig sums per kind: C_m, S_m weighted, U_m, V_m unweighted (m < 64)   // trig sums m = 0..63 (nred <= 31)
constexpr int VMAXR0 = 48;  // timing columns + residual staged from M (<= 3 row tiles)
constexpr int VMAXKP = 112; // widest k_gram_v LDS tile [T | r | slots | F] (7 column tiles: two
                            // row blocks of VMAXKP + 33 columns fit the 160 KB of LDS)
constexpr int VCH = 64;     // k_gram_v rows per chunk
constexpr int GW = 4;       // k_gram_v waves per workgroup (one per SIMD)
constexpr int GVB = 1;      // k_gram_v LDS row-block buffers (1: two workgroups per CU)
constexpr int GWG = 2;      // k_gram_v workgroups per CU
constexpr int VTG = 4;      // k_gram_v tiles per round of the cross-wave reduction

// sin/cos of 2 pi frac(x) for a phase x in cycles (double-double argument reduction)
__device__ __forceinline__ void dd_sincos_cyc(dd x, double* s, double* c) {
    const double fr = dd_to_d(dd_sub(x, dd_floor(x)));
    sincos(TWO_PI * fr, s, c);
}


// e^{i k theta} from e^{i theta} by binary powering (k >= 0)
__device__ __forceinline__ void cpow(double c1, double s1, int k, double& c, double& s) {
    c = 1.0;
    s = 0.0;
    double bc = c1, bs = s1;
    while (k) {
        if (k & 1) rot(c, s, bc, bs);
        k >>= 1;
        if (k) rot(bc, bs, bc, bs);
    }
}

// rows [i0, i1) of N-split `split` (k_gram's partition: a multiple of 4 rows per split)
__device__ __forceinline__ void split_rows(int n, int nsplit, int split, long& i0, long& i1) {
    long per = (n + nsplit - 1) / nsplit;
    per = (per + 3) / 4 * 4;
    i0 = split * per;
    i1 = i0 + per;
    if (i1 > n) i1 = n;
    if (i0 > n) i0 = n;
}

// LDS column order of k_gram_v -> compact column: timing [0, r0) stay, the residual (LDS
// column r0) goes to Kd, the Fourier columns (r0, Kd] move down by one, padding stays.
__device__ __forceinline__ int vg_cidx(int p, int r0, int Kd) {
    return p < r0 ? p : (p == r0 ? Kd : (p <= Kd ? p - 1 : p));
}

// p ? a : b as a per-lane value: the compiler turns a select between two store addresses
// on a wave-uniform condition into branches, which is what the staging must not have
__device__ __forceinline__ int vsel(bool p, int a, int b) {
    int r = p ? a : b;
    asm("" : "+v"(r));
    return r;
}


// (experiment) per-workgroup phase timestamps of k_gram_v
__device__ unsigned long long g_gvts[4096 * 5];
#define GVTS(k) do { const int b_ = blockIdx.y * gridDim.x + blockIdx.x; \
    if ((dbg & 8) && threadIdx.x == 0 && b_ < 4096) g_gvts[b_ * 5 + k] = (k) == 4 ? (unsigned long long)__smid() : __builtin_amdgcn_s_memrealtime(); } while (0)

// e^{i k theta} from e^{i theta} for a wave-uniform 0 <= k < 8: scalar branches on k's bits,
// at most two squarings and two products
__device__ __forceinline__ void cpow_u8(double c1, double s1, int k, double& c, double& s) {
    c = 1.0;
    s = 0.0;
    if (k & 1) {
        c = c1;
        s = s1;
    }
    if (k & 6) {
        double bc = c1, bs = s1;
        rot(bc, bs, c1, s1);  // e^{2 i theta}
        if (k & 2) rot(c, s, bc, bs);
        if (k & 4) {
            rot(bc, bs, bc, bs);  // e^{4 i theta}
            rot(c, s, bc, bs);
        }
    }
}

// k_gram_v: one GW-wave workgroup per (N-split, instance), GWG workgroups per CU.  Chunks of
// VCH = 64 rows are staged in LDS as the whitened row block [T | r | DMX slots | F | A | B]
// (column-major, stride VCH+2), one row per lane: wave w stages the timing columns w, w + GW,
// ..., the trig-block harmonics a = w, w + GW (A: e^{i a theta}, B: e^{i 8a theta}) and from
// each A harmonic the Fourier harmonics a + 1 + 8u, by short powers and rotations of the row's
// e^{i theta}, e^{i 8 theta} (k_trig_setup) that carry the weight along; the residual and the
// row's DMX slot entry (the slot block is zero except one entry per row, so only the previous
// and the new entry of the row are rewritten) come with wave 0's share.  Each wave then takes
// 16 rows of the chunk (four 4-row k-steps) and accumulates ALL the tiles (row tiles < ntr x
// column tiles >= row tile) of its rows with v_mfma_f64_16x16x4f64, plus the trig tile A^T B;
// the tiles whose rows and columns are all DMX slots hold only the bins' DD, which k_greduce
// forms from the TOAs, and are skipped.
// Measured on gfx950 (bench/coissue_probe.hip, bench/valu_probe.hip): an FP64 MFMA holds its
// SIMD's vector issue for its whole 64 cycles, and a dependent FP64 vector op has ~40 cycles
// of latency.  So staging and MFMAs cannot overlap within a SIMD; the layout minimises their
// sum and hides latencies with the second workgroup: with one LDS buffer each (GVB = 1) two
// workgroups share a CU, one's staging, barriers, loads, prologue and epilogue fill the
// other's gaps (0.125 ms on the bench PTA; one 8-wave double-buffered workgroup per CU:
// 0.15 ms).  The row data of chunk c+1 is loaded into registers while chunk c is in the MFMAs.
// Unused columns go to a dummy LDS column (no branches in the staging).  The waves' partial
// tiles are summed through LDS at the end.  (Built with MFMA accumulators in VGPRs: in AGPRs
// the loop-carried tiles were copied out and back every chunk.)
// VB (binned DMX x F): the DMX bin rows' Fourier entries sum_{i in bin} x_i w_i e^{i k theta_i}
// come from one more 16x16 tile per k-step, A^T B'' with A the trig block [cos a theta | sin a
// theta]/sigma and B'' = x [cos 8c theta | sin 8c theta]/sigma (c < 4) in the 8 columns of the
// row's bin parity (the other 8 zero), k = a + 8c: the accumulator holds two bins (even, odd)
// and a half is flushed to its bin's partial (per split and wave) when a new bin of its
// parity arrives.  It replaces the all-slot row tiles x F (4 tiles per k-step: each row has
// one nonzero slot).  Each wave takes a contiguous quarter of the split (lane l of a chunk
// stages row quarter (l >> 4), offset 16c + (l & 15)), so a wave meets each bin once; the
// flushes happen once per chunk, before its MFMAs, from the first and last bin of the wave's
// 16 rows: the host admits the layout only if every such 16-row group holds <= 2 bins, of
// distinct parity.
// VB: write the half of accB that holds a bin (parity p) to the bin's partial dst and clear it
// (lanes of columns 8p..8p+7 hold it: row 4q + (lane >> 4), column lane & 7)
__device__ __forceinline__ void vb_flush(double4_t& acc, double* __restrict__ dst, int p, int lane) {
    const bool mine = ((lane >> 3) & 1) == p;
    if (mine) {
#pragma unroll
        for (int q = 0; q < 4; q++) dst[(4 * q + (lane >> 4)) * 8 + (lane & 7)] = acc[q];
    }
#pragma unroll
    for (int q = 0; q < 4; q++) acc[q] = mine ? 0.0 : acc[q];
}
// VB: bin b enters the accumulator half of its parity; a half holding another bin is flushed.
// cur0/cur1 are updated by selects, not by stores in two branches: the branch form was merged
// into a parity-indexed private array (scratch), whose reload waited on vmcnt(0) -- i.e. on the
// next chunk's prefetch -- in every chunk
#define VB_ENTER(b)                                                                                  \
    do {                                                                                             \
        const int b_ = (b);                                                                          \
        const int p_ = b_ & 1;                                                                       \
        const int c_ = p_ ? cur1 : cur0;                                                             \
        if (c_ != b_) {                                                                              \
            if (c_ >= 0) vb_flush(accB, vbase + (long)(c_ % NS) * 128, p_, lane);                    \
            cur1 = __builtin_amdgcn_readfirstlane(p_ ? b_ : cur1);                                   \
            cur0 = __builtin_amdgcn_readfirstlane(p_ ? cur0 : b_);                                   \
        }                                                                                            \
    } while (0)

// The pre-fit residual pass folded into the Gram (k_gram_v's staging forms r itself): with
// `on`, the evaluation with the fit layout ran k_resid1 only, and wave 0 stages
// r = (p - mean) / F from k_resid1's phase residual p, the Taylor factor F and the weighted
// mean of the instance's block sums -- the same operations, in the same order, as k_resid2
// (whose launch is deferred to the first reader of the time residuals, pint_* flush_r2).
struct GvResid {
    const double* rph;    // k_resid1's phase residuals (output rows)
    const double* ftay;   // Taylor factors (n + 1 rows per instance)
    const double* rpart;  // residual blocks' (sum w, sum w x, -)
    int on;
    const double* epart;  // (non-null) the fused residual pass's partials instead, 2 per evaluation block
};

template <int NTR, int NTC, int NSK, bool VB>
__device__ __forceinline__ void gram_v_body(double* lds, const PsrDev* __restrict__ psrs,
                                            const InstDev* __restrict__ insts, const double* __restrict__ M,
                                            const double* __restrict__ rtime, const double* __restrict__ dmxv,
                                            int nsplit, double* __restrict__ Gpart, double* __restrict__ Sdp,
                                            double* __restrict__ colsq, double* __restrict__ TSp,
                                            double* __restrict__ BFp, int dbg, GvResid R) {
    constexpr int NTH = GW * 64;
    constexpr int CH = VCH;
    constexpr int CS = CH + 2;  // column stride (= 2 mod 32 doubles)
    constexpr int QL = (16 * NTR + GW - 1) / GW;  // timing columns staged per lane (r0 < 16 NTR)
    constexpr int NT = NTR * NTC - NTR * (NTR - 1) / 2;
    constexpr int KS = CH / 4 / GW;  // k-steps per wave per chunk
    constexpr int TA = 8 / GW;  // trig-block harmonics per wave
    constexpr int HMAX = 4;     // Fourier harmonics per A harmonic (a + 1 + 8u < 32)
    static_assert(8 % GW == 0 && KS >= 1 && (GVB == 1 || GVB == 2) && (!VB || (GVB == 1 && GW == 4 && NTC <= 6)),
                  "k_gram_v layout");
    GVTS(0);
    GVTS(4);
    const InstDev I = insts[blockIdx.y];
    const int split = blockIdx.x;
    const PsrDev& Pd = psrs[I.psr];
    const int n = I.n, Kd = Pd.Kd, Kp = Pd.Kpd, r0 = Pd.red0c, NS = Pd.vns, Kpv = Pd.vkp;
    const int nred = __builtin_amdgcn_readfirstlane(Pd.spec->nred);  // (a flat load: not known uniform)
    const int s0 = r0 + 1, f0 = r0 + 1 + NS, Wv = f0 + (Kd - r0);  // slot / Fourier / end columns
    // Kpv == 16 NTC and f0 == 16 NTR (the launch groups instances by both)
    const int SW = Kd + 3;  // Sdp row: compact columns 0..Kd, DD (+1 spare)
    // past Kpv (VB): the trig block A = [cos a theta | sin a theta]/sigma (a < 8) and the
    // binned block B'' (tX).  F^T W F comes from the weighted trig sums C_m, S_m, which depend
    // on the TOAs and sigma only (PsrDev::trigW, k_trig_setup); the unweighted sums for the Fourier
    // column norms likewise (PsrDev::trigU).  DUM: the write-only dummy column.
    const int tA = Kpv, DUM = Kpv + 16, tX = Kpv + 17, Kpt = Kpv + (VB ? 33 : 17);
    double* const Tb0 = lds;
    double* const Tb1 = lds + (GVB - 1) * Kpt * CS;
    long i0, i1;
    split_rows(n, nsplit, split, i0, i1);
    // VB: chunk c, lane l -> row i0 + (l >> 4) Q + 16 c + (l & 15) (each wave a quarter)
    const long QV = (i1 - i0 + CH - 1) / CH * 16;
    const double* Mi = M + I.moff;
    const double* ri = rtime + I.ooff;
    const double* xv = dmxv + I.ooff;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // (R.on) the weighted mean of the phase residuals, summed as k_resid2 sums it: partial k
    // of the instance's nrb <= 64 blocks on lane k of one wave, the same shuffle tree
    const bool fr = R.on != 0;
    const double* rpi = fr ? R.rph + I.ooff : ri;
    const double* fti = R.ftay + I.roff;
    double mean_r = 0.0;
    if (fr && wave == 0) {
        double a = 0.0, b = 0.0;
        if (R.epart) {
            if (lane < I.neb) {
                b = R.epart[2 * (I.eb0 + lane)];
                a = R.epart[2 * (I.eb0 + lane) + 1];
            }
        } else if (lane < I.nrb) {
            b = R.rpart[3 * (I.rb0 + lane)];
            a = R.rpart[3 * (I.rb0 + lane) + 1];
        }
        a = 0.0 + wave_sum(a);
        b = 0.0 + wave_sum(b);
        if (Pd.spec->subtract_mean) mean_r = a / b;
    }
    double4_t acc[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) acc[t] = (double4_t){0, 0, 0, 0};
    double csq[QL];  // sums of squares of this wave's timing columns (lanes = rows)
#pragma unroll
    for (int q = 0; q < QL; q++) csq[q] = 0.0;
    int sp0 = -1, sp1 = -1;  // per buffer: the slot column of this lane's row of two chunks ago
    double w_n = 0.0, r_n = 0.0, f_n = 1.0, x_n = 0.0, c1_n = 1.0, s1_n = 0.0, c8_n = 1.0, s8_n = 0.0;
    double st[QL] = {};
    int d_n = -1;
    bool ok_n = false;
    int binc = -1;              // VB: the DMX bin of this lane's staged row (-1: none)
    int cur0 = -1, cur1 = -1;   // VB: bins held by the even / odd half of accB (wave-uniform)
    double4_t accB = {0, 0, 0, 0};
    double* const vbase = BFp + I.vboff + ((long)split * GW + wave) * NS * 128;
    // Every staging / MFMA lambda takes the wave index as a compile-time constant W (the
    // chunk loop is instantiated once per wave and dispatched on the uniform wave id): the
    // wave's LDS columns and trig harmonics are then constants -- immediate offsets, no
    // runtime selects in the powers e^{i a theta}, fewer scalar registers (no SGPR spills).
    // With NTC - NTR >= 4 every harmonic h < 32 has a column inside the tile (f0 = 16 NTR):
    // the harmonics past nred are staged unconditionally into padding columns that the
    // epilogue never stores.
    constexpr bool FULLH = NTC - NTR >= 4;
    int sl_n = -1;  // the staged row's DMX slot (dslot; wave 0)
    auto load = [&](auto Wc, long c0) {  // the next chunk's row data -> registers (clamped rows)
        constexpr int W = decltype(Wc)::value;
        long row = c0 + lane;
        if (VB) {  // c0 = i0 + 16 c
            const long rel = (c0 - i0) + (long)(lane >> 4) * QV + (lane & 15);
            row = i0 + rel;
            if (rel >= (long)(lane >> 4) * QV + QV) row = i1;  // past this quarter (unused)
        }
        ok_n = row < i1;
        row = ok_n ? row : i1 - 1;
        // (global-address-space loads: through generic pointers they would be flat loads,
        // which also count against lgkmcnt, so every LDS wait would wait for them too)
        w_n = ok_n ? ((gptr<double>)Pd.isig)[row] : 0.0;  // rows past the split weigh 0
        if (W == 0) {
            r_n = rpi[row];  // (fr: the phase residual; its time residual is formed at the stage)
            if (fr) f_n = fti[row];
            x_n = xv[row];
            sl_n = ((gptr<int>)Pd.dslot)[row];
        }
        if (VB) {
            d_n = ((gptr<int>)Pd.drow)[row];
            if (W != 0) x_n = xv[row];
        }
        const double4_t z = ((gptr<double4_t>)Pd.red_cs)[row];
        c1_n = z[0];
        s1_n = z[1];
        c8_n = z[2];
        s8_n = z[3];
#pragma unroll
        for (int q = 0; q < QL; q++) {
            const int c = W + GW * q;
            if (c < r0) st[q] = ok_n ? Mi[(long)c * n + row] : 0.0;  // uniform guard
        }
    };
    // LDS stores through a 32-bit (address space 3) pointer: column index x CS + lane
    typedef double __attribute__((address_space(3))) ldsd;
    auto put = [&](ldsd* Ts, int colidx, double v) { Ts[colidx * CS + lane] = v; };
    auto stage = [&](auto Wc, double* Tsg, int& sp) {  // registers -> whitened row block in LDS
        constexpr int W = decltype(Wc)::value;
        ldsd* Ts = (ldsd*)Tsg;
        const double iw = w_n;
#pragma unroll
        for (int q = 0; q < QL; q++) {
            const int c = W + GW * q;
            if (c < r0) {  // uniform guard (scalar branch)
                put(Ts, c, st[q] * iw);
                csq[q] += st[q] * st[q];  // 0 past the split
            }
        }
        if (W == 0) {  // residual and DMX slot entry (wave 0's share)
            const int sl = ok_n ? sl_n : -1;
            const double rr = fr ? (r_n - mean_r) / f_n : r_n;  // (k_resid2: p = lr - mean; rt = p / lf)
            put(Ts, r0, rr * iw);
            put(Ts, vsel(sp >= 0, s0 + sp, DUM), 0.0);
            put(Ts, vsel(sl >= 0, s0 + sl, DUM), x_n * iw);
            sp = sl;
        }
        if (VB) binc = (ok_n && d_n >= 0) ? d_n : -1;
#pragma unroll
        for (int j = 0; j < TA; j++) {
            // trig blocks: harmonic a of A and 8a of B, a = W + GW j (weighted: the rotations
            // below are linear, so they carry the weight along)
            const int a = W + GW * j;
            double ca, sa;
            cpow_u8(c1_n, s1_n, a, ca, sa);
            ca *= iw;
            sa *= iw;
            if (VB) {  // the trig block A of the binned tile
                put(Ts, tA + a, ca);
                put(Ts, tA + 8 + a, sa);
            }
            if (VB && j == 0) {
                double cb, sb;
                cpow_u8(c8_n, s8_n, a, cb, sb);
                // B'' = x [cos 8a theta | sin 8a theta]/sigma (a < 4) in the 8 columns of the
                // row's bin parity, zeros in the other 8
                const bool odd = (d_n & 1) != 0;
                const double vx = (ok_n && d_n >= 0) ? x_n * iw : 0.0;
                put(Ts, vsel(odd, tX + 8 + a, tX + a), vx * cb);
                put(Ts, vsel(odd, tX + 12 + a, tX + 4 + a), vx * sb);
                put(Ts, vsel(odd, tX + a, tX + 8 + a), 0.0);
                put(Ts, vsel(odd, tX + 4 + a, tX + 12 + a), 0.0);
            }
            // Fourier harmonics a + 1 + 8u (<= nred): from the A harmonic by one rotation by
            // e^{i theta}, then by e^{i 8 theta}
            double c = ca, s = sa;
            rot(c, s, c1_n, s1_n);
#pragma unroll
            for (int u = 0; u < HMAX; u++) {
                const int h = a + 8 * u;  // harmonic h + 1 -> columns f0 + 2h (sin), +1 (cos)
                if (FULLH || h < nred) {  // uniform guard
                    put(Ts, f0 + 2 * h, s);
                    put(Ts, f0 + 2 * h + 1, c);
                }
                if (u + 1 < HMAX) rot(c, s, c8_n, s8_n);
            }
        }
    };
    auto mfma = [&](auto Wc, const double* Ts) {
        constexpr int W = decltype(Wc)::value;
#pragma unroll
        for (int ks = 0; ks < KS; ks++) {
            // the row offset of this k-step is laundered through an empty asm so the
            // compiler cannot pair reads of consecutive k-steps (4 doubles apart) into
            // ds_read2_b64: that form is serviced as 16-lane groups banked mod 32, where the
            // column stride CS = 66 puts lanes c and c + 8 on one bank (2-way conflict)
            int roff = (W * KS + ks) * 4;
            asm volatile("" : "+v"(roff));
            const double* Tr = Ts + (lane & 15) * CS + (lane >> 4) + roff;
            double a[NTR], b[NTC];
#pragma unroll
            for (int t = 0; t < NTR; t++) a[t] = Tr[t * 16 * CS];
#pragma unroll
            for (int t = 0; t < NTC; t++) b[t] = Tr[t * 16 * CS];
            int k = 0;
#pragma unroll
            for (int ti = 0; ti < NTR; ti++) {
#pragma unroll
                for (int tj = ti; tj < NTC; tj++, k++) {
                    // rows and columns all DMX slots (the last NSK row tiles, f0 = 16 NTR):
                    // only the DD diagonal (compile-time after unrolling)
                    if (ti >= NTR - NSK && (tj < NTR || VB)) continue;
                    acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ti], b[tj], acc[k], 0, 0, 0);
                }
            }
            // binned DMX x F tile (the weighted trig sums of F^T W F are formed once per pulsar,
            // k_trig_setup: TOA and sigma only)
            if (VB) accB = __builtin_amdgcn_mfma_f64_16x16x4f64(Tr[tA * CS], Tr[tX * CS], accB, 0, 0, 0);
        }
    };
    const long nch = i1 > i0 ? (i1 - i0 + CH - 1) / CH : 0;
    auto chunks = [&](auto Wc) {
        constexpr int W = decltype(Wc)::value;
        if (nch > 0) load(Wc, i0);  // in flight while the buffers are zeroed
        // the slot columns start at 0 (a row writes its own slot entry and clears the previous
        // one); every other column is rewritten each chunk or is padding the epilogue skips
        for (int bf = 0; bf < GVB; bf++)
            for (int k = tid; k < NS * CS; k += NTH) lds[bf * Kpt * CS + s0 * CS + k] = 0.0;
        __syncthreads();
        if constexpr (GVB == 2) {
            if (nch > 0) {
                stage(Wc, Tb0, sp0);
                load(Wc, i0 + CH);
            }
            __syncthreads();
            GVTS(1);
            for (long c = 0; c < nch; c++) {
                const bool odd = c & 1;
                // chunk c+1 into the other buffer (past the last chunk: rows with iw = 0, never read)
                int sp = odd ? sp0 : sp1;
                if (!(dbg & 4)) stage(Wc, odd ? Tb0 : Tb1, sp);
                if (odd) sp0 = sp;
                else sp1 = sp;
                if (!(dbg & 1)) load(Wc, i0 + (c + 2) * CH);
                if (!(dbg & 2)) mfma(Wc, odd ? Tb1 : Tb0);
                __syncthreads();
            }
        } else {
            // one buffer, two workgroups per CU: one's staging and barriers fill the other's gaps
            GVTS(1);
            const long CHS = VB ? 16 : CH;  // row step of a chunk (VB: per quarter)
            for (long c = 0; c < nch; c++) {
                if (!(dbg & 4)) stage(Wc, Tb0, sp0);
                if (!(dbg & 1)) load(Wc, i0 + (c + 1) * CHS);  // past the last chunk: clamped, unused
                __syncthreads();
                if (VB) {
                    // the bins of the wave's 16 rows (staging lanes 16 W ..): the first and the
                    // last row with a bin (bins are contiguous row ranges; the host admits <= 2
                    // per group, of distinct parity)
                    const unsigned long long m = __ballot(binc >= 0);
                    const unsigned mw = (unsigned)((m >> (16 * W)) & 0xffffull);
                    if (mw != 0u) {
                        const int lf = 16 * W + __builtin_ctz(mw), ll = 16 * W + 31 - __builtin_clz(mw);
                        const int bf = __builtin_amdgcn_readlane(binc, lf), bl = __builtin_amdgcn_readlane(binc, ll);
                        VB_ENTER(bf);
                        VB_ENTER(bl);
                    }
                }
                if (!(dbg & 2)) mfma(Wc, Tb0);
                __syncthreads();
            }
        }
    };
    static_assert(GW == 4, "k_gram_v: the chunk loop is dispatched over four waves");
    switch (wave) {
        case 0: chunks(std::integral_constant<int, 0>{}); break;
        case 1: chunks(std::integral_constant<int, 1>{}); break;
        case 2: chunks(std::integral_constant<int, 2>{}); break;
        default: chunks(std::integral_constant<int, 3>{}); break;
    }
    if (VB) {
        if (cur0 >= 0) vb_flush(accB, vbase + (long)(cur0 % NS) * 128, 0, lane);
        if (cur1 >= 0) vb_flush(accB, vbase + (long)(cur1 % NS) * 128, 1, lane);
    }
    GVTS(2);
    // timing-column sums of squares of this split (normalize_designmatrix)
#pragma unroll
    for (int q = 0; q < QL; q++) {
        const int c = wave + GW * q;
        if (c < r0) {
            const double v = wave_sum(csq[q]);
            if (lane == 0) colsq[(I.coff + c) * nsplit + split] = v;
        }
    }
    // sum the waves' partial tiles through LDS, TG tiles at a time, and store them:
    // [T|r] x [T|r|F] -> the Gram partial at (min, max) of the compact columns; slot rows /
    // columns -> this split's DMX partials
    double* G = Gpart + I.goff + (long)split * Kp * Kp;
    double* Sp = Sdp + I.vgoff + (long)split * NS * SW;
    auto cidx = [&](int p) { return p < r0 ? p : (p == r0 ? Kd : r0 + (p - f0)); };
    constexpr int TG = NT < VTG ? NT : VTG;
    double* red = lds;  // [GW][TG][256] (the host sizes LDS for it)
    // only the tiles the MFMAs formed (the all-slot row tiles' skipped tiles hold nothing to
    // store): groups of TG, every thread reducing element tid of each tile of the group; the
    // tile coordinates are compile-time constants after unrolling
    constexpr int NKEPT = [] {
        int c = 0;
        for (int ti = 0; ti < NTR; ti++)
            for (int tj = ti; tj < NTC; tj++)
                if (!(ti >= NTR - NSK && (tj < NTR || VB))) c++;
        return c;
    }();
    int gti[TG], gtj[TG];
    int k = 0, g = 0, kept = 0;
#pragma unroll
    for (int ti = 0; ti < NTR; ti++) {
#pragma unroll
        for (int tj = ti; tj < NTC; tj++, k++) {
            if (ti >= NTR - NSK && (tj < NTR || VB)) continue;
            if (g == 0) __syncthreads();  // the previous group's (or the MFMAs') readers are done
#pragma unroll
            for (int q = 0; q < 4; q++) red[((wave * TG + g) * 4 + q) * 64 + lane] = acc[k][q];
            gti[g] = ti;
            gtj[g] = tj;
            kept++;
            if (g == TG - 1 || kept == NKEPT) {
                __syncthreads();
                const int q = (tid >> 6) & 3, ln = tid & 63;  // NTH = 256: one element per thread
#pragma unroll
                for (int gg = 0; gg < TG; gg++) {
                    if (gg > g) break;
                    double v = 0.0;
#pragma unroll
                    for (int w = 0; w < GW; w++) v += red[((w * TG + gg) * 4 + q) * 64 + ln];
                    const int pr = gti[gg] * 16 + (ln >> 4) + 4 * q, pc = gtj[gg] * 16 + (ln & 15);
                    if (pr > pc || pc >= Wv) continue;
                    const bool rs = pr >= s0, cs = pc >= s0 && pc < f0;
                    if (!rs && !cs) {
                        int a_ = cidx(pr), b_ = cidx(pc);
                        if (a_ > b_) { const int x_ = a_; a_ = b_; b_ = x_; }
                        G[(long)a_ * Kp + b_] = v;
                    } else if (!rs) {
                        Sp[(long)(pc - s0) * SW + cidx(pr)] = v;            // DMX x [T|r]
                    } else if (cs) {
                        // DMX x DMX: diagonal, DD (k_greduce forms it from the TOAs)
                    } else if (!VB) {
                        Sp[(long)(pr - s0) * SW + cidx(pc)] = v;            // DMX x F (VB: binned)
                    }
                }
                g = 0;
            } else {
                g++;
            }
        }
    }
    GVTS(3);
}

// one launch per (row tiles, column tiles) layout; the number of trailing all-slot row tiles
// (whose tiles hold only DD and are skipped) picks the body inside, so layouts that differ
// only in it share the launch (a launch per variant would run their tails one after another)
template <int NTR, int NTC, bool VB>
__device__ __forceinline__ void gram_v_nsk(double* lds, const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                           const double* __restrict__ M, const double* __restrict__ rtime,
                                           const double* __restrict__ dmxv, int nsplit, double* __restrict__ Gpart,
                                           double* __restrict__ Sdp, double* __restrict__ colsq, double* __restrict__ TSp,
                                           double* __restrict__ BFp, int dbg, int nsk, GvResid R) {
    if (nsk <= 0) {  // no all-slot row tile: VB would add a tile and remove none (PsrDev::vb = 0)
        gram_v_body<NTR, NTC, 0, false>(lds, psrs, insts, M, rtime, dmxv, nsplit, Gpart, Sdp, colsq, TSp, BFp, dbg, R);
    } else if constexpr (NTR >= 2) {
        if (nsk == 1) gram_v_body<NTR, NTC, 1, VB>(lds, psrs, insts, M, rtime, dmxv, nsplit, Gpart, Sdp, colsq, TSp, BFp, dbg, R);
        else if constexpr (NTR >= 3) gram_v_body<NTR, NTC, 2, VB>(lds, psrs, insts, M, rtime, dmxv, nsplit, Gpart, Sdp, colsq, TSp, BFp, dbg, R);
    }
}

template <int NTR, int NTC, bool VB>
__global__ __launch_bounds__(GW * 64, GWG) void k_gram_v(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                    const double* __restrict__ M, const double* __restrict__ rtime,
                                                    const double* __restrict__ dmxv, int nsplit,
                                                    double* __restrict__ Gpart, double* __restrict__ Sdp,
                                                    double* __restrict__ colsq, double* __restrict__ TSp,
                                                    double* __restrict__ BFp, int dbg, GvResid R) {
    WgTimer wgt_(WGT_GRAMV);
    extern __shared__ double lds[];
    const PsrDev& Pd = psrs[insts[blockIdx.y].psr];
    const int nsk = __builtin_amdgcn_readfirstlane(NTR - (Pd.red0c + 1 + 15) / 16);
    if constexpr (!VB || NTC <= 6)
        gram_v_nsk<NTR, NTC, VB>(lds, psrs, insts, M, rtime, dmxv, nsplit, Gpart, Sdp, colsq, TSp, BFp, dbg, nsk, R);
}

// k_dm_resid: WidebandDMResiduals (residuals.py:1000-1031) of an instance, one workgroup per
// instance: the modelled DM (timing_model.py:1593 total_dm: DispersionDM.base_dm, a Taylor
// series in Julian years from DMEPOCH, dispersion_model.py:217-234; DispersionDMX.dmx_dm
// :659-678; DispersionJump.jump_dm, -DMJUMP on its TOAs :773-785) at the instance's
// parameters, r = pp_dm - DM; the mean (weights 1/pp_dme^2, unscaled) removed if asked; chi2
// with the scaled errors.  Sums in a fixed order (deterministic).  Bandwidth: ~48 B/TOA.
constexpr int DMR_T = 256;
__global__ __launch_bounds__(DMR_T) void k_dm_resid(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                    const double* __restrict__ tables, int subtract_mean,
                                                    int use_weighted_mean, double* __restrict__ rout,
                                                    double* __restrict__ chi2) {
    __shared__ double sh[DMR_T / 64];
    const InstDev I = insts[blockIdx.x];
    const PsrDev& Pd = psrs[I.psr];
    const int n = I.n;
    double* r = rout + I.ooff;
    if (!Pd.wb) {
        for (int i = threadIdx.x; i < n; i += DMR_T) r[i] = 0.0;
        if (threadIdx.x == 0) chi2[blockIdx.x] = __builtin_nan("");
        return;
    }
    const pint_spec_t& S = *Pd.spec;
    const double* P = tables + I.toff;
    bool any = false;
    for (int k = 1; k < S.ndm; k++) any |= (pval(P, S.o_DM + 2 * k) != 0.0);
    const dd ep = S.o_DMEPOCH >= 0 ? pdd(P, S.o_DMEPOCH) : dd_make(0.0);
    double swr = 0.0, sw = 0.0;
    for (int i = threadIdx.x; i < n; i += DMR_T) {
        double dm = 0.0;
        if (S.ndm > 0) {  // base_dm: Horner in dt (yr), 0 when only DM is nonzero
            const double x = any ? dd_to_d(dd_sub(dd_make(Pd.tdb_hi[i], Pd.tdb_lo[i]), ep)) * INV_DJY : 0.0;
            dm = pval(P, S.o_DM + 2 * (S.ndm - 1));
            for (int k = S.ndm - 1; k >= 1; k--) dm = dm * x * inv_int(k) + pval(P, S.o_DM + 2 * (k - 1));
        }
        if (S.ndmx > 0) {
            const int a = Pd.dmx_a[i], b = Pd.dmx_b[i];
            if (a >= 0) dm += pval(P, S.o_DMX + 2 * a);
            if (b >= 0) dm += pval(P, S.o_DMX + 2 * b);
            if (Pd.dmx_x)
                for (int k = Pd.dmx_x[i]; k < Pd.dmx_x[i + 1]; k++) dm += pval(P, S.o_DMX + 2 * Pd.dmx_x[k]);
        }
        if (S.ndmjump > 0) {
            const uint64_t m = Pd.dmjmask[i];
            for (int k = 0; k < S.ndmjump; k++)
                if ((m >> k) & 1ull) dm -= pval(P, S.o_DMJUMP + 2 * k);
        }
        const double v = Pd.pp_dm[i] - dm;
        r[i] = v;
        if (subtract_mean) {
            const double w = use_weighted_mean ? 1.0 / (Pd.pp_dme[i] * Pd.pp_dme[i]) : 1.0;
            swr += w * v;
            sw += w;
        }
    }
    double mean = 0.0;
    if (subtract_mean) {
        swr = block_sum<DMR_T / 64>(swr, sh);
        sw = block_sum<DMR_T / 64>(sw, sh);
        mean = swr / sw;
    }
    double c2 = 0.0;
    for (int i = threadIdx.x; i < n; i += DMR_T) {  // each thread rereads its own rows
        const double v = r[i] - mean;
        r[i] = v;
        const double z = v / Pd.dm_sig[i];
        c2 += z * z;
    }
    c2 = block_sum<DMR_T / 64>(c2, sh);
    if (threadIdx.x == 0) chi2[blockIdx.x] = c2;
}

// k_wb_gram: the DM rows of WidebandTOAFitter (fitter.py:2465-2637) added to an instance's
// normal equations after k_greduce: the combined design matrix is [M_toa | F; M_dm | 0] with
// M_dm the DM derivatives (Offset 0, DMk dt^k/k!, DMX 1 in its bin, DMJUMP -1 on its TOAs,
// every other column 0; pint_matrix.py:395-439), residuals pp_dm - DM and weights
// 1/sigma_dm^2.  Only the DM-type columns and the residual gain entries: the dense compact
// Gram (DM Taylor / DMJUMP columns x themselves and the residual, r^T W r), their column
// sums of squares (the normalisation, utils.py:2879), and per DMX bin DD += sum w, DCS +=
// count, Sd[.][c] += sum w d_c, Sd[.][res] += sum w r (the bin stays diagonal).  Compact
// layout only (the host checks).  One workgroup per instance; sums in a fixed order.
constexpr int WB_MAXC = 8;  // dense DM-type columns (DM Taylor terms + DMJUMPs)
__device__ __forceinline__ void wb_row(const PsrDev& Pd, const pint_spec_t& S, const double* P, int i, bool any,
                                       dd ep, double& r, double& w, double& dtyr) {
    double dm = 0.0;
    dtyr = S.o_DMEPOCH >= 0 ? dd_to_d(dd_sub(dd_make(Pd.tdb_hi[i], Pd.tdb_lo[i]), ep)) * INV_DJY : 0.0;
    if (S.ndm > 0) {
        const double x = any ? dtyr : 0.0;
        dm = pval(P, S.o_DM + 2 * (S.ndm - 1));
        for (int k = S.ndm - 1; k >= 1; k--) dm = dm * x * inv_int(k) + pval(P, S.o_DM + 2 * (k - 1));
    }
    if (S.ndmx > 0) {
        const int a = Pd.dmx_a[i], b = Pd.dmx_b[i];
        if (a >= 0) dm += pval(P, S.o_DMX + 2 * a);
        if (b >= 0) dm += pval(P, S.o_DMX + 2 * b);
        if (Pd.dmx_x)
            for (int k = Pd.dmx_x[i]; k < Pd.dmx_x[i + 1]; k++) dm += pval(P, S.o_DMX + 2 * Pd.dmx_x[k]);
    }
    if (S.ndmjump > 0) {
        const uint64_t m = Pd.dmjmask[i];
        for (int k = 0; k < S.ndmjump; k++)
            if ((m >> k) & 1ull) dm -= pval(P, S.o_DMJUMP + 2 * k);
    }
    r = Pd.pp_dm[i] - dm;
    const double is = 1.0 / Pd.dm_sig[i];
    w = is * is;
}
__device__ __forceinline__ double wb_deriv(const PsrDev& Pd, int kind, int idx, int i, double dtyr) {
    if (kind == PINT_COL_DM) {  // d_dm_d_DMs (dispersion_model.py:253-275)
        double v = 1.0;
        for (int j = 1; j <= idx; j++) v = v * dtyr * inv_int(j);
        return v;
    }
    return ((Pd.dmjmask[i] >> idx) & 1ull) ? -1.0 : 0.0;  // DMJUMP (:787-795)
}
__global__ __launch_bounds__(256) void k_wb_gram(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                 const double* __restrict__ tables, int nsplit,
                                                 double* __restrict__ Gpart, double* __restrict__ colsq,
                                                 double* __restrict__ Sd, double* __restrict__ DD,
                                                 double* __restrict__ DCS) {
    __shared__ double red[4][(WB_MAXC + 1) * (WB_MAXC + 2) / 2 + WB_MAXC];
    const InstDev I = insts[blockIdx.x];
    const PsrDev& Pd = psrs[I.psr];
    if (!Pd.wb || !Pd.dsplit) return;
    const pint_spec_t& S = *Pd.spec;
    const double* P = tables + I.toff;
    const int n = I.n, Kp = Pd.Kpd, Kres = Pd.Kd;
    // the dense DM-type columns (compact index, kind, index)
    int cc[WB_MAXC], kd[WB_MAXC], ix[WB_MAXC], m = 0;
    for (int c = 0; c < S.ncol && m < WB_MAXC; c++) {
        const int k = S.col_kind[c];
        if ((k == PINT_COL_DM || k == PINT_COL_ZERO) && Pd.cmap[c] >= 0) {
            cc[m] = Pd.cmap[c];
            kd[m] = k;
            ix[m] = S.col_index[c];
            m++;
        }
    }
    bool any = false;
    for (int k = 1; k < S.ndm; k++) any |= (pval(P, S.o_DM + 2 * k) != 0.0);
    const dd ep = S.o_DMEPOCH >= 0 ? pdd(P, S.o_DMEPOCH) : dd_make(0.0);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // (a) dense pairs (i <= j over the m columns and the residual) and column sums of squares
    constexpr int NP = (WB_MAXC + 1) * (WB_MAXC + 2) / 2;
    double acc[NP + WB_MAXC];
#pragma unroll
    for (int p = 0; p < NP + WB_MAXC; p++) acc[p] = 0.0;
    for (int i = tid; i < n; i += 256) {
        double r, w, dtyr;
        wb_row(Pd, S, P, i, any, ep, r, w, dtyr);
        double d[WB_MAXC + 1];
#pragma unroll
        for (int a = 0; a < WB_MAXC; a++) d[a] = a < m ? wb_deriv(Pd, kd[a], ix[a], i, dtyr) : 0.0;
        d[WB_MAXC] = r;
        int p = 0;
#pragma unroll
        for (int a = 0; a <= WB_MAXC; a++)
#pragma unroll
            for (int b = a; b <= WB_MAXC; b++, p++) acc[p] += w * d[a] * d[b];
#pragma unroll
        for (int a = 0; a < WB_MAXC; a++) acc[NP + a] += d[a] * d[a];
    }
#pragma unroll
    for (int p = 0; p < NP + WB_MAXC; p++) {
        const double v = wave_sum(acc[p]);
        if (lane == 0) red[wave][p] = v;
    }
    __syncthreads();
    double* G = Gpart + I.goff;
    if (tid < NP + WB_MAXC) {
        const double v = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
        if (tid < NP) {
            int a = 0, p = tid;  // pair (a, b), a <= b over columns 0..WB_MAXC (WB_MAXC = residual)
            while (p > WB_MAXC - a) { p -= WB_MAXC - a + 1; a++; }
            const int b = a + p;
            const bool va = a < m || a == WB_MAXC, vb = b < m || b == WB_MAXC;
            if (va && vb) {
                int ca = a == WB_MAXC ? Kres : cc[a], cb = b == WB_MAXC ? Kres : cc[b];
                if (ca > cb) { const int t = ca; ca = cb; cb = t; }
                G[(long)ca * Kp + cb] += v;
            }
        } else if (tid - NP < m) {
            colsq[(I.coff + cc[tid - NP]) * nsplit] += v;
        }
    }
    // (b) the DMX bins: one wave per bin
    for (int a = wave; a < Pd.ndc; a += 4) {
        const int k0 = Pd.dptr[a], k1 = Pd.dptr[a + 1];
        double sw = 0.0, cnt = 0.0, swr = 0.0, swd[WB_MAXC];
#pragma unroll
        for (int c = 0; c < WB_MAXC; c++) swd[c] = 0.0;
        for (int k = k0 + lane; k < k1; k += 64) {
            const int i = Pd.didx[k];
            double r, w, dtyr;
            wb_row(Pd, S, P, i, any, ep, r, w, dtyr);
            sw += w;
            cnt += 1.0;
            swr += w * r;
#pragma unroll
            for (int c = 0; c < WB_MAXC; c++) swd[c] += c < m ? w * wb_deriv(Pd, kd[c], ix[c], i, dtyr) : 0.0;
        }
        sw = wave_sum(sw);
        cnt = wave_sum(cnt);
        swr = wave_sum(swr);
#pragma unroll
        for (int c = 0; c < WB_MAXC; c++) swd[c] = wave_sum(swd[c]);
        if (lane == 0) {
            DD[I.ddoff + a] += sw;
            DCS[I.ddoff + a] += cnt;
            double* row = Sd + I.sdoff + (long)a * Kp;
            row[Kres] += swr;
            for (int c = 0; c < m; c++) row[cc[c]] += swd[c];
        }
    }
}

// k_trig_setup + k_trig_sum: the per-pulsar red-noise set-up of every pulsar of an upload in
// two launches (instead of k_redbase, k_trigu, k_trigu_sum, k_trigw, k_trigu_sum per pulsar).
// A job is one pulsar (or, from pint_set_sigma, one pulsar's weighted sums only); a block
// takes TRIG_RB rows of one job, one row per thread per pass:
//   * with `base`, the row's e^{i theta}, e^{i 8 theta} (theta = 2 pi t f_1, dd phase;
//     k_redbase's arithmetic) written to red_cs, else read from it;
//   * A = [cos a theta | sin a theta], B = [cos 8b theta | sin 8b theta] (a, b < 8, by
//     rotations) staged per wave in LDS, and two 16x16 MFMA tiles accumulated: A^T B
//     (unweighted) and A^T (w B) (w = 1/sigma^2);
// the block's two tiles (the waves' tiles summed in a fixed order) go to its partial slot.
// k_trig_sum adds a job's block partials in block order (deterministic) and forms, with
// e^{i(a + 8b) theta} = e^{i a theta} e^{i 8b theta},
//   U_m = T[a][b] - T[8+a][8+b],  V_m = T[8+a][b] + T[a][8+b]   (m = a + 8b)
// of the unweighted tile into trigU (cos, sin sums, TOA only) and of the weighted one into
// trigW (C_m, S_m).
constexpr int TRIG_RB = 1024;  // rows per block (4 per thread)
struct TrigJob {
    const double* tdb_hi;
    const double* tdb_lo;
    const double* isig;
    double* cs;      // red_cs (4 per row)
    double* trigU;   // nullptr: weighted sums only
    double* trigW;
    double f1, f1_lo;
    int n, b0, nb, base;
};

__global__ __launch_bounds__(256) void k_trig_setup(const TrigJob* __restrict__ jobs, int njob,
                                                    double* __restrict__ part) {
    extern __shared__ double xs[];  // per wave 48 * WT_CS: A (0-15), B (16-31), w B (32-47)
    int lo = 0, hi = njob - 1;      // the block's job (jobs sorted by b0)
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (jobs[mid].b0 <= (int)blockIdx.x) lo = mid;
        else hi = mid - 1;
    }
    const TrigJob J = jobs[lo];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r0 = ((int)blockIdx.x - J.b0) * TRIG_RB;
    typedef double __attribute__((address_space(3))) ldsd;
    ldsd* X = (ldsd*)(xs + wave * 48 * WT_CS);
    double4_t au[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, aw[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll 1
    for (int j = 0; j < TRIG_RB / 256; j++) {
        const int i = r0 + (int)threadIdx.x + j * 256;
        double c1 = 1.0, s1 = 0.0, c8 = 1.0, s8 = 0.0, w = 0.0, a0 = 0.0;
        if (i < J.n) {
            if (J.base) {
                const dd x = dd_mul(dd_mul_d(dd_make(J.tdb_hi[i], J.tdb_lo[i]), DAYSEC), dd_make(J.f1, J.f1_lo));
                dd_sincos_cyc(x, &s1, &c1);
                dd_sincos_cyc(dd_make(8.0 * x.hi, 8.0 * x.lo), &s8, &c8);  // 8 theta: exact scaling of the dd phase
                J.cs[4 * i] = c1;
                J.cs[4 * i + 1] = s1;
                J.cs[4 * i + 2] = c8;
                J.cs[4 * i + 3] = s8;
            } else {
                const double4_t zz = ((gptr<double4_t>)J.cs)[i];
                c1 = zz[0];
                s1 = zz[1];
                c8 = zz[2];
                s8 = zz[3];
            }
            w = J.isig[i] * J.isig[i];
            a0 = 1.0;
        }
        double ca = a0, sa = 0.0, cb = 1.0, sb = 0.0;
#pragma unroll
        for (int a = 0; a < 8; a++) {
            X[a * WT_CS + lane] = ca;
            X[(8 + a) * WT_CS + lane] = sa;
            X[(16 + a) * WT_CS + lane] = cb;
            X[(24 + a) * WT_CS + lane] = sb;
            X[(32 + a) * WT_CS + lane] = w * cb;
            X[(40 + a) * WT_CS + lane] = w * sb;
            rot(ca, sa, c1, s1);
            rot(cb, sb, c8, s8);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's stores before its reads
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int ks = 0; ks < 16; ks++) {
            const int row = 4 * ks + (lane >> 4);
            const double av = X[(lane & 15) * WT_CS + row];
            const double bv = X[(16 + (lane & 15)) * WT_CS + row], bw = X[(32 + (lane & 15)) * WT_CS + row];
            au[ks & 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, au[ks & 1], 0, 0, 0);
            aw[ks & 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bw, aw[ks & 1], 0, 0, 0);
        }
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    double* red = xs;  // the waves' tiles summed in a fixed order (acc[q]: D[4q + lane/16][lane%16])
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int e = (4 * q + (lane >> 4)) * 16 + (lane & 15);
        red[wave * 512 + e] = au[0][q] + au[1][q];
        red[wave * 512 + 256 + e] = aw[0][q] + aw[1][q];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 512; e += 256)
        part[(long)blockIdx.x * 512 + e] = (red[e] + red[512 + e]) + (red[1024 + e] + red[1536 + e]);
}

__global__ __launch_bounds__(256) void k_trig_sum(const TrigJob* __restrict__ jobs, const double* __restrict__ part) {
    __shared__ double T[512];
    const TrigJob J = jobs[blockIdx.x];
    for (int e = threadIdx.x; e < 512; e += 256) {
        double v = 0.0;
        for (int b = 0; b < J.nb; b++) v += part[(long)(J.b0 + b) * 512 + e];
        T[e] = v;
    }
    __syncthreads();
    const int m = threadIdx.x & 63, a = m & 7, b = m >> 3, kind = threadIdx.x >> 6;  // kind 0 U, 1 W
    if (kind < 2 && (kind == 1 || J.trigU)) {
        const double* D = T + kind * 256;
        double* o = kind ? J.trigW : J.trigU;
        o[m] = D[a * 16 + b] - D[(8 + a) * 16 + 8 + b];
        o[VTRIG + m] = D[(8 + a) * 16 + b] + D[a * 16 + 8 + b];
    }
}

// Sum the Gram partials of every N-split (+ the ECORR Schur slot) into slot 0, upper
// triangle only, in a fixed order (deterministic), and the column sums of squares.
// vg instances: the Fourier block F^T W F from the pulsar's weighted trig sums (trigW) by the
// product-to-sum identities (a, b = harmonics 1..nred), and past block nbg the DMX bin
// rows Sd, DD, DCS from k_gram_v's slot partials of the N-splits the bin's rows fall in:
//   sin a sin b = (C_|a-b| - C_a+b)/2,  cos a cos b = (C_|a-b| + C_a+b)/2,
//   sin a cos b = (S_a+b + S_a-b)/2     (S_-k = -S_k),
struct GredArgs {
    int nsplit, nparts, compact, vb;
    double* Gpart;
    double* colsq;
    const double* Sdp;
    const double* dmxv;
    double* Sd;
    double* DD;
    double* DCS;
    const double* BFp;
};

// DMX bin a of a vg instance (one wave, lane = lane index): its row Sd (DMX x [T|r|F], from
// the slot partials or the binned VB partials of the N-splits the bin's rows fall in), DD
// and DCS.  Wave-uniform: only wave-level reductions.
__device__ __forceinline__ void gred_bin(const InstDev& I, const PsrDev& Pd, const GredArgs& g, int a, int lane) {
    const int Kp = Pd.Kpd, Kc = Pd.Kd, r0 = Pd.red0c, nsplit = g.nsplit;
    const int SW = Kc + 3;
    const int cnt = Pd.dptr[a + 1] - Pd.dptr[a];
    const long lo = cnt > 0 ? Pd.didx[Pd.dptr[a]] : 0, hi = lo + cnt;
    long per = (I.n + nsplit - 1) / nsplit;
    per = (per + 3) / 4 * 4;
    const int q0 = (int)(lo / per), q1 = cnt > 0 ? (int)((hi - 1) / per) : q0 - 1;
    const double* part = g.Sdp + I.vgoff + (long)(a % Pd.vns) * SW;
    // Every load of the bin is issued before its sums (a bin's rows fall in at most two
    // N-splits but for bins longer than a split, GW wave quarters each): the partials of the
    // lane's two columns for the first two splits and the bin's first GRB_R rows per lane,
    // predicated, then summed in the loops' order (q, then w ascending; rows ascending) -- the
    // same operations in the same order as one dependent load per term, so the same bits
    // (that form waited on each load in turn: ~2 x GW dependent round trips per column).
    constexpr int GRB_R = 4;
    const bool vbp = g.vb && Pd.vb;
    double dcs[2][2 * GW][2];
    bool use[2 * GW];
    long doff[2 * GW];
#pragma unroll
    for (int k = 0; k < 2 * GW; k++) {
        const int q = q0 + k / GW, w = k % GW;
        const long s0_ = (long)q * per, s1_ = min((long)I.n, s0_ + per), len = s1_ - s0_;
        const long QV = (len + VCH - 1) / VCH * 16;
        const long w0 = s0_ + w * QV, w1 = min(s1_, w0 + QV);
        use[k] = q <= q1 && !(w0 >= w1 || hi <= w0 || lo >= w1);  // (a row of the bin in quarter (q, w))
        doff[k] = I.vboff + (((long)q * GW + w) * Pd.vns + a % Pd.vns) * 128;
    }
    double xr[GRB_R], sr[GRB_R];
#pragma unroll
    for (int u = 0; u < GRB_R; u++) {
        const long i = lo + lane + 64 * u;
        xr[u] = i < hi ? g.dmxv[I.ooff + i] : 0.0;
        sr[u] = i < hi ? Pd.isig[i] : 0.0;
    }
#pragma unroll
    for (int t = 0; t < 2; t++) {
        const int c = lane + 64 * t;
        const bool fc = vbp && c >= r0 && c < Kc;
        int e0 = 0, e1 = 0;
        if (fc) {
            const int h = (c - r0) >> 1, k = h + 1, a_ = k & 7, cc = k >> 3;
            const bool isin = ((c - r0) & 1) == 0;
            e0 = isin ? (8 + a_) * 8 + cc : a_ * 8 + cc;
            e1 = isin ? a_ * 8 + 4 + cc : (8 + a_) * 8 + 4 + cc;
        }
#pragma unroll
        for (int k = 0; k < 2 * GW; k++) {
            const bool ld = c <= Kc && (fc ? use[k] : (k % GW == 0 && q0 + k / GW <= q1));
            dcs[t][k][0] = ld ? (fc ? g.BFp[doff[k] + e0] : part[(long)(q0 + k / GW) * Pd.vns * SW + c]) : 0.0;
            dcs[t][k][1] = (ld && fc) ? g.BFp[doff[k] + e1] : 0.0;
        }
    }
#pragma unroll
    for (int t = 0; t < 2; t++) {
        const int c = lane + 64 * t;
        if (c > Kc) break;
        double v = 0.0;
        if (vbp && c >= r0 && c < Kc) {
            // binned DMX x F (k_gram_v VB): the 16x8 blocks D of the (split, wave) quarters
            // the bin's rows touch; harmonic k = a_ + 8 cc: cos = D[a_][cc] - D[8+a_][4+cc],
            // sin = D[8+a_][cc] + D[a_][4+cc]; column r0 + 2h is sin((h+1) theta), +1 cos
            const bool isin = ((c - r0) & 1) == 0;
            const double sg = isin ? 1.0 : -1.0;
#pragma unroll
            for (int k = 0; k < 2 * GW; k++)
                if (use[k]) v += dcs[t][k][0] + sg * dcs[t][k][1];
            for (int q = q0 + 2; q <= q1; q++) {  // (a bin longer than a split: the rest in place)
                const int h = (c - r0) >> 1, kk = h + 1, a_ = kk & 7, cc = kk >> 3;
                const int e0 = isin ? (8 + a_) * 8 + cc : a_ * 8 + cc;
                const int e1 = isin ? a_ * 8 + 4 + cc : (8 + a_) * 8 + 4 + cc;
                const long s0_ = (long)q * per, s1_ = min((long)I.n, s0_ + per), len = s1_ - s0_;
                const long QV = (len + VCH - 1) / VCH * 16;
                for (int w = 0; w < GW; w++) {
                    const long w0 = s0_ + w * QV, w1 = min(s1_, w0 + QV);
                    if (w0 >= w1 || hi <= w0 || lo >= w1) continue;  // no row of the bin here
                    const double* D = g.BFp + I.vboff + (((long)q * GW + w) * Pd.vns + a % Pd.vns) * 128;
                    v += D[e0] + sg * D[e1];
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < 2; k++)
                if (q0 + k <= q1) v += dcs[t][k * GW][0];
            for (int q = q0 + 2; q <= q1; q++) v += part[(long)q * Pd.vns * SW + c];
        }
        g.Sd[I.sdoff + (long)a * Kp + c] = v;
    }
    for (int c = lane + 128; c <= Kc; c += 64) {  // (columns past 128: one load at a time)
        double v = 0.0;
        if (vbp && c >= r0 && c < Kc) {
            const int h = (c - r0) >> 1, k = h + 1, a_ = k & 7, cc = k >> 3;
            const bool isin = ((c - r0) & 1) == 0;
            const int e0 = isin ? (8 + a_) * 8 + cc : a_ * 8 + cc;
            const int e1 = isin ? a_ * 8 + 4 + cc : (8 + a_) * 8 + 4 + cc;
            const double sg = isin ? 1.0 : -1.0;
            for (int q = q0; q <= q1; q++) {
                const long s0_ = (long)q * per, s1_ = min((long)I.n, s0_ + per), len = s1_ - s0_;
                const long QV = (len + VCH - 1) / VCH * 16;
                for (int w = 0; w < GW; w++) {
                    const long w0 = s0_ + w * QV, w1 = min(s1_, w0 + QV);
                    if (w0 >= w1 || hi <= w0 || lo >= w1) continue;
                    const double* D = g.BFp + I.vboff + (((long)q * GW + w) * Pd.vns + a % Pd.vns) * 128;
                    v += D[e0] + sg * D[e1];
                }
            }
        } else {
            for (int q = q0; q <= q1; q++) v += part[(long)q * Pd.vns * SW + c];
        }
        g.Sd[I.sdoff + (long)a * Kp + c] = v;
    }
    // DD = sum (x/sigma)^2 and DCS = sum x^2 over the bin (the whitened DMX column's
    // square norm is the bin's only DMX x DMX entry: k_gram_v skips those tiles)
    double q2 = 0.0, qw = 0.0;
#pragma unroll
    for (int u = 0; u < GRB_R; u++) {
        if (lo + lane + 64 * u < hi) {
            const double xx = xr[u], xw = xx * sr[u];
            q2 += xx * xx;
            qw += xw * xw;
        }
    }
    for (long i = lo + lane + 64 * GRB_R; i < hi; i += 64) {
        const double xx = g.dmxv[I.ooff + i], xw = xx * Pd.isig[i];
        q2 += xx * xx;
        qw += xw * xw;
    }
    q2 = wave_sum(q2);
    qw = wave_sum(qw);
    if (lane == 0) {
        g.DCS[I.ddoff + a] = q2;
        g.DD[I.ddoff + a] = qw;
    }
}

// element e of an instance's Gram (slot 0 <- sum of the N-split partials, upper triangle;
// vg: F^T W F from the trig sums, padding zero) and, for e < Kc, the column sum of squares
__device__ __forceinline__ void gred_elem(const InstDev& I, const PsrDev& Pd, const GredArgs& g, long e) {
    const bool cmp = g.compact && Pd.dsplit;
    const bool vg = cmp && Pd.vg;
    const int Kp = cmp ? Pd.Kpd : I.Kp, Kc = cmp ? Pd.Kd : I.K;
    const int r0 = Pd.red0c;
    const long KK = (long)Kp * Kp;
    if (e < KK) {
        const int i = (int)(e / Kp), j = (int)(e % Kp);
        if (i <= j) {
            double* G = g.Gpart + I.goff;
            if (vg && (j > Kc)) {
                G[e] = 0.0;  // padding
            } else if (vg && i >= r0 && j < Kc) {
                const double* C = Pd.trigW;  // C_m, S_m (k_trig_setup: TOA and sigma only)
                const double* Sn = C + VTRIG;
                const int ha = (i - r0) / 2 + 1, sa = (i - r0) & 1;  // 0 sin, 1 cos
                const int hb = (j - r0) / 2 + 1, sb = (j - r0) & 1;
                const int dm = ha > hb ? ha - hb : hb - ha, sm = ha + hb;
                const double sd = ha >= hb ? Sn[ha - hb] : -Sn[hb - ha];  // S_(a-b), signed
                double v;
                if (sa == 0 && sb == 0) v = 0.5 * (C[dm] - C[sm]);
                else if (sa == 1 && sb == 1) v = 0.5 * (C[dm] + C[sm]);
                else if (sa == 0) v = 0.5 * (Sn[sm] + sd);  // sin a cos b
                else v = 0.5 * (Sn[sm] - sd);               // cos a sin b
                G[e] = v;
            } else {
                // eight independent chains (eight partial loads in flight; a single chain
                // issued one load per add and waited on each: a 195-split single pulsar
                // took 127 us), combined in a fixed tree order (deterministic)
                double a[8] = {G[e], 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
                int q = 1;
                // 32 partial loads in flight per round (a small batch has ~56 splits: one
                // dependent load round per 8 partials was the kernel's latency), summed into
                // the same eight chains in the same order
                for (; q + 32 <= g.nparts; q += 32) {
                    double t[32];
#pragma unroll
                    for (int u = 0; u < 32; u++) t[u] = G[(long)(q + u) * KK + e];
#pragma unroll
                    for (int u = 0; u < 32; u++) a[u & 7] += t[u];
                }
                {
                    // the < 32 remaining partials loaded at once (predicated), then summed in
                    // rounds of eight and a tail into chain 0 as one load at a time would be
                    const int rem = g.nparts - q;
                    double t[31];
#pragma unroll
                    for (int u = 0; u < 31; u++) t[u] = u < rem ? G[(long)(q + u) * KK + e] : 0.0;
#pragma unroll
                    for (int r = 0; r < 3; r++)
                        if (8 * r + 8 <= rem) {
#pragma unroll
                            for (int u = 0; u < 8; u++) a[u] += t[8 * r + u];
                        }
#pragma unroll
                    for (int u = 0; u < 31; u++)
                        if (u >= (rem & ~7) && u < rem) a[0] += t[u];
                }
                G[e] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
            }
        }
    }
    if (e < Kc) {
        double* cs = g.colsq + (I.coff + e) * g.nsplit;
        if (vg && e >= r0) {  // Fourier column: sum sin^2 = (N - U_2h)/2, cos^2 = (N + U_2h)/2
            const double* U = Pd.trigU;  // U_m (k_trig_setup: TOA only)
            const int h = (int)(e - r0) / 2 + 1;
            cs[0] = 0.5 * (U[0] + (((e - r0) & 1) ? U[2 * h] : -U[2 * h]));
        } else {
            double a[4] = {cs[0], 0.0, 0.0, 0.0};
            int q = 1;
            for (; q + 32 <= g.nsplit; q += 32) {  // (as above: same chains, same order)
                double t[32];
#pragma unroll
                for (int u = 0; u < 32; u++) t[u] = cs[q + u];
#pragma unroll
                for (int u = 0; u < 32; u++) a[u & 3] += t[u];
            }
            {
                const int rem = g.nsplit - q;
                double t[31];
#pragma unroll
                for (int u = 0; u < 31; u++) t[u] = u < rem ? cs[q + u] : 0.0;
#pragma unroll
                for (int r = 0; r < 7; r++)
                    if (4 * r + 4 <= rem) {
#pragma unroll
                        for (int u = 0; u < 4; u++) a[u] += t[4 * r + u];
                    }
#pragma unroll
                for (int u = 0; u < 31; u++)
                    if (u >= (rem & ~3) && u < rem) a[0] += t[u];
            }
            cs[0] = (a[0] + a[1]) + (a[2] + a[3]);
        }
    }
}

// Sum the Gram partials of every N-split (+ the ECORR Schur slot) into slot 0, upper
// triangle only, in a fixed order (deterministic), and the column sums of squares.
// vg instances: the Fourier block F^T W F from the pulsar's weighted trig sums (trigW) by the
// product-to-sum identities (a, b = harmonics 1..nred), and past block nbg the DMX bin
// rows Sd, DD, DCS from k_gram_v's slot partials of the N-splits the bin's rows fall in:
//   sin a sin b = (C_|a-b| - C_a+b)/2,  cos a cos b = (C_|a-b| + C_a+b)/2,
//   sin a cos b = (S_a+b + S_a-b)/2     (S_-k = -S_k),
__global__ __launch_bounds__(256) void k_greduce(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                 int nbg, GredArgs g) {
    WgTimer wgt_(WGT_GRED);
    const InstDev I = insts[blockIdx.y];
    const PsrDev& Pd = psrs[I.psr];
    const bool vg = g.compact && Pd.dsplit && Pd.vg;
    if ((int)blockIdx.x >= nbg) {  // DMX bins of a vg instance (one per wave)
        const int a = (blockIdx.x - nbg) * 4 + (threadIdx.x >> 6);
        if (!vg || a >= Pd.ndc) return;  // wave-uniform
        gred_bin(I, Pd, g, a, threadIdx.x & 63);
        return;
    }
    gred_elem(I, Pd, g, (long)blockIdx.x * blockDim.x + threadIdx.x);
}

// PhaseOffset with a frozen PHOFF: the fit has no Offset column, yet the Woodbury chi2
// appends the ones column with Phi = 1e40 (residuals.py:583-585).  Its row of Sigma cannot
// come from the Gram (no column of M is the ones column), so k_onesrow forms it per instance
// before the solve: 1^T W~ F_j and 1^T W~ 1 (W~: ECORR eliminated, as the Gram is), the
// PLRedNoise part from the pulsar's weighted trig sums (F_2h = sin (h+1) theta, F_2h+1 =
// cos), the PLDMNoise modes' (their (1400 MHz / f)^2 scale per TOA has no trig-sum form) as
// weighted sums of their stored columns of M, and the ECORR Schur term from k_ecorr's epoch
// sums.  vg instances take the same row from trig_uwu (no ECORR, no PLDMNoise there).
__device__ __forceinline__ bool ones_virtual(const pint_spec_t& S) { return S.o_PHOFF >= 0 && !S.wb_noones; }

__global__ __launch_bounds__(64) void k_onesrow(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                const double* __restrict__ esum, const double* __restrict__ eD,
                                                const double* __restrict__ eW, const double* __restrict__ eC,
                                                int compact, const double* __restrict__ M, double* __restrict__ ones) {
    const InstDev I = insts[blockIdx.x];
    const PsrDev& Pd = psrs[I.psr];
    const pint_spec_t& S = *Pd.spec;
    if (!ones_virtual(S) || !(S.nred > 0 || Pd.nep > 0)) return;
    const bool cmp = compact && Pd.dsplit;
    const int R = 2 * S.nred, jd = 2 * S.dmn0;  // columns >= jd (< R): PLDMNoise modes
    if (jd < R) {  // sum_i w_i F_ij over the stored DM-noise columns, in a fixed order
        const int n = I.n;
        const double* Fb = M + I.moff + (long)(cmp ? Pd.red0c : S.ncol) * n;
        for (int j = jd; j < R; j++) {
            double acc = 0.0;
            for (int i = threadIdx.x; i < n; i += 64) {
                const double is = Pd.isig[i];
                acc += Fb[(long)j * n + i] * (is * is);
            }
            acc = wave_sum(acc);
            if (threadIdx.x == 0) {
                for (int e = 0; e < Pd.nep; e++) {
                    const double w = eW[I.epoff + e];
                    acc -= w * esum_col(Pd, I, esum, eC, cmp, e, S.ncol + j) / eD[I.epoff + e];
                }
                ones[I.coff + j] = acc;
            }
        }
    }
    for (int j = threadIdx.x; j <= R; j += 64) {
        if (j >= jd && j < R) continue;  // (above)
        double v;
        if (j < R) {
            const int h = j / 2 + 1;
            v = (j & 1) ? Pd.trigW[h] : Pd.trigW[VTRIG + h];
        } else {
            v = Pd.sumw;
        }
        for (int e = 0; e < Pd.nep; e++) {
            const double w = eW[I.epoff + e];
            v -= w * (j < R ? esum_col(Pd, I, esum, eC, cmp, e, S.ncol + j) : w) / eD[I.epoff + e];
        }
        ones[I.coff + j] = v;
    }
}

// ---------------------------------------------------------------------------------
// k_solve: one 1024-thread workgroup per instance, everything in LDS (packed lower
// triangle, K <= 199).  mode 0: WLS (fitter.py:1282-1359: whitened-column normalisation,
// timing columns only); mode 1: GLS (fitter.py:2164-2202 / 1425-1507: unweighted column
// norms, phiinv/norm^2 on the noise columns).
//   left-looking Cholesky (row groups of 16 lanes, shuffle-reduced dot products)
//   -> in-place triangular inverse L^-1 -> xhat = L^-T (L^-1 b) -> cov = L^-T L^-1
// The reference solves the same normal equations with cho_factor/cho_solve (GLSFitter)
// or an SVD (GLSState / WLS on the N x P matrix); for a positive-definite normal matrix
// these give the same solution (SURVEY.md §7 "Linear algebra").
// Also factors the Woodbury Sigma (residuals.py:567-589: U = [F, 1], Phi = [phi, 1e40])
// for k_woodbury.
// ---------------------------------------------------------------------------------
constexpr int SOLVE_T = 1024;
constexpr int RG = 16;             // lanes per row group
constexpr int NGRP = SOLVE_T / RG;  // 64 row groups

__device__ __forceinline__ int tri(int i, int j) { return i * (i + 1) / 2 + j; }
__device__ __forceinline__ double grp_sum(double v) {
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 1, 64);
    return v;
}

// Left-looking Cholesky of packed-lower A in LDS; strict lower part is overwritten by L,
// the diagonal of L goes to D (A's diagonal is left untouched).  Returns 1 if not PD.
__device__ int chol_lds(double* A, double* D, int K, double* tmp) {
    const int g = threadIdx.x / RG, l = threadIdx.x % RG;
    for (int j = 0; j < K; j++) {
        for (int i = j + g; i < K; i += NGRP) {
            double sacc = 0.0;
            for (int k = l; k < j; k += RG) sacc += A[tri(i, k)] * A[tri(j, k)];
            sacc = grp_sum(sacc);
            if (l == 0) tmp[i] = sacc;
        }
        __syncthreads();
        double djj = A[tri(j, j)] - tmp[j];
        if (!(djj > 0.0)) return 1;  // uniform: every thread reads the same LDS values
        double ljj = sqrt(djj);
        for (int i = j + 1 + threadIdx.x; i < K; i += blockDim.x) A[tri(i, j)] = (A[tri(i, j)] - tmp[i]) / ljj;
        if (threadIdx.x == 0) D[j] = ljj;
        __syncthreads();
    }
    return 0;
}

// In-place inverse of the Cholesky factor (strict lower in A, diagonal in D):
// afterwards A's strict lower part holds L^-1 and D holds 1/diag(L).
__device__ void trinv_lds(double* A, double* D, int K, double* tmp) {
    const int g = threadIdx.x / RG, l = threadIdx.x % RG;
    for (int j = K - 1; j >= 0; j--) {
        double dj = D[j];
        for (int i = j + 1 + g; i < K; i += NGRP) {
            // sum_{k=j+1..i} Linv[i][k] * L[k][j]; Linv[i][i] = D[i] (already inverted)
            double sacc = 0.0;
            for (int k = j + 1 + l; k <= i; k += RG) {
                double li = (k == i) ? D[i] : A[tri(i, k)];
                sacc += li * A[tri(k, j)];
            }
            sacc = grp_sum(sacc);
            if (l == 0) tmp[i] = -sacc / dj;
        }
        __syncthreads();
        for (int i = j + 1 + threadIdx.x; i < K; i += blockDim.x) A[tri(i, j)] = tmp[i];
        if (threadIdx.x == 0) D[j] = 1.0 / dj;
        __syncthreads();
    }
}

__device__ __forceinline__ double linv(const double* A, const double* D, int i, int j) {
    return i == j ? D[i] : A[tri(i, j)];
}

__global__ __launch_bounds__(SOLVE_T) void k_solve(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                   const double* __restrict__ tables, const double* __restrict__ Gpart,
                                                   const double* __restrict__ colsq, int nsplit, int nparts, int mode,
                                                   int compact, const double* __restrict__ Sd,
                                                   const double* __restrict__ DD, const double* __restrict__ DCS,
                                                   double* __restrict__ work, double* __restrict__ dpars,
                                                   double* __restrict__ errs, double* __restrict__ cov,
                                                   double* __restrict__ chi2lin, double* __restrict__ sigL,
                                                   int* __restrict__ status, int skip_dsplit, int do_sigma,
                                                   const double* __restrict__ ones) {
    extern __shared__ double lds[];
    __shared__ double sh[SOLVE_T / 64];
    const int inst = blockIdx.x;
    const InstDev I = insts[inst];
    const PsrDev& Pd = psrs[I.psr];
    if (skip_dsplit && compact && Pd.dsplit) return;  // solved by k_solve_dmx
    const pint_spec_t& S = *Pd.spec;
    const int Kfull = I.K, Kp = I.Kp, ncol = S.ncol;
    const int K = (mode == 0) ? ncol : Kfull;  // WLS ignores the noise basis (fitter.py:1965)
    const double* P = tables + I.toff;
    double* A = lds;                        // packed lower K(K+1)/2
    double* D = A + K * (K + 1) / 2;        // K
    double* tmp = D + K;                    // K
    double* bv = tmp + K;                   // K
    double* yv = bv + K;                    // K
    double* nrm = yv + K;                   // K
    const bool cmp = compact && Pd.dsplit;
    const GramView G = gram_view(Pd, I, Gpart, cmp, Sd, DD);  // (partials summed into slot 0 by k_greduce)
    // column norms (utils.py:2879 normalize_designmatrix: zero norm -> 1)
    for (int j = threadIdx.x; j < K; j += blockDim.x) {
        double v;
        if (mode == 0) v = G(j, j);
        else {
            v = colsq_of(Pd, I, colsq, nsplit, cmp, DCS, j);
        }
        v = sqrt(v);
        nrm[j] = (v == 0.0) ? 1.0 : v;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < K * (K + 1) / 2; e += blockDim.x) {
        int i = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
        while (i * (i + 1) / 2 > e) i--;
        while ((i + 1) * (i + 2) / 2 <= e) i++;
        int j = e - i * (i + 1) / 2;
        double v = G(i, j) / (nrm[i] * nrm[j]);
        if (i == j && mode == 1 && i >= ncol) v += 1.0 / Pd.red_phi[i - ncol] / (nrm[i] * nrm[i]);
        A[e] = v;
    }
    for (int j = threadIdx.x; j < K; j += blockDim.x) bv[j] = G(j, Kfull) / nrm[j];
    double rwr = G(Kfull, Kfull);
    __syncthreads();
    if (chol_lds(A, D, K, tmp)) {
        if (threadIdx.x == 0) atomicOr(status, 1 << PINT_E_NOT_PD);
        return;
    }
    trinv_lds(A, D, K, tmp);
    // y = L^-1 b ; xhat = L^-T y   (row-group dot products)
    const int g = threadIdx.x / RG, l = threadIdx.x % RG;
    for (int m = g; m < K; m += NGRP) {
        double sacc = 0.0;
        for (int k = l; k <= m; k += RG) sacc += linv(A, D, m, k) * bv[k];
        sacc = grp_sum(sacc);
        if (l == 0) yv[m] = sacc;
    }
    __syncthreads();
    for (int i = g; i < K; i += NGRP) {
        double sacc = 0.0;
        for (int m = i + l; m < K; m += RG) sacc += linv(A, D, m, i) * yv[m];
        sacc = grp_sum(sacc);
        if (l == 0) tmp[i] = sacc;  // xhat (normalised)
    }
    __syncthreads();
    double bx = 0.0;
    for (int j = threadIdx.x; j < K; j += blockDim.x) {
        bx += bv[j] * tmp[j];
        dpars[I.coff + j] = tmp[j] / nrm[j];
    }
    bx = block_sum<SOLVE_T / 64>(bx, sh);
    if (threadIdx.x == 0) chi2lin[inst] = rwr - bx;
    // cov = L^-T L^-1 / (n n^T): timing block (ncol x ncol, compact), errs for all K
    double* C = cov + (long)I.cvoff;
    const int npair = ncol * (ncol + 1) / 2 + (K - ncol);
    for (int e = threadIdx.x; e < npair; e += blockDim.x) {
        int i, j;
        if (e < ncol * (ncol + 1) / 2) {
            j = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
            while (j * (j + 1) / 2 > e) j--;
            while ((j + 1) * (j + 2) / 2 <= e) j++;
            i = e - j * (j + 1) / 2;  // i <= j
        } else {
            i = j = ncol + (e - ncol * (ncol + 1) / 2);
        }
        double sacc = 0.0;
        for (int m = j; m < K; m++) sacc += linv(A, D, m, i) * linv(A, D, m, j);
        double v = sacc / (nrm[i] * nrm[j]);
        if (j < ncol) {
            C[(long)i * ncol + j] = v;
            C[(long)j * ncol + i] = v;
        }
        if (i == j) errs[I.coff + i] = sqrt(sacc) / nrm[i];
    }
    // Woodbury Sigma = diag(1/Phi) + U^T N^-1 U, U = [F, 1] (ones = F0 * Offset column):
    // factor in LDS, store L^-1 (diag in place) packed to sigL for k_wsolve (unless k_sigma does).
    if (do_sigma && mode == 1 && (S.nred > 0 || Pd.nep > 0)) {
        __syncthreads();
        const int R = 2 * S.nred, Kn = R + 1;
        const double F0 = pval(P, S.o_F);
        double* Sg = lds;
        double* Dg = Sg + Kn * (Kn + 1) / 2;
        double* tg = Dg + Kn;
        for (int e = threadIdx.x; e < Kn * (Kn + 1) / 2; e += blockDim.x) {
            int i = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
            while (i * (i + 1) / 2 > e) i--;
            while ((i + 1) * (i + 2) / 2 <= e) i++;
            int j = e - i * (i + 1) / 2;
            int ci = (i < R) ? ncol + i : 0, cj = (j < R) ? ncol + j : 0;
            double si = (i < R) ? 1.0 : F0, sj = (j < R) ? 1.0 : F0;
            double v;
            if (S.wb_noones && (i == R || j == R)) {
                v = (i == j) ? 1.0 : 0.0;  // no ones column: a decoupled unit row
            } else if (ones && ones_virtual(S) && (i == R || j == R)) {
                v = ones[I.coff + (i == R ? j : i)] + (i == j ? 1e-40 : 0.0);  // k_onesrow (no Offset column)
            } else {
                v = G(ci, cj) * si * sj;
                if (i == j) v += (i < R) ? 1.0 / Pd.red_phi[i] : 1e-40;
            }
            Sg[e] = v;
        }
        __syncthreads();
        if (chol_lds(Sg, Dg, Kn, tg)) {
            if (threadIdx.x == 0) atomicOr(status, 1 << PINT_E_SIGMA);
            return;
        }
        trinv_lds(Sg, Dg, Kn, tg);  // k_wsolve applies L^-1 as a matrix-vector product
        double* L = sigL + (long)I.soff;
        for (int e = threadIdx.x; e < Kn * (Kn + 1) / 2; e += blockDim.x) L[e] = Sg[e];
        __syncthreads();
        for (int i = threadIdx.x; i < Kn; i += blockDim.x) L[tri(i, i)] = Dg[i];
    }
}

// ---------------------------------------------------------------------------------
// k_solve_blk: the same solve, blocked on 16x16 tiles so the work runs on FP64 MFMA and
// the sequential depth is nb = ceil(K/16) block steps instead of K column steps.
//
// LDS holds the lower block triangle of the (padded) normal matrix, each 16x16 block
// column-major with an XOR swizzle (element (r,c) at c*16 + (r ^ (c & 14))), so both the
// plain and the transposed MFMA operand reads, and the accumulator stores, hit distinct
// bank pairs within each half-wave.  Padding rows/columns (K..16*nb-1) are identity.
//   Cholesky, right-looking: wave 0 factors the diagonal block in registers (readlane
//     broadcasts) and overwrites it with L_kk^-1; the panel L_ik = A_ik L_kk^-T and the
//     trailing update A_ij -= L_ik L_jk^T are v_mfma_f64_16x16x4f64 block products
//     spread over the waves;
//   X = L^-1 in place, block row by block row: X_ij = -L_ii^-1 sum_{k=j}^{i-1} L_ik X_kj;
//   covariance C = X^T X (timing block, straight from the accumulators to HBM), errors
//     from the column norms of X, xhat = X^T (X b).
// The Woodbury Sigma of the GLS chi2 is factored by the same routine; its X = L^-1 goes
// to sigL (packed lower incl. diagonal) for k_wsolve.
// ---------------------------------------------------------------------------------
// phase timestamps of workgroup 0 (s_memrealtime, 100 MHz), read by pint_debug_read(.., 4, ..)
__device__ unsigned long long g_ts[32];
#define TS(k) do { if (blockIdx.x == 0 && threadIdx.x == 0) g_ts[k] = __builtin_amdgcn_s_memrealtime(); } while (0)

constexpr int BS_MAXNB = 12;  // 78 blocks x 2 KiB + 2 vectors fit the 160 KiB LDS
constexpr int RSCR = 4 * 512;   // per-instance global scratch of the solves (4 vectors <= 512)

__device__ __forceinline__ int swz(int r, int c) { return (c << 4) + (r ^ (c & 14)); }
__device__ __forceinline__ int lblk(int I, int J) { return ((I * (I + 1)) / 2 + J) << 8; }


// acc(D) += opX(X) opY(Y)^T; X, Y swizzled LDS blocks, TX/TY = read transposed.
// D[(lane>>4)+4q][lane&15] is acc[q].
template <bool TX, bool TY>
__device__ __forceinline__ void bmma(double4_t& acc, const double* X, const double* Y, int lane, bool neg) {
    const int m = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int c = 4 * q + kq;
        double a = TX ? X[swz(c, m)] : X[swz(m, c)];
        double b = TY ? Y[swz(c, m)] : Y[swz(m, c)];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(neg ? -a : a, b, acc, 0, 0, 0);
    }
}
// acc += X Dp, with Dp an accumulator (D layout) used directly as the B operand
__device__ __forceinline__ void bmma_reg(double4_t& acc, const double* X, const double4_t& Dp, int lane) {
    const int m = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int q = 0; q < 4; q++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(X[swz(m, 4 * q + kq)], Dp[q], acc, 0, 0, 0);
}
__device__ __forceinline__ double4_t bload(const double* Z, int lane) {
    double4_t v;
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = Z[swz((lane >> 4) + 4 * q, lane & 15)];
    return v;
}
__device__ __forceinline__ void bstore(double* Z, const double4_t& v, int lane, double s) {
#pragma unroll
    for (int q = 0; q < 4; q++) Z[swz((lane >> 4) + 4 * q, lane & 15)] = s * v[q];
}

// Iterative refinement residuals r = b - A x are accumulated in double-double (two_prod +
// dd_add, error-free): with an extended-precision residual each refinement pass contracts
// the error by ~cond * eps, so one pass takes the error from ~cond * eps to ~(cond * eps)^2 of the FP64
// system even at cond 1e12 -- below the rounding of the reference's own cho_solve.
__device__ __forceinline__ void dd_acc(dd& s, double a, double b) { s = dd_add(s, two_prod(a, b)); }
__device__ __forceinline__ dd dd_quad_sum(dd s) {  // sum over the 4 lanes of a lane quad
    s = dd_add(s, dd_make(__shfl_xor(s.hi, 1, 64), __shfl_xor(s.lo, 1, 64)));
    s = dd_add(s, dd_make(__shfl_xor(s.hi, 2, 64), __shfl_xor(s.lo, 2, 64)));
    return s;
}
__device__ __forceinline__ dd dd_wave_sum(dd s) {  // sum over the 64 lanes of a wave
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s = dd_add(s, dd_make(__shfl_xor(s.hi, o, 64), __shfl_xor(s.lo, o, 64)));
    return s;
}
// the block maxima of two values with one pair of barriers (sh: 2 NW doubles)
template <int NW>
__device__ void block_max2(double* v, double* sh) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        v[0] = fmax(v[0], __shfl_xor(v[0], o, 64));
        v[1] = fmax(v[1], __shfl_xor(v[1], o, 64));
    }
    if constexpr (NW == 1) return;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) {
        sh[w] = v[0];
        sh[NW + w] = v[1];
    }
    __syncthreads();
    double a = sh[0], b = sh[NW];
#pragma unroll
    for (int i = 1; i < NW; i++) {
        a = fmax(a, sh[i]);
        b = fmax(b, sh[NW + i]);
    }
    v[0] = a;
    v[1] = b;
}
constexpr int REFINE_PASSES = 1;
constexpr double REFINE_KAPPA = 1e8;  // refine when the condition estimate exceeds this
template <int NW>
__device__ double block_max(double v, double* sh) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    if constexpr (NW == 1) return v;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) sh[w] = v;
    __syncthreads();
    double t = sh[0];
#pragma unroll
    for (int i = 1; i < NW; i++) t = fmax(t, sh[i]);
    return t;
}

// One wave: Cholesky of the (full, symmetric) 16x16 block in registers (lane r holds row
// r, readlane broadcasts), then its inverse column by column (lane c solves L x = e_c);
// the block is overwritten by L^-1 (zeros above the diagonal).  Returns false if not
// positive definite.
// 1/sqrt(d) as v_rsq_f64 + two Newton steps: within 1 ulp like the library rsqrt (max 0.993
// vs 0.987 ulp over 1e6 pivots in (1e-8, 4]) at 52 instead of 67 cycles of dependent latency
// (bench/rsq_probe.hip); the Cholesky pivot chain is serial, so the latency is what counts
__device__ __forceinline__ double rsq2(double d) {
    double y = __builtin_amdgcn_rsq(d);
    const double h = 0.5 * d;
    y = __builtin_fma(y, __builtin_fma(-h * y, y, 0.5), y);
    return __builtin_fma(y, __builtin_fma(-h * y, y, 0.5), y);
}

// N = 8: a block whose rows and columns 8..15 are identity padding (K <= 8 in a single-block
// solve): only the leading 8 x 8 is factored -- the same operations on it as N = 16 does
// (the padding's updates are exact no-ops), and the padding of L^-1 is identity as stored
template <int N = 16, bool SB = false>
__device__ __forceinline__ bool diag_factor(double* Akk, int lane) {
    const int r = lane & 15;
    // Cholesky (lane r holds row r) and X = L^-1 (lane r its column r) in one pass: pivot j's
    // column L[c][j] is broadcast once (v_readlane) and used by both the trailing update of A
    // and the forward substitution, in axpy order (x[t] -= L[t][u] x[u], u ascending: the
    // same operations and rounding as a separate substitution after the factorisation, with
    // half the lane reads)
    double a[N], x[N];
#pragma unroll
    for (int c = 0; c < N; c++) {
        a[c] = Akk[swz(r, c)];
        x[c] = (r == c) ? 1.0 : 0.0;
    }
    bool ok = true;
#pragma unroll
    for (int j = 0; j < N; j++) {
        const double djj = rdlane(a[j], j);
        ok = ok && (djj > 0.0);
        const double il = rsq2(djj);
        // every lane scales its entry: rows r >= j get L[r][j] (row j: djj il, the same
        // product), rows r < j an upper-triangle value no later pivot reads -- no per-pivot
        // lane masks (the selects' 32 loop-invariant masks were hoisted into SGPRs and
        // spilled to VGPR lanes, ~half the pivot loop's instructions)
        a[j] *= il;
        x[j] *= il;
#pragma unroll
        for (int c = j + 1; c < N; c++) {
            const double Lcj = rdlane(a[j], c);
            a[c] -= a[j] * Lcj;
            x[c] -= Lcj * x[j];
        }
        // right-looking order kept: without the barrier the scheduler sank every column's
        // updates to just before its own pivot (left-looking), a dependent chain of j FMAs
        // ahead of pivot j (and the pivot columns parked in SGPRs spilled to VGPR lanes)
        if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
    }
    if (lane < N) {
#pragma unroll
        for (int t = 0; t < N; t++) Akk[swz(t, r)] = x[t];
    }
    return ok;
}

// (Tried in round 4: a scheduling barrier after each pivot -- 11 % fewer cycles in
// bench/diag_probe.hip (7506 vs 8413), no change inside the solve (3.6 us per block).
// Broadcasting L[.][j] through LDS instead of v_readlane -- 914 instead of
// 1356 instructions and 21 % faster alone (bench/diag_probe.hip), but its VGPR operands do not
// fit the solves' 128-VGPR budget (1024-thread workgroups): 1 KiB/lane of scratch, the solve
// 59 -> 152 us; the same with the inverse on a second wave fed through LDS (variant 6) spilled
// as well.  The readlane form keeps the broadcasts in SGPRs.  A one-step rsqrt (19 ulp)
// moved J0740's unrefined covariance by 1.3e-3 of its scale: also dropped.)

__device__ __forceinline__ void tri_decode(int p, int& i, int& j) {  // p = i(i+1)/2 + j, j <= i
    int ii = (int)((sqrt(8.0 * p + 1.0) - 1.0) * 0.5);
    while (ii * (ii + 1) / 2 > p) ii--;
    while ((ii + 1) * (ii + 2) / 2 <= p) ii++;
    i = ii;
    j = p - ii * (ii + 1) / 2;
}

// Blocked Cholesky + in-place inverse of the nb x nb block lower matrix A in LDS:
// afterwards A holds X = L^-1.  Needs NW >= nb - 1.  Returns false (uniformly) if A is
// not positive definite.
// (Tried in round 4: forming X's block row k - 1 on the waves off wave 0's SIMD while wave 0
// factors diagonal block k, or X's block row k on the waves the trailing update leaves idle --
// the same operations, stored after a barrier -- removed the row loop below (3.3 -> 0.1 us)
// but either way the diagonal factor doubled (3.7 -> 6.9-7.2 us per block, also at k = 0
// where no row is formed: the register allocation of the loop): dropped.)
template <int NW, bool SMALLK = false>
__device__ __forceinline__ bool blk_cholinv(double* A, int nb, int wave, int lane, int* sflag, int K = 1 << 30) {
    for (int k = 0; k < nb; k++) {
        if (k == 0) TS(9);
        if (wave == 0) {
            // (K: the matrix's order, its rows past K identity padding -- a last block of at
            // most 8 rows takes the 8 x 8 factor)
            // (SMALLK: only k_solve_blk instantiates the 8 x 8 form -- compiled into the
            // DMX-eliminated solve as a dead branch it slowed that solve's 16 x 16 factor)
            bool ok = (SMALLK && K - 16 * k <= 8) ? diag_factor<8>(A + lblk(k, k), lane)
                                                 : diag_factor<16>(A + lblk(k, k), lane);
            if (!ok && lane == 0) *sflag = 1;
        }
        if (k == 0) TS(10);
        bsync<NW>();
        if (k == 0) TS(11);
        if (*sflag) return false;
        const double* Lkk = A + lblk(k, k);
        for (int i = k + 1 + wave; i < nb; i += NW) {  // panel: L_ik = A_ik L_kk^-T
            double* Aik = A + lblk(i, k);
            double4_t acc = {0, 0, 0, 0};
            bmma<false, false>(acc, Aik, Lkk, lane, false);
            bstore(Aik, acc, lane, 1.0);
        }
        bsync<NW>();
        if (k == 0) TS(12);
        const int m = nb - k - 1;
        if (m == 0) break;
        for (int p = wave; p < m * (m + 1) / 2; p += NW) {  // trailing: A_ij -= L_ik L_jk^T
            int ii, jj;
            tri_decode(p, ii, jj);
            double* Aij = A + lblk(k + 1 + ii, k + 1 + jj);
            double4_t acc = bload(Aij, lane);
            bmma<false, false>(acc, A + lblk(k + 1 + ii, k), A + lblk(k + 1 + jj, k), lane, true);
            bstore(Aij, acc, lane, 1.0);
        }
        bsync<NW>();
        if (k == 0) TS(13);
    }
    TS(14);
    for (int i = 1; i < nb; i++) {  // X = L^-1, block row i (diagonal blocks already hold L_ii^-1)
        double4_t acc2 = {0, 0, 0, 0};
        const int j = wave;
        if (j < i) {
            double4_t acc = {0, 0, 0, 0};
            for (int k = j; k < i; k++) bmma<false, true>(acc, A + lblk(i, k), A + lblk(k, j), lane, false);
            bmma_reg(acc2, A + lblk(i, i), acc, lane);
        }
        bsync<NW>();
        if (j < i) bstore(A + lblk(i, j), acc2, lane, -1.0);
        bsync<NW>();
        if (i == 1) TS(15);
    }
    TS(16);
    return true;
}

// blk_cholinv with look-ahead (k_solve_dmx): the same operations on the same blocks in the
// same order -- each block's trailing updates T_0..T_k, its panel, its diagonal factor, X's
// block rows -- so the same X, scheduled in two phases per block column k:
//   A: the panels L_ik = A_ik L_kk^-T (i > k) and, on further waves, X's block row k
//      (X_kj = -X_kk sum_{m=j..k-1} L_km X_mj, j < k) in registers;
//   B: wave 0 applies T_k to block (k+1, k+1) and factors it at once while the other waves
//      apply T_k to the rest; X's row k is stored over L's (no longer read).
// Two barriers per block column instead of three, the diagonal factor k+1 beside the rest of
// T_k, and no separate X loop after the factorisation (round 5: 27.6 us for five 16 x 16
// blocks, 4.6 of them X's rows).  Needs NW >= nb - 1.
template <int NW>
__device__ __forceinline__ bool blk_cholinv_la(double* A, int nb, int wave, int lane, int* sflag) {
    TS(9);
    if (wave == 0) {
        const bool ok = diag_factor<16, true>(A, lane);
        if (!ok && lane == 0) *sflag = 1;
    }
    TS(10);
    bsync<NW>();
    TS(11);
    for (int k = 0; k < nb; k++) {
        if (*sflag) return false;  // (uniform: read after a barrier)
        const int npan = nb - k - 1;
        const bool xrow = wave >= npan && wave - npan < k;  // X_kj, j = wave - npan
        double4_t xacc = {0, 0, 0, 0};
        if (wave < npan) {
            double* Aik = A + lblk(k + 1 + wave, k);
            double4_t acc = {0, 0, 0, 0};
            bmma<false, false>(acc, Aik, A + lblk(k, k), lane, false);
            bstore(Aik, acc, lane, 1.0);
        } else if (xrow) {
            const int j = wave - npan;
            double4_t acc = {0, 0, 0, 0};
            for (int m = j; m < k; m++) bmma<false, true>(acc, A + lblk(k, m), A + lblk(m, j), lane, false);
            bmma_reg(xacc, A + lblk(k, k), acc, lane);
        }
        bsync<NW>();
        if (k == 0) TS(12);
        if (xrow) bstore(A + lblk(k, wave - npan), xacc, lane, -1.0);
        if (npan > 0) {
            const int ntr = npan * (npan + 1) / 2;
            if (wave == 0) {
                double* Akk = A + lblk(k + 1, k + 1);
                double4_t acc = bload(Akk, lane);
                bmma<false, false>(acc, A + lblk(k + 1, k), A + lblk(k + 1, k), lane, true);
                bstore(Akk, acc, lane, 1.0);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // (its lanes' stores before its reads)
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const bool ok = diag_factor<16, true>(Akk, lane);
                if (!ok && lane == 0) *sflag = 1;
            } else {
                for (int p = wave; p < ntr; p += NW - 1) {
                    int ii, jj;
                    tri_decode(p, ii, jj);
                    double* Aij = A + lblk(k + 1 + ii, k + 1 + jj);
                    double4_t acc = bload(Aij, lane);
                    bmma<false, false>(acc, A + lblk(k + 1 + ii, k), A + lblk(k + 1 + jj, k), lane, true);
                    bstore(Aij, acc, lane, 1.0);
                }
            }
        }
        bsync<NW>();
        if (k == 0) TS(13);
    }
    TS(14);
    TS(16);
    return true;
}

// U^T W U entry (i, j) of U = [F, 1] (F: sin, cos of harmonics 1..R/2 at 2h, 2h + 1; the ones
// column at R) from the weighted trig sums C_m = sum w cos m theta, S_m (trigW):
//   sin a sin b = (C_|a-b| - C_a+b)/2,  cos a cos b = (C_|a-b| + C_a+b)/2,
//   sin a cos b = (S_a+b + S_a-b)/2,  1 sin b = S_b,  1 cos b = C_b,  1 1 = C_0
__device__ __forceinline__ double trig_uwu(const double* C, int i, int j, int R) {
    const double* Sn = C + VTRIG;
    if (i > j) { const int t = i; i = j; j = t; }
    if (i == R) return C[0];
    const int ha = i / 2 + 1, sa = i & 1;
    if (j == R) return sa ? C[ha] : Sn[ha];
    const int hb = j / 2 + 1, sb = j & 1;
    const int dm = ha > hb ? ha - hb : hb - ha, sm = ha + hb;
    const double sd = ha >= hb ? Sn[ha - hb] : -Sn[hb - ha];
    if (sa == 0 && sb == 0) return 0.5 * (C[dm] - C[sm]);
    if (sa == 1 && sb == 1) return 0.5 * (C[dm] + C[sm]);
    if (sa == 0) return 0.5 * (Sn[sm] + sd);
    return 0.5 * (Sn[sm] - sd);
}

// Woodbury Sigma = diag(1/Phi) + U^T N^-1 U, U = [F, 1] (ones = F0 * Offset column), from
// the (ECORR Schur-reduced) Gram; factored with blk_cholinv in the LDS region A and its
// X = L^-1 stored packed lower (incl. diagonal) to Xout for k_wsolve (residuals.py:567-589).
template <int NW>
__device__ __forceinline__ bool woodbury_sigma(const GramView& G, const PsrDev& Pd, const pint_spec_t& S, double F0, double* A,
                               int wave, int lane, int* sflag, double* Xout, const double* ones) {
    const int ncol = S.ncol, R = 2 * S.nred, Kn = R + 1;
    const int nbs = (Kn + 15) >> 4;
    const int tid = threadIdx.x;
    for (int e = tid; e < nbs * (nbs + 1) / 2 * 256; e += NW * 64) {
        int Ib, Jb;
        tri_decode(e >> 8, Ib, Jb);
        const int r = e & 15, c = (e >> 4) & 15;
        const int gi = Ib * 16 + r, gj = Jb * 16 + c;
        double v;
        if (gi < Kn && gj < Kn) {
            const int ci = (gi < R) ? ncol + gi : 0, cj = (gj < R) ? ncol + gj : 0;
            const double si = (gi < R) ? 1.0 : F0, sj = (gj < R) ? 1.0 : F0;
            if (S.wb_noones && (gi == R || gj == R)) {
                v = (gi == gj) ? 1.0 : 0.0;  // no ones column (PHOFF free): a decoupled unit row
            } else if (!Pd.vg && ones && ones_virtual(S) && (gi == R || gj == R)) {
                v = ones[gi == R ? gj : gi] + (gi == gj ? 1e-40 : 0.0);  // k_onesrow (no Offset column)
            } else {
                // vg: U^T W U from the pulsar's weighted trig sums (U's ones column is the
                // constant column itself, not F0 x the Offset column of M): F^T W F by the
                // product-to-sum identities, 1^T W F_h = S_h / C_h, 1^T W 1 = C_0
                v = Pd.vg ? trig_uwu(Pd.trigW, gi, gj, R) : G(ci, cj) * si * sj;
                if (gi == gj) v += (gi < R) ? 1.0 / Pd.red_phi[gi] : 1e-40;
            }
        } else {
            v = (gi == gj) ? 1.0 : 0.0;
        }
        A[((e >> 8) << 8) + swz(r, c)] = v;
    }
    __syncthreads();
    if (!blk_cholinv<NW>(A, nbs, wave, lane, sflag)) return false;
    for (int e = tid; e < Kn * (Kn + 1) / 2; e += NW * 64) {
        int i, j;
        tri_decode(e, i, j);
        Xout[e] = A[lblk(i >> 4, j >> 4) + swz(i & 15, j & 15)];
    }
    return true;
}

template <int NW>
__global__ __launch_bounds__(NW == 1 ? 256 : NW * 64) void k_solve_blk(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                       const double* __restrict__ tables, const double* __restrict__ Gpart,
                                                       const double* __restrict__ colsq, int nsplit, int mode,
                                                       int compact, const double* __restrict__ Sd,
                                                       const double* __restrict__ DD, const double* __restrict__ DCS,
                                                       double* __restrict__ dpars, double* __restrict__ errs,
                                                       double* __restrict__ cov, double* __restrict__ chi2lin,
                                                       double* __restrict__ sigL, int* __restrict__ status,
                                                       int skip_dsplit, double* __restrict__ rscr, int refine,
                                                       int ninst, int lds_stride) {
    extern __shared__ double lds_all[];
    // NW == 1: four instances per workgroup, a wave each (own LDS region, flag, barriers)
    constexpr int IPB = NW == 1 ? 4 : 1;
    const int wv = IPB > 1 ? (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
    __shared__ int sflags[IPB];
    __shared__ double sh[NW];
    int& sflag = sflags[wv];
    double* lds = lds_all + (long)wv * lds_stride;
    const int inst = blockIdx.x * IPB + wv;
    if (inst >= ninst) return;  // (wave-uniform; NW == 1 only)
    const InstDev I = insts[inst];
    const PsrDev& Pd = psrs[I.psr];
    if (skip_dsplit && compact && Pd.dsplit) return;  // solved by k_solve_dmx
    const pint_spec_t& S = *Pd.spec;
    const int Kfull = I.K, ncol = S.ncol;
    const int K = (mode == 0) ? ncol : Kfull;
    const int nb = (K + 15) >> 4;
    const int nblk = nb * (nb + 1) / 2;
    double* A = lds;
    double* bv = A + nblk * 256;
    double* yv = bv + nb * 16;
    // per-instance vectors in global scratch (the LDS holds the factor and two vectors at
    // nb = 12): reciprocal column norms, the normalised solution, the refinement residual;
    // the one-wave form (nb <= 2) keeps them in its LDS region too (no global round trips)
    double* inv = NW == 1 ? yv + nb * 16 : rscr + (long)inst * RSCR;
    double* xs = NW == 1 ? inv + nb * 16 : inv + RSCR / 4;
    double* rv = NW == 1 ? xs + nb * 16 : xs + RSCR / 4;
    const bool cmp = compact && Pd.dsplit;
    const GramView G = gram_view(Pd, I, Gpart, cmp, Sd, DD);
    const int tid = NW == 1 ? (threadIdx.x & 63) : threadIdx.x, lane = tid & 63;
    const int wave = NW == 1 ? 0 : __builtin_amdgcn_readfirstlane(tid >> 6);
    if (tid == 0) sflag = 0;
    // column norms (utils.py:2879 normalize_designmatrix: zero norm -> 1), as reciprocals
    for (int j = tid; j < nb * 16; j += NW * 64) {
        double v = 1.0;
        if (j < K) {
            v = sqrt(mode == 0 ? G(j, j) : colsq_of(Pd, I, colsq, nsplit, cmp, DCS, j));
            v = v == 0.0 ? 1.0 : v;
        }
        inv[j] = 1.0 / v;
    }
    bsync<NW>();
    // the normalised normal matrix element (i, j < K), built from the Gram in global memory
    auto Aij = [&](int i, int j) {
        double v = G(i, j) * (inv[i] * inv[j]);
        if (i == j && mode == 1 && i >= ncol) v += (inv[i] * inv[i]) / Pd.red_phi[i - ncol];
        return v;
    };
    for (int e = tid; e < nblk * 256; e += NW * 64) {
        int Ib = 0, Jb = 0;
        if (nblk > 1) tri_decode(e >> 8, Ib, Jb);  // (one block: no square root per element)
        const int r = e & 15, c = (e >> 4) & 15;
        const int gi = Ib * 16 + r, gj = Jb * 16 + c;
        const double v = (gi < K && gj < K) ? Aij(gi, gj) : (gi == gj ? 1.0 : 0.0);
        A[((e >> 8) << 8) + swz(r, c)] = v;
    }
    for (int j = tid; j < nb * 16; j += NW * 64) bv[j] = j < K ? G(j, Kfull) * inv[j] : 0.0;
    const double rwr = G(Kfull, Kfull);
    bsync<NW>();
    if (!blk_cholinv<NW, true>(A, nb, wave, lane, &sflag, K)) {
        if (tid == 0) atomicOr(status, 1 << PINT_E_NOT_PD);
        return;
    }
    // covariance of the timing block: C = X^T X / (n n^T)
    {
        const int nbt = (ncol + 15) >> 4;
        double* C = cov + (long)I.cvoff;
        for (int p = wave; p < nbt * (nbt + 1) / 2; p += NW) {
            int bj, bi;
            tri_decode(p, bj, bi);  // bi <= bj
            double4_t acc = {0, 0, 0, 0};
            for (int k = bj; k < nb; k++) bmma<true, true>(acc, A + lblk(k, bi), A + lblk(k, bj), lane, false);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int row = bi * 16 + (lane >> 4) + 4 * q, col = bj * 16 + (lane & 15);
                if (row < ncol && col < ncol) {
                    const double v = acc[q] * (inv[row] * inv[col]);
                    C[(long)row * ncol + col] = v;
                    C[(long)col * ncol + row] = v;
                }
            }
        }
    }
    // errors (all K columns); x = X^T (X b), then one step of iterative refinement
    // x += X^T X (b - A x) with A rebuilt from the Gram: the explicit L^-1 loses ~cond(L)
    // digits that LAPACK's triangular solves (cho_solve, fitter.py:2197) keep, and on a
    // normalised system of cond 1e12 (J0740) that is ~10x the reference's own rounding
    const int g0 = tid >> 2, sub = tid & 3;
    double amax = 0.0, vmax = 0.0;
    for (int g = g0; g < nb * 16; g += NW * 16) {
        const int Jb = g >> 4, cc = g & 15;
        double se = 0.0;
        for (int rr = g + sub; rr < nb * 16; rr += 4) {
            const double x = A[lblk(rr >> 4, Jb) + swz(rr & 15, cc)];
            se += x * x;
        }
        se += __shfl_xor(se, 1, 64);
        se += __shfl_xor(se, 2, 64);
        if (sub == 0 && g < K) {
            errs[I.coff + g] = sqrt(se) * inv[g];
            vmax = fmax(vmax, se);
            amax = fmax(amax, Aij(g, g));
        }
    }
    // refine only where the solve can lose digits (see k_solve_dmx)
    const bool do_ref = refine && block_max<NW>(amax, sh) * block_max<NW>(vmax, sh) > REFINE_KAPPA;
    for (int pass = 0; pass <= REFINE_PASSES; pass++) {
        const double* rhs = pass == 0 ? bv : rv;
        for (int g = g0; g < nb * 16; g += NW * 16) {  // y = X rhs
            const int Jb = g >> 4, cc = g & 15;
            double sy = 0.0;
            for (int c = sub; c <= g; c += 4) sy += A[lblk(Jb, c >> 4) + swz(cc, c & 15)] * rhs[c];
            sy += __shfl_xor(sy, 1, 64);
            sy += __shfl_xor(sy, 2, 64);
            if (sub == 0) yv[g] = sy;
        }
        bsync<NW>();
        for (int g = g0; g < nb * 16; g += NW * 16) {  // x (+)= X^T y
            const int Jb = g >> 4, cc = g & 15;
            double sx = 0.0;
            for (int rr = g + sub; rr < nb * 16; rr += 4) sx += A[lblk(rr >> 4, Jb) + swz(rr & 15, cc)] * yv[rr];
            sx += __shfl_xor(sx, 1, 64);
            sx += __shfl_xor(sx, 2, 64);
            if (sub == 0) xs[g] = (pass == 0 ? 0.0 : xs[g]) + (g < K ? sx : 0.0);
        }
        bsync<NW>();
        if (pass == REFINE_PASSES || !do_ref) break;
        for (int g = g0; g < nb * 16; g += NW * 16) {  // r = b - A x, double-double, a lane quad per row
            dd sa = dd_make(0.0);
            if (g < K)
                for (int j = sub; j < K; j += 4) dd_acc(sa, Aij(g, j), xs[j]);
            sa = dd_quad_sum(sa);
            if (sub == 0) rv[g] = g < K ? dd_to_d(dd_sub(dd_make(bv[g]), sa)) : 0.0;
        }
        bsync<NW>();
    }
    // dpars = x / norm; chi2lin = r^T W r - b^T x (= the minimised linearised chi2)
    double q2 = 0.0;
    for (int g = tid; g < K; g += NW * 64) {
        dpars[I.coff + g] = xs[g] * inv[g];
        q2 += bv[g] * xs[g];
    }
    q2 = block_sum<NW>(q2, sh);
    if (tid == 0) chi2lin[inst] = rwr - q2;
}

// k_solve_lanes<KT>: k_solve_blk's solve for instances of at most KT <= 8 columns (a grid's
// points) with one LANE per instance instead of one wave: 64 instances per wave.  The same
// normalisation, factor and solve, in the same operations per element where the wave form
// reduces over lanes in one order and this one in another (the errors' and covariance's
// sums of squares, the MFMA covariance product, the dot products): the results agree to
// rounding (test_lane_solve_matches_wave_solve).  A wave per 4-column instance ran ~1,240
// wave instructions per point (round 5: 204 us of the 65,536-point NGC6440E grid).
//   A = the normalised normal matrix (fitter.py:1282-1359 WLS / 2164-2202 GLS), L L^T = A by
//   the diagonal factor's per-pivot operations (rsq2; x = L^-1 in axpy order), C = X^T X,
//   x = X^T (X b) with one double-double refinement pass when max diag(A) max diag(A^-1)
//   exceeds REFINE_KAPPA, chi2lin = r^T W r - b^T x.
template <int KT>
__global__ __launch_bounds__(64) void k_solve_lanes(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                    const double* __restrict__ Gpart, const double* __restrict__ colsq,
                                                    int nsplit, int mode, double* __restrict__ dpars,
                                                    double* __restrict__ errs, double* __restrict__ cov,
                                                    double* __restrict__ chi2lin, int* __restrict__ status, int refine,
                                                    int ninst) {
    const int inst = blockIdx.x * 64 + threadIdx.x;
    if (inst >= ninst) return;
    const InstDev I = insts[inst];
    const PsrDev& Pd = psrs[I.psr];
    const pint_spec_t& S = *Pd.spec;
    const int Kfull = I.K, ncol = S.ncol;
    const int K = (mode == 0) ? ncol : Kfull;
    const double* Gp = Gpart + I.goff;
    const int Kp = I.Kp;
    auto G = [&](int i, int j) { return i <= j ? Gp[(long)i * Kp + j] : Gp[(long)j * Kp + i]; };
    double inv[KT], b[KT], a[KT][KT], x[KT][KT];
#pragma unroll
    for (int j = 0; j < KT; j++) {
        double v = 1.0;
        if (j < K) {
            v = sqrt(mode == 0 ? G(j, j) : colsq[(I.coff + j) * nsplit]);
            v = v == 0.0 ? 1.0 : v;
        }
        inv[j] = 1.0 / v;
    }
    auto Aij = [&](int i, int j) {
        double v = G(i, j) * (inv[i] * inv[j]);
        if (i == j && mode == 1 && i >= ncol) v += (inv[i] * inv[i]) / Pd.red_phi[i - ncol];
        return v;
    };
#pragma unroll
    for (int i = 0; i < KT; i++) {
        b[i] = i < K ? G(i, Kfull) * inv[i] : 0.0;
#pragma unroll
        for (int j = 0; j < KT; j++) {
            a[i][j] = (i < K && j < K) ? Aij(i, j) : (i == j ? 1.0 : 0.0);
            x[i][j] = (i == j) ? 1.0 : 0.0;
        }
    }
    const double rwr = G(Kfull, Kfull);
    // Cholesky and X = L^-1 (diag_factor's per-pivot operations: row r of the wave form is a[r])
    bool ok = true;
#pragma unroll
    for (int j = 0; j < KT; j++) {
        const double djj = a[j][j];
        ok = ok && (djj > 0.0);
        const double il = rsq2(djj);
#pragma unroll
        for (int r = 0; r < KT; r++) {
            a[r][j] = (r == j) ? djj * il : (r > j ? a[r][j] * il : 0.0);
            x[r][j] *= il;
        }
#pragma unroll
        for (int c = j + 1; c < KT; c++) {
            const double Lcj = a[c][j];
#pragma unroll
            for (int r = 0; r < KT; r++) {
                a[r][c] -= a[r][j] * Lcj;
                x[r][c] -= Lcj * x[r][j];
            }
        }
    }
    if (!ok) {
        atomicOr(status, 1 << PINT_E_NOT_PD);
        return;
    }
    // x[r][t] = (L^-1)[t][r] (lane r of the wave form held column r of X): X[t][r] = x[r][t]
    // covariance of the timing block C = X^T X / (n n^T)
    double* C = cov + (long)I.cvoff;
    double amax = 0.0, vmax = 0.0;
#pragma unroll
    for (int r = 0; r < KT; r++) {
#pragma unroll
        for (int c = r; c < KT; c++) {
            if (r < ncol && c < ncol) {
                double acc = 0.0;
#pragma unroll
                for (int m = 0; m < KT; m++) acc += x[r][m] * x[c][m];
                const double v = acc * (inv[r] * inv[c]);
                C[(long)r * ncol + c] = v;
                C[(long)c * ncol + r] = v;
            }
        }
        if (r < K) {
            double se = 0.0;
#pragma unroll
            for (int m = 0; m < KT; m++) se += x[r][m] * x[r][m];
            errs[I.coff + r] = sqrt(se) * inv[r];
            vmax = fmax(vmax, se);
            amax = fmax(amax, Aij(r, r));
        }
    }
    const bool do_ref = refine && amax * vmax > REFINE_KAPPA;
    double xs[KT], rv[KT];
#pragma unroll
    for (int pass = 0; pass <= REFINE_PASSES; pass++) {
        double yv[KT];
#pragma unroll
        for (int g = 0; g < KT; g++) {  // y = X rhs
            double sy = 0.0;
#pragma unroll
            for (int c = 0; c <= g; c++) sy += x[c][g] * (pass == 0 ? b[c] : rv[c]);
            yv[g] = sy;
        }
#pragma unroll
        for (int g = 0; g < KT; g++) {  // x (+)= X^T y
            double sx = 0.0;
#pragma unroll
            for (int rr = g; rr < KT; rr++) sx += x[g][rr] * yv[rr];
            xs[g] = (pass == 0 ? 0.0 : xs[g]) + (g < K ? sx : 0.0);
        }
        if (pass == REFINE_PASSES || !do_ref) break;
#pragma unroll
        for (int g = 0; g < KT; g++) {  // r = b - A x in double-double
            dd sa = dd_make(0.0);
            if (g < K)
                for (int j = 0; j < K; j++) dd_acc(sa, Aij(g, j), xs[j]);
            rv[g] = g < K ? dd_to_d(dd_sub(dd_make(b[g]), sa)) : 0.0;
        }
    }
    double q2 = 0.0;
#pragma unroll
    for (int g = 0; g < KT; g++) {
        if (g < K) {
            dpars[I.coff + g] = xs[g] * inv[g];
            q2 += b[g] * xs[g];
        }
    }
    chi2lin[inst] = rwr - q2;
}

// ---------------------------------------------------------------------------------
// k_solve_dmx: the normal equations of the compact fit layout with the DMX block
// eliminated.  In the normalised system A = [A_dd A_dx; A_xd D] the DMX-DMX block D is
// diagonal (a TOA lies in at most one free bin), so
//   S = A_dd - A_dx D^-1 A_xd = A_dd - U U^T,  U = A_dx D^-1/2       (rank-ndc update, MFMA)
//   x_d = S^-1 (b_d - U D^-1/2 b_x),  x_x = D^-1 b_x - D^-1/2 U^T x_d
//   C_dd = S^-1 = X^T X (X = L_S^-1),  W = X U,
//   C_xd = -D^-1/2 W^T X,  C_xx = D^-1 + D^-1/2 W^T W D^-1/2.
// This is the same solution and covariance as the dense solve of A (fitter.py:2196-2202
// cho_factor/cho_solve); only the Cholesky depth shrinks from ceil(K/16) to ceil(Kd/16).
// LDS: S (lower blocks) and U (nbd x nbk blocks), then W in place of U.
// ---------------------------------------------------------------------------------
constexpr int SD_MAXBLK = 76;  // S + U blocks (2 KiB each) that fit next to the vectors

__device__ __forceinline__ int ublk(int I, int k, int nbk, int nblkS) { return (nblkS + I * nbk + k) << 8; }

// The timing covariance (ncol x ncol, original order) of the DMX-eliminated solve from X =
// L_S^-1 (lower blocks of A) and W = X U (U blocks): C_dd = X^T X, C_xx = D^-1 + D^-1/2 W^T W
// D^-1/2, C_xd = -D^-1/2 W^T X; block pairs w0, w0 + ws, ... (wave-uniform)
__device__ __forceinline__ void cov_dmx_blocks(const double* A, const double* ind, const double* inx, const double* isd,
                                               const double* Dn, const PsrDev& Pd, double* __restrict__ C, int ncol,
                                               int red0, int ndc, int nbd, int nbk, int nblkS, int w0, int ws, int lane) {
    const int nbt = (red0 + 15) >> 4;  // dense timing columns: compact 0..red0-1
    const int nd_pairs = nbt * (nbt + 1) / 2, nx_pairs = nbk * (nbk + 1) / 2, ndx = nbk * nbt;
    for (int p = w0; p < nd_pairs + nx_pairs + ndx; p += ws) {
        double4_t acc = {0, 0, 0, 0};
        int kind, bi, bj;
        if (p < nd_pairs) {  // C_dd = X^T X
            kind = 0;
            tri_decode(p, bj, bi);
            for (int k = bj; k < nbd; k++) bmma<true, true>(acc, A + lblk(k, bi), A + lblk(k, bj), lane, false);
        } else if (p < nd_pairs + nx_pairs) {  // (W^T W)_ab
            kind = 1;
            tri_decode(p - nd_pairs, bj, bi);
            for (int k = 0; k < nbd; k++)
                bmma<true, true>(acc, A + ublk(k, bi, nbk, nblkS), A + ublk(k, bj, nbk, nblkS), lane, false);
        } else {  // (W^T X)_{a c}: DMX block bi x dense block bj
            kind = 2;
            const int q = p - nd_pairs - nx_pairs;
            bi = q / nbt;
            bj = q % nbt;
            for (int k = bj; k < nbd; k++)
                bmma<true, true>(acc, A + ublk(k, bi, nbk, nblkS), A + lblk(k, bj), lane, false);
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int ri = bi * 16 + (lane >> 4) + 4 * q, cj = bj * 16 + (lane & 15);
            int oi, oj;
            double v;
            if (kind == 0) {
                if (ri >= red0 || cj >= red0) continue;
                oi = Pd.dorig[ri];
                oj = Pd.dorig[cj];
                v = acc[q] * (ind[ri] * ind[cj]);
            } else if (kind == 1) {
                if (ri >= ndc || cj >= ndc) continue;
                oi = Pd.xorig[ri];
                oj = Pd.xorig[cj];
                v = acc[q] * (isd[ri] * isd[cj]) + (ri == cj ? 1.0 / Dn[ri] : 0.0);
                v *= inx[ri] * inx[cj];
            } else {
                if (ri >= ndc || cj >= red0) continue;
                oi = Pd.xorig[ri];
                oj = Pd.dorig[cj];
                v = -acc[q] * isd[ri] * (inx[ri] * ind[cj]);
            }
            C[(long)oi * ncol + oj] = v;
            C[(long)oj * ncol + oi] = v;
        }
    }
}

// W = X U in place of U (X = L_S^-1 in the lower blocks of A, U in the nbd x nbk U blocks):
// (block row Ib, block column kb) pairs in rounds of NW waves, block rows descending: a
// round's products have read their U blocks before its W blocks are stored, and a later
// round (smaller or equal Ib, other pairs) never reads a block stored earlier
template <int NW>
__device__ __forceinline__ void w_from_xu(double* A, int nbd, int nbk, int nblkS, int wave, int lane) {
    const int npair = nbd * nbk;
    for (int r = 0; r < npair; r += NW) {
        const int p = r + wave, Ib = nbd - 1 - p / nbk, kb = p % nbk;
        double4_t acc = {0, 0, 0, 0};
        if (p < npair)
            for (int Jb = 0; Jb <= Ib; Jb++)
                bmma<false, true>(acc, A + lblk(Ib, Jb), A + ublk(Jb, kb, nbk, nblkS), lane, false);
        __syncthreads();
        if (p < npair) bstore(A + ublk(Ib, kb, nbk, nblkS), acc, lane, 1.0);
    }
}

// the DMX parameters' errors: sqrt of C_xx's diagonal D^-1 + D^-1 |W_a|^2 (normalised), a lane
// quad per DMX column (W in the U blocks of A)
template <int NW>
__device__ __forceinline__ void dmx_errors(const double* A, const double* inx, const double* Dn, const PsrDev& Pd,
                                           double* __restrict__ errs, int ndc, int nbd, int nbk, int nblkS) {
    const int g0 = threadIdx.x >> 2, sub = threadIdx.x & 3;
    for (int a = g0; a < ndc; a += NW * 16) {
        double sw = 0.0;
        for (int rr = sub; rr < nbd * 16; rr += 4) {
            const double w = A[ublk(rr >> 4, a >> 4, nbk, nblkS) + swz(rr & 15, a & 15)];
            sw += w * w;
        }
        sw += __shfl_xor(sw, 1, 64);
        sw += __shfl_xor(sw, 2, 64);
        if (sub == 0) errs[Pd.xorig[a]] = sqrt(1.0 / Dn[a] + sw / Dn[a]) * inx[a];
    }
}

// pint_fit_step_apply: k_apply's work inside the solve -- tables += lam * step (dd, timing
// columns, Offset skipped) and the instance's constants of the updated table -- so a GLS step
// (lambda 1) needs no apply launch.  The spec header and the table are staged in LDS beyond
// the solve's own data when the kernel starts (their loads overlap the build), each step
// element updates its table entry where it is written (LDS and HBM), and after the solve every
// thread calls inst_setup_wave (which synchronises the block) on the staged copy: no global
// round trip after the step.  The staging region: PREP_HDR + tstride + 16 doubles, then the
// constants
static inline size_t apply_tail_lds(int tstride) {
    return sizeof(double) * ((size_t)PREP_HDR + tstride + 16) + sizeof(InstConst) + 16;
}
template <int NW>
__device__ __forceinline__ void apply_stage(const PsrDev& Pd, const InstDev& I, const double* tables, double* tail) {
    const double* hg = reinterpret_cast<const double*>(Pd.spec);
    const int ts = Pd.spec->tstride;
    const double* P = tables + I.toff;
    for (int i = threadIdx.x; i < PREP_HDR; i += NW * 64) tail[i] = hg[i];
    for (int i = threadIdx.x; i < ts; i += NW * 64) tail[PREP_HDR + i] = P[i];
}
// a column's step dp: the staged (LDS) and the HBM table entry o (the column's col_toff)
// += lam * dp in double-double
__device__ __forceinline__ void apply_col(double* __restrict__ P, double* tailP, int o, double dp, double lam) {
    if (o < 0 || lam == 0.0) return;
    const dd v = dd_add_d(dd_make(tailP[o], tailP[o + 1]), lam * dp);
    tailP[o] = v.hi;
    tailP[o + 1] = v.lo;
    P[o] = v.hi;
    P[o + 1] = v.lo;
}
// wave 0 only (the other waves export the solve meanwhile); the staged table complete (the
// caller's block barrier after the step writes)
// (not inlined: the setup's code stays out of the solve's hot loops -- inlined it grew the
// kernel by ~10k instructions and its register spills)
__device__ __attribute__((noinline)) void apply_setup(int inst, double* tail, int ts, InstConst* __restrict__ ic) {
    double* sx = tail + PREP_HDR + ts;
    InstConst* sC = reinterpret_cast<InstConst*>(sx + 16);
    const int lane = threadIdx.x;
    TS(22);
    inst_setup_wave(*reinterpret_cast<const pint_spec_t*>(tail), tail + PREP_HDR, *sC, sx, lane);
    TS(23);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int* cs = reinterpret_cast<const int*>(sC);
    int* cd = reinterpret_cast<int*>(ic + inst);
    for (int k = lane; k < (int)(sizeof(InstConst) / 4); k += 64) cd[k] = cs[k];
}

// k_schur: k_solve_dmx's build phase for deferred solves (xw), spread over the chip -- the
// norms (utils.py:2879), S = A_dd and U = A_dx D^-1/2 normalised, S -= U U^T and b'_d = b_d -
// U D^-1/2 b_x -- one 256-thread workgroup per (lower block of S, instance), each staging the
// U block rows it needs in LDS.  At 9 pulsars the same work inside the one-workgroup-per-
// instance solve took ~16 us of its ~63 (profiles: solve phases, round 4).  The operations
// and their order are the solve's own (wave 0 runs the block's MFMA chain in k order, b'_d
// by the same lane quads), so the solve that loads the result gives the same bits.
// Output per instance at xw + xwoff: the S' blocks and U blocks in the solve's LDS layout,
// then ind (nbd*16), inx, isd, Dn (nbk*16 each) -- k_cov_dmx's export layout -- then b'_d
// (nbd*16), b_x (nbk*16) and the normalised Gram diagonal rd (nbd*16).
constexpr int SCHUR_T = 256;
__global__ __launch_bounds__(SCHUR_T) void k_schur(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                   const double* __restrict__ Gpart, const double* __restrict__ colsq,
                                                   int nsplit, int mode, const double* __restrict__ Sd,
                                                   const double* __restrict__ DD, const double* __restrict__ DCS,
                                                   double* __restrict__ xw) {
    WgTimer wgt_(WGT_SCHUR);
    extern __shared__ double lds[];
    const InstDev I = insts[blockIdx.y];
    const PsrDev& Pd = psrs[I.psr];
    if (!Pd.dsplit) return;
    const int ndc = Pd.ndc, Kp = Pd.Kpd, Kres = Pd.Kd;
    const int Kd = (mode == 0) ? Pd.red0c : Pd.Kd;
    const int red0 = Pd.red0c;
    const int nbd = (Kd + 15) >> 4, nbk = (ndc + 15) >> 4;
    const int nblkS = nbd * (nbd + 1) / 2;
    const int p = blockIdx.x;
    if (p >= nblkS) return;
    int Ib, Jb;
    tri_decode(p, Ib, Jb);
    const bool diag = Ib == Jb;
    const double* Gp = Gpart + I.goff;
    const double* Sdi = Sd + I.sdoff;
    auto Gd = [&](int i, int j) {
        if (i > j) { int t = i; i = j; j = t; }
        return Gp[(long)i * Kp + j];
    };
    double* uI = lds;                               // nbk blocks: U(Ib, k)
    double* uJ = diag ? uI : uI + nbk * 256;        // nbk blocks: U(Jb, k)
    double* inx = uI + (diag ? 1 : 2) * nbk * 256;  // nbk*16
    double* isd = inx + nbk * 16;                   // nbk*16
    double* Dn = isd + nbk * 16;                    // nbk*16
    double* bx = Dn + nbk * 16;                     // nbk*16
    double* indI = bx + nbk * 16;                   // 16: rows of Ib
    double* indJ = indI + 16;                       // 16: rows of Jb
    const int tid = threadIdx.x, lane = tid & 63;
    // ---- every global load of the workgroup issued first (one load latency, not one per
    //      phase): the DMX norms' inputs, the two row blocks' column norms, the U elements,
    //      the S block's Gram entries and b_d's ----
    constexpr int URB = 8;  // U elements per thread and row block held in registers (nbk <= 8)
    const int nrow = diag ? 1 : 2;
    double gU[2][URB];
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
        for (int u = 0; u < URB; u++) {
            const int e = tid + u * SCHUR_T, r = e & 15, a = e >> 4;
            const int gi = (t == 0 ? Ib : Jb) * 16 + r;
            gU[t][u] = (t < nrow && e < nbk * 256 && gi < Kd && a < ndc) ? Sdi[(long)a * Kp + gi] : 0.0;
        }
    double gD = 0.0, gC = 0.0, gB = 0.0, gN = 0.0, gS[4] = {0, 0, 0, 0}, gb = 0.0;
    if (tid < nbk * 16 && tid < ndc) {
        gD = DD[I.ddoff + tid];
        gC = mode == 0 ? gD : DCS[I.ddoff + tid];
        gB = Sdi[(long)tid * Kp + Kres];
    }
    if (tid >= 128 && tid < 160) {
        const int c = ((tid - 128) < 16 ? Ib : Jb) * 16 + ((tid - 128) & 15);
        if (c < Kd) gN = mode == 0 ? Gd(c, c) : colsq[(I.coff + c) * nsplit];
    }
    if (tid < 64) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int gi = Ib * 16 + (lane >> 4) + 4 * q, gj = Jb * 16 + (lane & 15);
            if (gi < Kd && gj < Kd) gS[q] = Gd(gi, gj);
        }
    } else if (diag && tid < 128) {
        const int c = Ib * 16 + ((tid - 64) >> 2);
        if (c < Kd) gb = Gd(c, Kres);
    }
    // ---- norms (the solve's formulas) ----
    for (int a = tid; a < nbk * 16; a += SCHUR_T) {
        double d = 1.0, b = 0.0, na = 1.0;
        if (a < ndc) {
            const double dd_ = a == tid ? gD : DD[I.ddoff + a];
            na = sqrt(a == tid ? gC : (mode == 0 ? dd_ : DCS[I.ddoff + a]));
            na = na == 0.0 ? 1.0 : na;
            d = dd_ / (na * na);
            b = (a == tid ? gB : Sdi[(long)a * Kp + Kres]) / na;
        }
        inx[a] = 1.0 / na;
        Dn[a] = d;
        isd[a] = 1.0 / sqrt(d);
        bx[a] = b;
    }
    if (tid >= 128 && tid < 160) {
        const int k = tid - 128, c = (k < 16 ? Ib : Jb) * 16 + (k & 15);
        double v = 1.0;
        if (c < Kd) {
            v = sqrt(gN);
            v = v == 0.0 ? 1.0 : v;
        }
        (k < 16 ? indI : indJ)[k & 15] = 1.0 / v;
    }
    __syncthreads();
    // ---- U block rows Ib (and Jb), scaled: U[gi][a] = A_dx[gi][a] ind[gi] inx[a] isd[a] ----
#pragma unroll
    for (int t = 0; t < 2; t++) {
        if (t >= nrow) break;
        const double* ind = t == 0 ? indI : indJ;
        double* u = t == 0 ? uI : uJ;
        const int B = t == 0 ? Ib : Jb;
#pragma unroll
        for (int uu = 0; uu < URB; uu++) {
            const int e = tid + uu * SCHUR_T, r = e & 15, a = e >> 4;
            if (e < nbk * 256) {
                const int gi = B * 16 + r;
                u[((a >> 4) << 8) + swz(r, a & 15)] = (gi < Kd && a < ndc) ? gU[t][uu] * (ind[r] * inx[a]) * isd[a] : 0.0;
            }
        }
        for (int e = tid + URB * SCHUR_T; e < nbk * 256; e += SCHUR_T) {  // (nbk > URB: the tail)
            const int r = e & 15, a = e >> 4, gi = B * 16 + r;
            const double g = (gi < Kd && a < ndc) ? Sdi[(long)a * Kp + gi] : 0.0;
            u[((a >> 4) << 8) + swz(r, a & 15)] = (gi < Kd && a < ndc) ? g * (ind[r] * inx[a]) * isd[a] : 0.0;
        }
    }
    __syncthreads();
    double* o = xw + I.xwoff;
    const int na = (nblkS + nbd * nbk) * 256;
    double* o_ind = o + na;
    double* o_inx = o_ind + nbd * 16;
    double* o_isd = o_inx + nbk * 16;
    double* o_Dn = o_isd + nbk * 16;
    double* o_bd = o_Dn + nbk * 16;
    double* o_bx = o_bd + nbd * 16;
    double* o_rd = o_bx + nbk * 16;
    if (tid < 64) {
        // the S block (the solve's put_S) and S -= sum_k U(Ib,k) U(Jb,k)^T in k order
        double4_t acc;
        const int c = lane & 15;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int r = (lane >> 4) + 4 * q;
            const int gi = Ib * 16 + r, gj = Jb * 16 + c;
            double v;
            if (gi < Kd && gj < Kd) {
                const double ni = indI[r], nj = indJ[c];
                v = gS[q] * (ni * nj);
                if (gi == gj) o_rd[gi] = v;
                if (gi == gj && mode == 1 && gi >= red0) v += (ni * ni) / Pd.red_phi[gi - red0];
            } else {
                v = (gi == gj) ? 1.0 : 0.0;
            }
            acc[q] = v;
        }
        for (int k = 0; k < nbk; k++) bmma<false, false>(acc, uI + k * 256, uJ + k * 256, lane, true);
        double* So = o + ((long)p << 8);
#pragma unroll
        for (int q = 0; q < 4; q++) So[swz((lane >> 4) + 4 * q, lane & 15)] = acc[q];
    } else if (diag && tid < 128) {
        // b'_d of the block's rows, by the solve's lane quads: b_d - sum_a U[c][a] (b_x[a] isd[a])
        const int l = tid - 64, cr = l >> 2, sub = l & 3;
        const int c = Ib * 16 + cr;
        double sacc = 0.0;
        for (int a = sub; a < ndc; a += 4) sacc += uI[((a >> 4) << 8) + swz(cr, a & 15)] * (bx[a] * isd[a]);
        sacc += __shfl_xor(sacc, 1, 64);
        sacc += __shfl_xor(sacc, 2, 64);
        const double bd = c < Kd ? gb * indI[cr] : 0.0;
        if (sub == 0) o_bd[c] = bd - sacc;
    } else if (diag) {
        // the block row's U blocks and norms; workgroup 0 the DMX vectors
        const int t0 = tid - 128;
        for (int e = t0; e < nbk * 256; e += SCHUR_T - 128) o[ublk(Ib, e >> 8, nbk, nblkS) + (e & 255)] = uI[e];
        if (t0 < 16) o_ind[Ib * 16 + t0] = indI[t0];
        if (p == 0)
            for (int a = t0; a < nbk * 16; a += SCHUR_T - 128) {
                o_inx[a] = inx[a];
                o_isd[a] = isd[a];
                o_Dn[a] = Dn[a];
                o_bx[a] = bx[a];
            }
    }
}
static inline size_t schur_lds(int nbk) { return sizeof(double) * ((size_t)2 * nbk * 256 + 4 * nbk * 16 + 32); }
static inline long schur_xw_extra(long nbd, long nbk) { return (2 * nbd + nbk) * 16; }

template <int NW>
__global__ __launch_bounds__(NW * 64) void k_solve_dmx(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                       const double* __restrict__ tables, const double* __restrict__ Gpart,
                                                       const double* __restrict__ colsq, int nsplit, int mode,
                                                       const double* __restrict__ Sd, const double* __restrict__ DD,
                                                       const double* __restrict__ DCS, double* __restrict__ dpars,
                                                       double* __restrict__ errs, double* __restrict__ cov,
                                                       double* __restrict__ chi2lin, double* __restrict__ sigL,
                                                       int* __restrict__ status, int fuse_sigma, int refine,
                                                       double* __restrict__ xw, const double* __restrict__ ones,
                                                       double* __restrict__ apply_tables, InstConst* __restrict__ apply_ic,
                                                       double apply_lam, int pre, int la_chol) {
    WgTimer wgt_(WGT_SOLVE);
    extern __shared__ double lds[];
    __shared__ int sflag;
    __shared__ double sh[2 * NW];  // block_sum / block_max2
    if (fuse_sigma && (int)blockIdx.x >= (int)gridDim.x / 2) {
        // the Woodbury Sigma factor (k_sigma's work) in the second half of the grid, so it
        // runs concurrently with the solves without a second stream
        const InstDev I = insts[blockIdx.x - gridDim.x / 2];
        const PsrDev& Pd = psrs[I.psr];
        const pint_spec_t& S = *Pd.spec;
        if (!(S.nred > 0 || Pd.nep > 0)) return;
        if (threadIdx.x == 0) sflag = 0;
        __syncthreads();
        const int lane = threadIdx.x & 63;
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const GramView G = gram_view(Pd, I, Gpart, Pd.dsplit != 0, Sd, DD);
        // F0 scales the stored Offset column only (not on the vg path, whose ones column
        // comes from the trig sums).  With the fused apply the other half of this grid
        // rewrites the tables, so F0 must not be read then: the host fuses only all-vg
        // batches, and an instance that breaks that invariant fails here instead of racing.
        if (apply_tables && !Pd.vg) {
            if (threadIdx.x == 0) atomicOr(status, 1 << PINT_E_SIGMA);
            return;
        }
        const double F0 = Pd.vg ? 0.0 : pval(tables + I.toff, S.o_F);
        if (!woodbury_sigma<NW>(G, Pd, S, F0, lds, wave, lane, &sflag, sigL + (long)I.soff,
                                ones ? ones + I.coff : nullptr))
            if (threadIdx.x == 0) atomicOr(status, 1 << PINT_E_SIGMA);
        return;
    }
    const int inst = blockIdx.x;
    const InstDev I = insts[inst];
    const PsrDev& Pd = psrs[I.psr];
    if (!Pd.dsplit) return;  // full layout: k_solve_blk / k_solve
    const pint_spec_t& S = *Pd.spec;
    const int ncol = S.ncol, ndc = Pd.ndc, Kp = Pd.Kpd, Kres = Pd.Kd;
    const int Kd = (mode == 0) ? Pd.red0c : Pd.Kd;  // dense columns in the solve (WLS: no noise basis)
    const int red0 = Pd.red0c;
    const int nbd = (Kd + 15) >> 4, nbk = (ndc + 15) >> 4;
    const int nblkS = nbd * (nbd + 1) / 2;
    double* A = lds;                                  // S blocks, then U/W blocks
    double* bd = A + (nblkS + nbd * nbk) * 256;       // nbd*16: b_d, then b'_d
    double* yv = bd + nbd * 16;                       // nbd*16
    double* bx = yv + nbd * 16;                       // nbk*16: b_x (normalised)
    double* Dn = bx + nbk * 16;                       // nbk*16: normalised D
    double* ind = Dn + nbk * 16;                      // nbd*16: 1 / dense column norms
    double* inx = ind + nbd * 16;                     // nbk*16: 1 / DMX column norms
    double* isd = inx + nbk * 16;                     // nbk*16: 1 / sqrt(normalised D)
    double* xd = isd + nbk * 16;                      // nbd*16: normalised x_d (refinement)
    double* xx = xd + nbd * 16;                       // nbk*16: normalised x_x
    double* rd = xx + nbk * 16;                       // nbd*16: residual r_d
    double* rx = rd + nbd * 16;                       // nbk*16: residual r_x
    double* tail = rx + nbk * 16;                     // pint_fit_step_apply: spec header, table, setup
    const double* Gp = Gpart + I.goff;
    const double* Sdi = Sd + I.sdoff;
    auto Gd = [&](int i, int j) {  // dense compact Gram (upper storage)
        if (i > j) { int t = i; i = j; j = t; }
        return Gp[(long)i * Kp + j];
    };
    // reciprocal norms (and D^-1/2), staged in LDS below: the per-element scalings are
    // multiplications
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (tid == 0) sflag = 0;
    TS(0);
    if (apply_tables) apply_stage<NW>(Pd, I, apply_tables, tail);
    const double rwr = Gd(Kres, Kres);
    if (pre) {
        // k_schur formed S' = S - U U^T, U, the norms and b'_d in xw (its layout): load them
        const double* o = xw + I.xwoff;
        const int na = (nblkS + nbd * nbk) * 256;
        copy_in<NW * 64, 16>(A, o, na, tid);
        const double* v = o + na;
        for (int e = tid; e < nbd * 16; e += NW * 64) {
            ind[e] = v[e];
            bd[e] = v[nbd * 16 + 3 * nbk * 16 + e];
            rd[e] = v[2 * nbd * 16 + 4 * nbk * 16 + e];
        }
        for (int e = tid; e < nbk * 16; e += NW * 64) {
            inx[e] = v[nbd * 16 + e];
            isd[e] = v[nbd * 16 + nbk * 16 + e];
            Dn[e] = v[nbd * 16 + 2 * nbk * 16 + e];
            bx[e] = v[2 * nbd * 16 + 3 * nbk * 16 + e];
        }
        __syncthreads();
        TS(1);
    } else {
    // ---- loads first: each thread's Gram (S) and DMX-row (U) elements are issued before the
    //      norms and held in registers across them, so building S and U costs one global-load
    //      latency instead of one per phase (systems larger than RS / RU elements per thread
    //      load the rest in the tail loops) ----
    constexpr int RS = 4, RU = 12;
    const int nS = nblkS * 256, nU = nbd * nbk * 256;
    double gS[RS], gU[RU];
#pragma unroll
    for (int u = 0; u < RS; u++) {
        const int e = tid + u * NW * 64;
        gS[u] = 0.0;
        if (e < nS) {
            int Ib, Jb;
            tri_decode(e >> 8, Ib, Jb);
            const int gi = Ib * 16 + (e & 15), gj = Jb * 16 + ((e >> 4) & 15);
            if (gi < Kd && gj < Kd) gS[u] = Gd(gi, gj);
        }
    }
#pragma unroll
    for (int u = 0; u < RU; u++) {
        const int e = tid + u * NW * 64;
        const int blk = e >> 8, Ib = blk / nbk, kb = blk % nbk;
        const int gi = Ib * 16 + (e & 15), a = kb * 16 + ((e >> 4) & 15);
        gU[u] = (e < nU && gi < Kd && a < ndc) ? Sdi[(long)a * Kp + gi] : 0.0;
    }
    // b_d's Gram entries (one column per thread), not after the barrier
    const double gb_pre = tid < Kd ? Gd(tid, Kres) : 0.0;
    // ---- column norms (utils.py:2879: zero norm -> 1), b_x, D (normalised) ----
    for (int c = tid; c < nbd * 16; c += NW * 64) {
        double v = 1.0;
        if (c < Kd) {
            v = sqrt(mode == 0 ? Gd(c, c) : colsq[(I.coff + c) * nsplit]);
            v = v == 0.0 ? 1.0 : v;
        }
        ind[c] = 1.0 / v;
    }
    for (int a = tid; a < nbk * 16; a += NW * 64) {
        double d = 1.0, b = 0.0, na = 1.0;
        if (a < ndc) {
            const double dd_ = DD[I.ddoff + a];
            na = sqrt(mode == 0 ? dd_ : DCS[I.ddoff + a]);
            na = na == 0.0 ? 1.0 : na;
            d = dd_ / (na * na);
            b = Sdi[(long)a * Kp + Kres] / na;
        }
        inx[a] = 1.0 / na;
        Dn[a] = d;
        isd[a] = 1.0 / sqrt(d);
        bx[a] = b;
    }
    __syncthreads();
    // ---- build S = A_dd, U = A_dx D^-1/2, b_d ----
    // the normalised Gram diagonal, for the condition estimate's max diag(A), parked in rd
    // (the refinement's residual, unused until then) instead of a register held across the
    // register-hungry Cholesky
    auto put_S = [&](int e, double g) {
        int Ib, Jb;
        tri_decode(e >> 8, Ib, Jb);
        const int r = e & 15, c = (e >> 4) & 15;
        const int gi = Ib * 16 + r, gj = Jb * 16 + c;
        double v;
        if (gi < Kd && gj < Kd) {
            const double ni = ind[gi], nj = ind[gj];
            v = g * (ni * nj);
            if (gi == gj) rd[gi] = v;
            if (gi == gj && mode == 1 && gi >= red0) v += (ni * ni) / Pd.red_phi[gi - red0];
        } else {
            v = (gi == gj) ? 1.0 : 0.0;
        }
        A[((e >> 8) << 8) + swz(r, c)] = v;
    };
    auto put_U = [&](int e, double g) {
        const int blk = e >> 8, Ib = blk / nbk, kb = blk % nbk;
        const int r = e & 15, c = (e >> 4) & 15;
        const int gi = Ib * 16 + r, a = kb * 16 + c;
        A[ublk(Ib, kb, nbk, nblkS) + swz(r, c)] = (gi < Kd && a < ndc) ? g * (ind[gi] * inx[a]) * isd[a] : 0.0;
    };
#pragma unroll
    for (int u = 0; u < RS; u++)
        if (tid + u * NW * 64 < nS) put_S(tid + u * NW * 64, gS[u]);
    for (int e = tid + RS * NW * 64; e < nS; e += NW * 64) {  // tail
        int Ib, Jb;
        tri_decode(e >> 8, Ib, Jb);
        const int gi = Ib * 16 + (e & 15), gj = Jb * 16 + ((e >> 4) & 15);
        put_S(e, (gi < Kd && gj < Kd) ? Gd(gi, gj) : 0.0);
    }
#pragma unroll
    for (int u = 0; u < RU; u++)
        if (tid + u * NW * 64 < nU) put_U(tid + u * NW * 64, gU[u]);
    for (int e = tid + RU * NW * 64; e < nU; e += NW * 64) {  // tail
        const int blk = e >> 8, Ib = blk / nbk, kb = blk % nbk;
        const int gi = Ib * 16 + (e & 15), a = kb * 16 + ((e >> 4) & 15);
        put_U(e, (gi < Kd && a < ndc) ? Sdi[(long)a * Kp + gi] : 0.0);
    }
    if (tid < nbd * 16) bd[tid] = tid < Kd ? gb_pre * ind[tid] : 0.0;
    __syncthreads();
    TS(1);
    // ---- S -= U U^T (lower blocks), b'_d = b_d - U D^-1/2 b_x ----
    for (int p = wave; p < nblkS; p += NW) {
        int Ib, Jb;
        tri_decode(p, Ib, Jb);
        double4_t acc = bload(A + lblk(Ib, Jb), lane);
        for (int k = 0; k < nbk; k++)
            bmma<false, false>(acc, A + ublk(Ib, k, nbk, nblkS), A + ublk(Jb, k, nbk, nblkS), lane, true);
        bstore(A + lblk(Ib, Jb), acc, lane, 1.0);
    }
    TS(27);
    if (blockIdx.x == 0 && tid == 14 * 64) g_ts[29] = __builtin_amdgcn_s_memrealtime();  // (ts probe: wave 14)
    {
        // (8 lanes per row counted from the idle last wave, two chains each, measured no
        // faster: the phase is bound by the CU's MFMA issue, 15 blocks x 32 MFMAs on 4 SIMDs)
        const int g0 = tid >> 2, sub = tid & 3;
        double bnew = 0.0;
        for (int c = g0; c < nbd * 16; c += NW * 16) {
            double sacc = 0.0;
            for (int a = sub; a < ndc; a += 4)
                sacc += A[ublk(c >> 4, a >> 4, nbk, nblkS) + swz(c & 15, a & 15)] * (bx[a] * isd[a]);
            sacc += __shfl_xor(sacc, 1, 64);
            sacc += __shfl_xor(sacc, 2, 64);
            bnew = bd[c] - sacc;
        }
        TS(28);
        __syncthreads();
        if (sub == 0 && g0 < nbd * 16) bd[g0] = bnew;  // NW*16 >= nbd*16 groups
    }
    __syncthreads();
    }  // (build)
    TS(2);
    if (!(la_chol ? blk_cholinv_la<NW>(A, nbd, wave, lane, &sflag) : blk_cholinv<NW>(A, nbd, wave, lane, &sflag))) {
        if (tid == 0) atomicOr(status, 1 << PINT_E_NOT_PD);
        if (xw) {  // no X/W to export: the deferred covariance of this instance comes out NaN,
                   // not from the previous step's (or uninitialised) export
            double* o = xw + I.xwoff + (nblkS + nbd * nbk) * 256;
            for (int e = tid; e < nbd * 16; e += NW * 64) o[e] = __builtin_nan("");
            for (int e = tid; e < 3 * nbk * 16; e += NW * 64) o[nbd * 16 + e] = __builtin_nan("");
        }
        return;
    }
    TS(3);
    // the steps' and errors' bookkeeping loads (original column indices, b_d's Gram entry),
    // issued here so their latency passes under y and x_d (one column per thread: Kd, ndc
    // <= 16 BS_MAXNB <= NW 64)
    static_assert(16 * BS_MAXNB <= NW * 64, "k_solve_dmx: one dense / DMX column per thread");
    const int h0 = tid >> 3, hs = tid & 7;
    const int od_t = tid < Kd ? Pd.dorig[tid] : 0;       // the step loop's column (g = tid)
    const int ox_t = tid < ndc ? Pd.xorig[tid] : 0;      // ... and DMX column (a = tid)
    const double gb_t = tid < Kd ? Gd(tid, Kres) : 0.0;
    const int od_h = h0 < Kd ? Pd.dorig[h0] : 0;         // the x_d loop's column (g = h0)
    // ---- y = X b'_d ----
    const int g0 = tid >> 2, sub = tid & 3;
    for (int g = g0; g < nbd * 16; g += NW * 16) {
        double sy = 0.0;
        for (int c = sub; c <= g; c += 4) sy += A[lblk(g >> 4, c >> 4) + swz(g & 15, c & 15)] * bd[c];
        sy += __shfl_xor(sy, 1, 64);
        sy += __shfl_xor(sy, 2, 64);
        if (sub == 0) yv[g] = sy;
    }
    // the table offsets of the step loop's columns (pint_fit_step_apply)
    const int to_d = (apply_tables && tid < Kd && od_t < ncol) ? S.col_toff[od_t] : -1;
    const int to_x = (apply_tables && tid < ndc) ? S.col_toff[ox_t] : -1;
    // the step needs only z = W^T y = U^T X^T y = U^T x_d, so U stays in LDS as it is: W = X U
    // (for the DMX errors and the covariance) is formed after the step, here or -- deferred
    // solves (xw) -- by k_cov_dmx at the read, off the step's critical path; both orders give
    // the same bits
    __syncthreads();
    TS(4);
    // ---- x_d = X^T y ; errors of the dense columns (8 lanes per column: one round of
    //      groups, ~10-long chains instead of ~20 with lane quads) ----
    double vmax = 0.0, amax = 0.0;  // max diag(A^-1), max diag(A) (from the build, in rd)
    for (int g = h0; g < Kd; g += NW * 8) {
        double s1 = 0.0, se = 0.0;
        for (int rr = g + hs; rr < nbd * 16; rr += 8) {
            const double x = A[lblk(rr >> 4, g >> 4) + swz(rr & 15, g & 15)];
            s1 += x * yv[rr];
            se += x * x;
        }
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) {
            s1 += __shfl_xor(s1, o, 64);
            se += __shfl_xor(se, o, 64);
        }
        if (hs == 0) {
            xd[g] = s1;
            errs[I.coff + (g == h0 ? od_h : Pd.dorig[g])] = sqrt(se) * ind[g];  // (g = h0: the first round of groups)
            vmax = fmax(vmax, se);
            amax = fmax(amax, rd[g]);
        }
    }
    // the DMX entries of diag(A^-1) are (1 + |W_a|^2) / d >= 1 / d: the estimate stays a
    // lower bound without W.  Both maxima are reduced here, over the barrier x_d needs anyway
    for (int a = tid; a < ndc; a += NW * 64) {
        const double d = Dn[a];
        vmax = fmax(vmax, 1.0 / d);
        amax = fmax(amax, d);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        vmax = fmax(vmax, __shfl_xor(vmax, o, 64));
        amax = fmax(amax, __shfl_xor(amax, o, 64));
    }
    if (lane == 0) {
        sh[wave] = amax;
        sh[NW + wave] = vmax;
    }
    __syncthreads();  // x_d and the maxima visible: z = U^T x_d below
    TS(25);
    {
        double a_ = sh[0], b_ = sh[NW];
#pragma unroll
        for (int i = 1; i < NW; i++) {
            a_ = fmax(a_, sh[i]);
            b_ = fmax(b_, sh[NW + i]);
        }
        amax = a_;
        vmax = b_;
    }
    // ---- z = U^T x_d, x_x = D^-1 b_x - D^-1/2 z ----
    for (int a = h0; a < ndc; a += NW * 8) {
        double sz = 0.0;
        for (int rr = hs; rr < Kd; rr += 8) sz += A[ublk(rr >> 4, a >> 4, nbk, nblkS) + swz(rr & 15, a & 15)] * xd[rr];
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) sz += __shfl_xor(sz, o, 64);
        if (hs == 0) xx[a] = bx[a] / Dn[a] - sz * isd[a];
    }
    // refine only where the solve can lose digits: kappa >= max diag(A) max diag(A^-1)
    // (a lower bound of cond(A)); measured, the unrefined error is ~1e-17 kappa sigma
    // (PTA pulsars kappa 1e5..1e7: <= 3e-12 sigma; J0740 7e12: 8e-5 sigma)
    const bool do_ref = refine && amax * vmax > REFINE_KAPPA;
    TS(26);
    __syncthreads();  // x_x visible (and the maxima read before block_sum reuses sh)
    // ---- iterative refinement: r = b - A x with A from the Gram in global memory (dd
    // residual), then the same Schur solve of r (b'' = r_d - A_dx D^-1 r_x, y = X b'', dx_d =
    // X^T y, dx_x = D^-1 r_x - D^-1/2 W^T y with W^T y = U^T dx_d).  The explicit
    // L^-1 loses ~cond(L) digits that LAPACK's triangular solves keep (cho_solve,
    // fitter.py:2197) ----
    auto Ad = [&](int i, int j) {
        double v = Gd(i, j) * (ind[i] * ind[j]);
        if (i == j && mode == 1 && i >= red0) v += (ind[i] * ind[i]) / Pd.red_phi[i - red0];
        return v;
    };
    TS(17);
    for (int pass = 0; do_ref && pass < REFINE_PASSES; pass++) {
        // r_d = b_d - A_dd x_d - A_dx x_x and r_x = b_x - A_xd x_d - D x_x in double-double,
        // a lane quad per row: every row's loads are in flight at once
        for (int c = g0; c < Kd + ndc; c += NW * 16) {
            dd sa = dd_make(0.0);
            if (c < Kd) {
                for (int j = sub; j < Kd; j += 4) dd_acc(sa, Ad(c, j), xd[j]);
                for (int a = sub; a < ndc; a += 4) dd_acc(sa, Sdi[(long)a * Kp + c] * (ind[c] * inx[a]), xx[a]);
            } else {
                const int a = c - Kd;
                for (int j = sub; j < Kd; j += 4) dd_acc(sa, Sdi[(long)a * Kp + j] * (ind[j] * inx[a]), xd[j]);
                if (sub == 0) dd_acc(sa, Dn[a], xx[a]);
            }
            sa = dd_quad_sum(sa);
            if (sub == 0) {
                if (c < Kd) rd[c] = dd_to_d(dd_sub(dd_make(Gd(c, Kres) * ind[c]), sa));
                else rx[c - Kd] = dd_to_d(dd_sub(dd_make(bx[c - Kd]), sa));
            }
        }
        __syncthreads();
        TS(18);
        for (int c = g0; c < nbd * 16; c += NW * 16) {
            double sa = 0.0;
            if (c < Kd)
                for (int a = sub; a < ndc; a += 4) sa += Sdi[(long)a * Kp + c] * (ind[c] * inx[a]) * (rx[a] / Dn[a]);
            sa += __shfl_xor(sa, 1, 64);
            sa += __shfl_xor(sa, 2, 64);
            if (sub == 0) bd[c] = c < Kd ? rd[c] - sa : 0.0;
        }
        __syncthreads();
        TS(19);
        for (int g = g0; g < nbd * 16; g += NW * 16) {
            double sy = 0.0;
            for (int c = sub; c <= g; c += 4) sy += A[lblk(g >> 4, c >> 4) + swz(g & 15, c & 15)] * bd[c];
            sy += __shfl_xor(sy, 1, 64);
            sy += __shfl_xor(sy, 2, 64);
            if (sub == 0) yv[g] = sy;
        }
        __syncthreads();
        TS(20);
        for (int g = g0; g < Kd; g += NW * 16) {
            double s1 = 0.0;
            for (int rr = g + sub; rr < nbd * 16; rr += 4) s1 += A[lblk(rr >> 4, g >> 4) + swz(rr & 15, g & 15)] * yv[rr];
            s1 += __shfl_xor(s1, 1, 64);
            s1 += __shfl_xor(s1, 2, 64);
            if (sub == 0) {
                xd[g] += s1;
                rd[g] = s1;  // dx_d (rd is consumed): U^T dx_d below
            }
        }
        __syncthreads();
        for (int a = g0; a < ndc; a += NW * 16) {
            double sz = 0.0;
            for (int rr = sub; rr < Kd; rr += 4) sz += A[ublk(rr >> 4, a >> 4, nbk, nblkS) + swz(rr & 15, a & 15)] * rd[rr];
            sz += __shfl_xor(sz, 1, 64);
            sz += __shfl_xor(sz, 2, 64);
            if (sub == 0) xx[a] += rx[a] / Dn[a] - sz * isd[a];
        }
        __syncthreads();
    }
    TS(21);
    // ---- steps (par units), chi2lin = r^T W r - b . x ----
    double bx_dot = 0.0;
    double* Papp = apply_tables ? apply_tables + I.toff : nullptr;
    // (one column per thread; the column indices, their table offsets and b_d's Gram entry
    // loaded before)
    if (tid < Kd) {
        const int g = tid;
        const double v = xd[g] * ind[g];
        dpars[I.coff + od_t] = v;
        bx_dot += gb_t * ind[g] * xd[g];
        if (Papp && od_t < ncol) apply_col(Papp, tail + PREP_HDR, to_d, v, apply_lam);
    }
    if (tid < ndc) {
        const int a = tid;
        const double v = xx[a] * inx[a];
        dpars[I.coff + ox_t] = v;
        bx_dot += bx[a] * xx[a];
        if (Papp) apply_col(Papp, tail + PREP_HDR, to_x, v, apply_lam);
    }
    bx_dot = block_sum<NW>(bx_dot, sh);  // (its barriers also complete the staged table's updates)
    if (tid == 0) chi2lin[inst] = rwr - bx_dot;
    TS(5);
    // pint_fit_step_apply: the updated table's constants on wave 0, beside the export
    const bool setup_w0 = apply_tables && xw;
    if (setup_w0 && wave == 0) apply_setup(inst, tail, S.tstride, apply_ic);
    // ---- covariance of the timing parameters ----
    if (xw) {  // deferred to k_cov_dmx (several workgroups per instance, at the read): X, U
        double* o = xw + I.xwoff;
        // (after k_schur the U blocks and the scalings are in xw already: X alone)
        const int na = pre ? nblkS * 256 : (nblkS + nbd * nbk) * 256;
        const int t0 = setup_w0 ? tid - 64 : tid, ts_ = setup_w0 ? (NW - 1) * 64 : NW * 64;
        if (t0 >= 0 && pre) {
            for (int e = t0; e < na; e += ts_) o[e] = A[e];
        } else if (t0 >= 0) {
            for (int e = t0; e < na; e += ts_) o[e] = A[e];
            for (int e = t0; e < nbd * 16; e += ts_) o[na + e] = ind[e];
            for (int e = t0; e < nbk * 16; e += ts_) {
                o[na + nbd * 16 + e] = inx[e];
                o[na + nbd * 16 + nbk * 16 + e] = isd[e];
                o[na + nbd * 16 + 2 * nbk * 16 + e] = Dn[e];
            }
        }
        if (blockIdx.x == 0 && tid == 64) g_ts[24] = __builtin_amdgcn_s_memrealtime();  // (ts probe)
    } else {
        // in the kernel: W = X U in place of U, the DMX errors (C_xx's diagonal D^-1 + D^-1
        // |W_a|^2) and the covariance blocks, as k_cov_dmx forms them
        w_from_xu<NW>(A, nbd, nbk, nblkS, wave, lane);
        __syncthreads();
        dmx_errors<NW>(A, inx, Dn, Pd, errs + I.coff, ndc, nbd, nbk, nblkS);
        cov_dmx_blocks(A, ind, inx, isd, Dn, Pd, cov + (long)I.cvoff, ncol, red0, ndc, nbd, nbk, nblkS, wave, NW, lane);
    }
    TS(6);
    if (apply_tables && !setup_w0) {
        __syncthreads();  // (the covariance blocks read A, not the staged table; kept simple)
        if (wave == 0) apply_setup(inst, tail, S.tstride, apply_ic);
    }
    TS(7);
}

// k_cov_dmx: W = X U, the DMX errors and the covariance blocks of k_solve_dmx (deferred
// solves export X, U and the scalings to d_xw); COV_WG workgroups per instance, each staging
// the instance's export in LDS and forming W itself; launched by pint_read_step when the
// errors or the covariance are read (on the copy stream, off the fit step's critical path)
constexpr int COV_WG = 3;
template <int NW>
__global__ __launch_bounds__(NW * 64) void k_cov_dmx(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                     const double* __restrict__ xw, int mode, double* __restrict__ cov,
                                                     double* __restrict__ errs) {
    WgTimer wgt_(WGT_COV);
    extern __shared__ double lds[];
    const InstDev I = insts[blockIdx.x];
    const PsrDev& Pd = psrs[I.psr];
    if (!Pd.dsplit) return;
    const int ndc = Pd.ndc, red0 = Pd.red0c;
    const int Kd = (mode == 0) ? red0 : Pd.Kd;
    const int nbd = (Kd + 15) >> 4, nbk = (ndc + 15) >> 4, nblkS = nbd * (nbd + 1) / 2;
    const int na = (nblkS + nbd * nbk) * 256, nv = na + (nbd + 3 * nbk) * 16;
    const double* src = xw + I.xwoff;
    copy_in<NW * 64, 16>(lds, src, nv, threadIdx.x);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const double* ind = lds + na;
    const double* inx = ind + nbd * 16;
    const double* isd = inx + nbk * 16;
    const double* Dn = isd + nbk * 16;
    w_from_xu<NW>(lds, nbd, nbk, nblkS, wave, lane);
    __syncthreads();
    if (blockIdx.y == 0 && errs) dmx_errors<NW>(lds, inx, Dn, Pd, errs + I.coff, ndc, nbd, nbk, nblkS);
    if (cov)
        cov_dmx_blocks(lds, ind, inx, isd, Dn, Pd, cov + (long)I.cvoff, Pd.spec->ncol, red0, ndc, nbd, nbk, nblkS,
                       blockIdx.y * NW + wave, gridDim.y * NW, lane);
}

// ---------------------------------------------------------------------------------
// k_eig: the SVD path of the fitters for degenerate normal equations (fitter.py:1282-1359
// WLSState.step: SVD of the whitened normalised M, singular values <= threshold * s_max
// dropped; fitter.py:2196-2230 GLSFitter: Cholesky, on failure SVD of mtcm).  The
// normalised normal matrix A (= M^T M for WLS, mtcm for GLS) is symmetric, so its SVD is
// its eigendecomposition: cyclic Jacobi with the round-robin ordering (K/2 disjoint
// rotations per round, applied as a row pass and a column pass), one 1024-thread
// workgroup per instance, A and V in global scratch (K x K each).  WLS: s = sqrt(lambda);
// GLS: s = |lambda|; directions with s <= threshold * s_max are dropped and reported.
// ---------------------------------------------------------------------------------
constexpr int EIG_T = 1024;
constexpr int EIG_MAXDEG = PINT_EIG_MAXDEG;
__global__ __launch_bounds__(EIG_T) void k_eig(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                               const double* __restrict__ Gpart, const double* __restrict__ colsq,
                                               int nsplit, int mode, int compact, const double* __restrict__ Sd,
                                               const double* __restrict__ DD, const double* __restrict__ DCS,
                                               const double* __restrict__ thresholds, double* __restrict__ work,
                                               long wstride,
                                               double* __restrict__ dpars, double* __restrict__ errs,
                                               double* __restrict__ cov, double* __restrict__ chi2lin,
                                               int* __restrict__ ndeg, double* __restrict__ degvec, int degstride) {
    extern __shared__ double lds[];
    __shared__ double sh[EIG_T / 64];
    __shared__ int sflag;
    const int inst = blockIdx.x;
    const InstDev I = insts[inst];
    const PsrDev& Pd = psrs[I.psr];
    const pint_spec_t& S = *Pd.spec;
    const int Kfull = I.K, ncol = S.ncol;
    const int K = (mode == 0) ? ncol : Kfull;
    const int Ke = (K + 1) & ~1;  // even: one dummy index when K is odd
    const bool cmp = compact && Pd.dsplit;
    const GramView G = gram_view(Pd, I, Gpart, cmp, Sd, DD);
    double* A = work + (long)inst * wstride;  // K x K, row-major
    double* V = A + (long)K * K;              // K x K, columns = eigenvectors
    double* nrm = lds;                        // K
    double* bv = nrm + K;                     // K
    double* cs = bv + K;                      // Ke/2 cosines
    double* sn = cs + Ke / 2;                 // Ke/2 sines
    double* lam = sn + Ke / 2;                // K
    double* xh = lam + K;                     // K
    const int tid = threadIdx.x;
    for (int j = tid; j < K; j += EIG_T) {
        double v = sqrt(mode == 0 ? G(j, j) : colsq_of(Pd, I, colsq, nsplit, cmp, DCS, j));
        nrm[j] = (v == 0.0) ? 1.0 : v;
    }
    __syncthreads();
    for (long e = tid; e < (long)K * K; e += EIG_T) {
        const int i = (int)(e / K), j = (int)(e % K);
        double v = G(i, j) / (nrm[i] * nrm[j]);
        if (i == j && mode == 1 && i >= ncol) v += 1.0 / Pd.red_phi[i - ncol] / (nrm[i] * nrm[i]);
        A[e] = v;
        V[e] = (i == j) ? 1.0 : 0.0;
    }
    for (int j = tid; j < K; j += EIG_T) bv[j] = G(j, Kfull) / nrm[j];
    const double rwr = G(Kfull, Kfull);
    __syncthreads();
    double fro = 0.0;
    for (long e = tid; e < (long)K * K; e += EIG_T) fro += A[e] * A[e];
    fro = block_sum<EIG_T / 64>(fro, sh);
    for (int sweep = 0; sweep < 40; sweep++) {
        double off = 0.0;
        for (long e = tid; e < (long)K * K; e += EIG_T)
            if (e / K != e % K) off += A[e] * A[e];
        off = block_sum<EIG_T / 64>(off, sh);
        if (off <= 1e-30 * fro || off == 0.0) break;
        for (int r = 0; r < Ke - 1; r++) {
            // round-robin pairs: position 0 fixed, positions 1..Ke-1 rotated by r
            auto at = [&](int k) { return k == 0 ? 0 : 1 + (k - 1 + r) % (Ke - 1); };
            for (int k = tid; k < Ke / 2; k += EIG_T) {
                int p = at(k), q = at(Ke - 1 - k);
                if (p > q) { const int t = p; p = q; q = t; }
                double c = 1.0, s = 0.0;
                if (q < K) {
                    const double apq = A[(long)p * K + q];
                    if (apq != 0.0) {
                        const double tau = (A[(long)q * K + q] - A[(long)p * K + p]) / (2.0 * apq);
                        const double t = (tau >= 0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
                        c = 1.0 / sqrt(1.0 + t * t);
                        s = t * c;
                    }
                }
                cs[k] = c;
                sn[k] = s;
            }
            __syncthreads();
            // rows: p' = c p - s q, q' = s p + c q (J^T A)
            for (long e = tid; e < (long)(Ke / 2) * K; e += EIG_T) {
                const int k = (int)(e / K), j = (int)(e % K);
                int p = at(k), q = at(Ke - 1 - k);
                if (p > q) { const int t = p; p = q; q = t; }
                if (q >= K || sn[k] == 0.0) continue;
                const double c = cs[k], s = sn[k];
                const double ap = A[(long)p * K + j], aq = A[(long)q * K + j];
                A[(long)p * K + j] = c * ap - s * aq;
                A[(long)q * K + j] = s * ap + c * aq;
            }
            __syncthreads();
            // columns of A and V: p' = c p - s q, q' = s p + c q (A J, V J)
            for (long e = tid; e < (long)(Ke / 2) * K; e += EIG_T) {
                const int k = (int)(e / K), i = (int)(e % K);
                int p = at(k), q = at(Ke - 1 - k);
                if (p > q) { const int t = p; p = q; q = t; }
                if (q >= K || sn[k] == 0.0) continue;
                const double c = cs[k], s = sn[k];
                double ap = A[(long)i * K + p], aq = A[(long)i * K + q];
                A[(long)i * K + p] = c * ap - s * aq;
                A[(long)i * K + q] = s * ap + c * aq;
                ap = V[(long)i * K + p];
                aq = V[(long)i * K + q];
                V[(long)i * K + p] = c * ap - s * aq;
                V[(long)i * K + q] = s * ap + c * aq;
            }
            __syncthreads();
        }
    }
    // singular values and the dropped directions
    for (int j = tid; j < K; j += EIG_T) lam[j] = A[(long)j * K + j];
    __syncthreads();
    const double threshold = thresholds[inst];
    double smax = 0.0;
    for (int j = 0; j < K; j++) {
        const double sv = mode == 0 ? sqrt(fmax(lam[j], 0.0)) : fabs(lam[j]);
        smax = fmax(smax, sv);
    }
    auto bad = [&](int j) {
        const double sv = mode == 0 ? sqrt(fmax(lam[j], 0.0)) : fabs(lam[j]);
        return !(sv > threshold * smax);
    };
    // xhat = sum_good V_j (V_j . b) / lambda_j
    for (int j = tid; j < K; j += EIG_T) {
        double pr = 0.0;
        if (!bad(j)) {
            for (int i = 0; i < K; i++) pr += V[(long)i * K + j] * bv[i];
            pr /= lam[j];
        }
        xh[j] = pr;  // coefficient of eigenvector j
    }
    __syncthreads();
    double bx = 0.0;
    for (int i = tid; i < K; i += EIG_T) {
        double x = 0.0;
        for (int j = 0; j < K; j++) x += V[(long)i * K + j] * xh[j];
        dpars[I.coff + i] = x / nrm[i];
        bx += bv[i] * x;
    }
    bx = block_sum<EIG_T / 64>(bx, sh);
    if (tid == 0) chi2lin[inst] = rwr - bx;
    // xvar = sum_good V_j V_j^T / s_j (s_j = lambda_j for WLS, |lambda_j| for GLS)
    double* C = cov + (long)I.cvoff;
    for (long e = tid; e < (long)K * K; e += EIG_T) {
        const int i = (int)(e / K), l = (int)(e % K);
        if (i > l) continue;
        if (l >= ncol && i != l) continue;  // timing block + the diagonal
        double v = 0.0;
        for (int j = 0; j < K; j++)
            if (!bad(j)) v += V[(long)i * K + j] * V[(long)l * K + j] / fabs(lam[j]);
        const double vv = v / (nrm[i] * nrm[l]);
        if (l < ncol) {
            C[(long)i * ncol + l] = vv;
            C[(long)l * ncol + i] = vv;
        }
        if (i == l) errs[I.coff + i] = sqrt(v) / nrm[i];
    }
    // dropped directions, smallest singular value first, each scaled to max |component| = 1
    if (tid == 0) {
        int nd = 0;
        unsigned long long used[4] = {0, 0, 0, 0};
        while (nd < EIG_MAXDEG) {
            int best = -1;
            for (int j = 0; j < K; j++)
                if (bad(j) && !((used[j >> 6] >> (j & 63)) & 1) &&
                    (best < 0 || fabs(lam[j]) < fabs(lam[best])))
                    best = j;
            if (best < 0) break;
            used[best >> 6] |= 1ull << (best & 63);
            double mx = 0.0;
            for (int i = 0; i < K; i++) mx = fmax(mx, fabs(V[(long)i * K + best]));
            double* out = degvec + ((long)inst * EIG_MAXDEG + nd) * degstride;
            for (int i = 0; i < K; i++) out[i] = V[(long)i * K + best] / (mx > 0 ? mx : 1.0);
            nd++;
        }
        ndeg[inst] = nd;
        sflag = nd;
    }
}

// k_sigma: the Woodbury Sigma factor of every GLS instance (woodbury_sigma), launched on a
// side stream right after the Gram so it runs on the CUs the per-instance solve leaves idle.
template <int NW>
__global__ __launch_bounds__(NW * 64) void k_sigma(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                   const double* __restrict__ tables, const double* __restrict__ Gpart,
                                                   int compact, const double* __restrict__ Sd,
                                                   const double* __restrict__ DD, double* __restrict__ sigL,
                                                   int* __restrict__ status, const double* __restrict__ ones) {
    extern __shared__ double lds[];
    __shared__ int sflag;
    const InstDev I = insts[blockIdx.x];
    const PsrDev& Pd = psrs[I.psr];
    const pint_spec_t& S = *Pd.spec;
    if (!(S.nred > 0 || Pd.nep > 0)) return;
    if (threadIdx.x == 0) sflag = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const GramView G = gram_view(Pd, I, Gpart, compact && Pd.dsplit, Sd, DD);
    if (!woodbury_sigma<NW>(G, Pd, S, pval(tables + I.toff, S.o_F), lds, wave, lane, &sflag, sigL + (long)I.soff,
                            ones ? ones + I.coff : nullptr)) {
        if (threadIdx.x == 0) atomicOr(status, 1 << PINT_E_SIGMA);
    }
}

// Woodbury GLS chi2 of the current residuals (utils.py:3074-3126 woodbury_dot):
// chi2 = r^T N^-1 r - d^T Sigma^-1 d, d = U^T N^-1 r, U = [F, ECORR, 1].  The ECORR block
// is eliminated: with c_e = sum_{i in e} w_i r_i, r^T N^-1 r -= sum c_e^2 / D_e and
// d_j -= sum_e B_je c_e / D_e (B from k_ecorr's epoch sums); Sigma' (Schur-reduced) was
// factored by k_solve from the reduced Gram.
//   k_wdot    grid (nsplit, ninst): per-split partial dot products F_j^T W r, r^T W r,
//             1^T W r; one wave per column (coalesced column reads, shuffle reduction)
//   k_wsolve  one workgroup per instance: split sums, ECORR correction, forward
//             substitution with Sigma's Cholesky factor, chi2
// one wave per column (coalesced column reads, 4 row-slices in flight per lane), shuffle
// reduction; columns R and R+1 are r^T W r and 1^T W r
__global__ __launch_bounds__(256) void k_wdot(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                              const double* __restrict__ M, const double* __restrict__ rtime,
                                              int nsplit, int stride, int compact, double* __restrict__ wpart) {
    const int inst = blockIdx.y, split = blockIdx.x;
    const InstDev I = insts[inst];
    const PsrDev& Pd = psrs[I.psr];
    const pint_spec_t& S = *Pd.spec;
    const int n = I.n, R = 2 * S.nred;
    const double* ri = rtime + (I.roff - inst);
    long per = (n + nsplit - 1) / nsplit;
    long i0 = split * per, i1 = i0 + per;
    if (i1 > n) i1 = n;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double* out = wpart + ((long)inst * nsplit + split) * stride;
    if (compact && Pd.dsplit && Pd.vg) {
        // Fourier columns generated per row by rotations of the fundamental (k_trig_setup):
        // wave w takes harmonics 8w .. 8w+7; wave 0 also accumulates r^T W r and 1^T W r
        const int h0 = 8 * wave;
        const bool act = h0 < S.nred;
        double a[16];
#pragma unroll
        for (int u = 0; u < 16; u++) a[u] = 0.0;
        double rr = 0.0, r1 = 0.0;
        for (long i = i0 + lane; i < i1; i += 64) {
            const double is = Pd.isig[i], r = ri[i], wr = is * is * r;
            if (wave == 0) {
                rr += wr * r;
                r1 += wr;
            }
            if (act) {
                const double c1 = Pd.red_cs[4 * i], s1 = Pd.red_cs[4 * i + 1];
                double sn, cs;
                cpow(Pd.red_cs[4 * i + 2], Pd.red_cs[4 * i + 3], wave, cs, sn);  // e^{i 8w theta}
                rot(cs, sn, c1, s1);                                             // e^{i (8w+1) theta}
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    a[2 * u] += sn * wr;
                    a[2 * u + 1] += cs * wr;
                    rot(cs, sn, c1, s1);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            if (h0 + u < S.nred) {
                const double vs = wave_sum(a[2 * u]), vc = wave_sum(a[2 * u + 1]);
                if (lane == 0) {
                    out[2 * (h0 + u)] = vs;
                    out[2 * (h0 + u) + 1] = vc;
                }
            }
        }
        if (wave == 0) {
            rr = wave_sum(rr);
            r1 = wave_sum(r1);
            if (lane == 0) {
                out[R] = rr;
                out[R + 1] = r1;
            }
        }
        return;
    }
    const double* Fb = M + I.moff + (long)(compact && Pd.dsplit ? Pd.red0c : S.ncol) * n;
    for (int j = wave; j < R + 2; j += 4) {
        const double* col = Fb + (long)(j < R ? j : 0) * n;
        double acc = 0.0;
#pragma unroll 4
        for (long i = i0 + lane; i < i1; i += 64) {
            const double is = Pd.isig[i], r = ri[i];
            const double f = j < R ? col[i] : (j == R ? r : 1.0);
            acc += f * is * is * r;
        }
        acc = wave_sum(acc);
        if (lane == 0) out[j] = acc;
    }
}

__global__ __launch_bounds__(256) void k_wsolve(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                const double* __restrict__ rtime, const double* __restrict__ sigL,
                                                const double* __restrict__ esum, const double* __restrict__ eD,
                                                const double* __restrict__ eW, const double* __restrict__ wpart,
                                                int nsplit, int stride, double* __restrict__ ecs,
                                                double* __restrict__ chi2, double* __restrict__ lognorm,
                                                const double* __restrict__ wtile, const double* __restrict__ rpart,
                                                double* __restrict__ chi2w, int compact) {
    WgTimer wgt_(WGT_WSOLVE);
    extern __shared__ double lds[];
    __shared__ double sh[12];  // block_sums<4, 3>
    __shared__ double Dt[256], wloc[130];
    const int inst = blockIdx.x;
    const InstDev I = insts[inst];
    const PsrDev& Pd = psrs[I.psr];
    const pint_spec_t& S = *Pd.spec;
    const int R = 2 * S.nred, Kn = R + 1;
    const double* ri = rtime + (I.roff - inst);
    double* d = lds;  // Kn
    const double* wp = wpart + (long)inst * nsplit * stride;
    // the packed inverse factor of Sigma (from the solve) staged in LDS first, with coalesced
    // loads that are in flight while the dot products below are summed; with no noise basis
    // Sigma is the 1x1 [1e-40 + 1^T N^-1 1], which the solves do not factor
    const bool nobasis = (R == 0 && Pd.nep == 0);
    double* Xs = d + Kn;  // Kn (Kn + 1) / 2
    {
        const double* X = sigL + I.soff;
        const int nX = nobasis ? 0 : Kn * (Kn + 1) / 2;
        copy_in<256, 8>(Xs, X, nX, threadIdx.x);
    }
    if (wtile) {
        // r^T W r: the residual pass's chi2 partials of the instance summed exactly as k_rsum
        // does (wave 0, same order: the same bits), stored as the residuals' chi2 (k_rsum is
        // then not launched for this pass)
        if (threadIdx.x < 64) {
            double t = 0.0;
            for (int k = threadIdx.x; k < I.nrb; k += 64) t += rpart[3 * (I.rb0 + k) + 2];
            t = wave_sum(t);
            if (threadIdx.x == 0) {
                chi2w[inst] = t;
                wloc[R] = t;
            }
        }
        // the dots from k_resid2's trig tiles (one per residual block of the instance, summed
        // in block order): F_j^T W r (sin, cos of harmonic h + 1 at 2h, 2h + 1), r^T W r (the
        // residual pass's chi2) at R, 1^T W r = D[0][0] at R + 1 -- k_wdot's layout, one split
        // the instance's block tiles summed in block order in four interleaved chains (four
        // loads in flight instead of one dependent load per block), combined in a fixed order
        double v4[4] = {0.0, 0.0, 0.0, 0.0};
        int k = 0;
        for (; k + 4 <= I.nrb; k += 4) {
#pragma unroll
            for (int u = 0; u < 4; u++) v4[u] += wtile[(long)(I.rb0 + k + u) * 256 + threadIdx.x];
        }
        for (; k < I.nrb; k++) v4[0] += wtile[(long)(I.rb0 + k) * 256 + threadIdx.x];
        Dt[threadIdx.x] = (v4[0] + v4[1]) + (v4[2] + v4[3]);
        __syncthreads();
        for (int h = threadIdx.x; h < R / 2; h += blockDim.x) {
            const int k = h + 1, a = k & 7, b = k >> 3;
            wloc[2 * h] = Dt[(8 + a) * 16 + b] + Dt[a * 16 + 8 + b];      // sum w r sin(k theta)
            wloc[2 * h + 1] = Dt[a * 16 + b] - Dt[(8 + a) * 16 + 8 + b];  // sum w r cos(k theta)
        }
        if (threadIdx.x == 0) wloc[R + 1] = Dt[0];
        __syncthreads();
        wp = wloc;
        nsplit = 1;
    }
    double rwr = 0.0, rw1 = 0.0;
    if (threadIdx.x == 0) {
        for (int q = 0; q < nsplit; q++) {
            rwr += wp[(long)q * stride + R];
            rw1 += wp[(long)q * stride + R + 1];
        }
    }
    // ECORR epochs: c_e / D_e of the current residuals
    const int nep = Pd.nep;
    const double* Ei = esum + I.eoff;
    double* ce = ecs + I.epoff;
    // log-normalisation of the likelihood, logdet(C)/2 (residuals.py:567-589 via
    // utils.py:3074 woodbury_dot): logdet C = logdet N + logdet Phi + logdet Sigma, Phi =
    // [phi_red, phi_ecorr, 1e40]; with the ECORR block eliminated, logdet Sigma =
    // sum_e log D_e + logdet Sigma' and Sigma' = L L^T (X = L^-1 holds 1/L_jj on its diagonal).
    // Its inputs are ready at launch: formed here, off the dot products' chain, and reduced
    // with the ECORR sums
    const double x00 = S.wb_noones ? 1.0 : 1.0 / sqrt(1e-40 + Pd.sumw);
    double ld = 0.0;
    {
        const double* X = sigL + I.soff;
        for (int e = threadIdx.x; e < nep; e += blockDim.x) ld += log(Pd.ep_phi[e]) + log(eD[I.epoff + e]);
        for (int k = threadIdx.x; k < R; k += blockDim.x) ld += log(Pd.red_phi[k]);
        for (int j = threadIdx.x; j < Kn; j += blockDim.x) ld -= 2.0 * log(nobasis ? x00 : X[tri(j, j)]);
    }
    double erwr = 0.0, erw1 = 0.0;
    for (int e = threadIdx.x; e < nep; e += blockDim.x) {
        double c = 0.0;
        for (int k = Pd.ep_ptr[e]; k < Pd.ep_ptr[e + 1]; k++) {
            int i = Pd.ep_idx[k];
            c += ri[i] / (Pd.sigma[i] * Pd.sigma[i]);
        }
        double De = eD[I.epoff + e];
        erwr += c * c / De;
        erw1 += eW[I.epoff + e] * c / De;
        ce[e] = c / De;
    }
    {
        double v[3] = {erwr, erw1, ld};
        block_sums<4, 3>(v, sh);  // (its barriers also make ce visible)
        erwr = v[0];
        erw1 = v[1];
        ld = v[2];
    }
    // the Fourier columns of the epoch sums: after the timing columns (full layout) or at
    // red0c of the compact dense columns
    const bool ecmp = compact && Pd.dsplit;
    const int es = ecmp ? Pd.Kpd : I.Kp, ef = ecmp ? Pd.red0c : S.ncol;
    for (int j = threadIdx.x; j < R; j += blockDim.x) {
        double v = 0.0;
        for (int q = 0; q < nsplit; q++) v += wp[(long)q * stride + j];
        double t[4] = {0.0, 0.0, 0.0, 0.0};  // four independent chains (loads in flight)
        int e = 0;
        for (; e + 4 <= nep; e += 4) {
#pragma unroll
            for (int u = 0; u < 4; u++) t[u] += Ei[(long)(e + u) * es + ef + j] * ce[e + u];
        }
        for (; e < nep; e++) t[0] += Ei[(long)e * es + ef + j] * ce[e];
        d[j] = v - ((t[0] + t[1]) + (t[2] + t[3]));
    }
    if (threadIdx.x == 0) d[R] = S.wb_noones ? 0.0 : rw1 - erw1;  // the ones column's entry
    __syncthreads();
    // y = L^-1 d with the explicit inverse factor (staged above), four lanes per row
    double q = 0.0;
    for (int i0 = 0; i0 < Kn; i0 += blockDim.x / 4) {
        const int i = i0 + (threadIdx.x >> 2), sub = threadIdx.x & 3;
        double s = 0.0;
        if (i < Kn) {
            if (nobasis) s = sub == 0 ? x00 * d[0] : 0.0;
            else
                for (int j = sub; j <= i; j += 4) s += Xs[tri(i, j)] * d[j];
        }
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        if (sub == 0 && i < Kn) q += s * s;
    }
    q = block_sum<4>(q, sh);
    if (threadIdx.x == 0) {
        chi2[inst] = (rwr - erwr) - q;
        lognorm[inst] = 0.5 * (ld + 2.0 * Pd.logsig + (S.wb_noones ? 0.0 : log(1e40)));
    }
}

// tables += lambda * dpars on every timing column (skips Offset), double-double add; then
// the per-instance constants of the updated table (k_prep's work, saving its launch).
// Launched with PREP_T threads: the bound lets the setup keep k_prep's registers (the
// default 1024-thread budget of 128 VGPRs spilled 252 B/lane into its serial chain)
__global__ __launch_bounds__(PREP_T) void k_apply(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts, double* __restrict__ tables,
                        const double* __restrict__ dpars, const double* __restrict__ lam,
                        InstConst* __restrict__ ic, double lam_u) {
    const int inst = blockIdx.x;
    const InstDev I = insts[inst];
    const pint_spec_t& S = *psrs[I.psr].spec;
    double* P = tables + I.toff;
    const double li = lam ? lam[inst] : lam_u;  // per instance, or one lambda for the batch
    for (int c = threadIdx.x; c < S.ncol; c += blockDim.x) {
        int o = S.col_toff[c];
        if (o < 0) continue;
        if (li == 0.0) continue;  // decided instances: a non-finite step must not touch them
        dd v = dd_add_d(dd_make(P[o], P[o + 1]), li * dpars[I.coff + c]);
        P[o] = v.hi;
        P[o + 1] = v.lo;
    }
    __syncthreads();
    prep_one(psrs[I.psr].spec, P, S.tstride, ic + inst);
}

// k_chi2w: the WLS chi2 sum_i (r_i / sigma_i)^2 of the current time residuals of every
// instance (residuals.py:638-667 _calc_wls_chi2), one workgroup per instance, wave-shuffle
// reductions in a fixed order (deterministic); pint_chi2_wls, for residuals replaced by
// pint_debug_set_resids / pint_set_resids (the residual pass computes its own chi2).
__global__ __launch_bounds__(256) void k_chi2w(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                               const double* __restrict__ rtime, double* __restrict__ chi2) {
    __shared__ double sh[4];
    const InstDev I = insts[blockIdx.x];
    const PsrDev& Pd = psrs[I.psr];
    const double* r = rtime + (I.roff - blockIdx.x);
    double a = 0.0;
    for (int i = threadIdx.x; i < I.n; i += 256) {
        const double x = r[i] * Pd.isig[i];
        a += x * x;
    }
    a = block_sum<4>(a, sh);
    if (threadIdx.x == 0) chi2[blockIdx.x] = a;
}

// ---------------------------------------------------------------------------------
// Noise realisations of the last fit step (fitter.py:2270-2282 GLSFitter, :1582-1605
// DownhillGLSFitter: noise_resids[comp] = M[:, comp] @ xhat[comp] with M, xhat normalised,
// i.e. F @ dpars in par units).
//   k_noise_red    PLRedNoise: sum_k a_k sin(2 pi t f_k) + b_k cos(2 pi t f_k) per TOA, the
//                  argument reduced in double-double as k_eval forms the basis
//   k_noise_ecorr  ECORR: the eliminated epoch coefficients, back-substituted from the Schur
//                  system, c_e = (s_e[r] - s_e . x) / D_e  (s_e = sum_{i in e} w_i [M | r]_i,
//                  D_e = W_e + 1/phi_e from k_ecorr), written to every TOA of epoch e
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_noise_red(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                   const double* __restrict__ dpars, double* __restrict__ out,
                                                   int dm, const double* __restrict__ dfac) {
    WgTimer wgt_(WGT_NOISE);
    __shared__ double sa[256];  // the component's amplitudes (a_k, b_k), staged once per block
    const int inst = blockIdx.y;
    const InstDev I = insts[inst];
    const PsrDev& Pd = psrs[I.psr];
    const pint_spec_t& S = *Pd.spec;
    const int i = blockIdx.x * 256 + threadIdx.x;
    // block-uniform bounds (readfirstlane: the spec is read through a generic pointer)
    const int ncol = __builtin_amdgcn_readfirstlane(S.ncol), nred = __builtin_amdgcn_readfirstlane(S.nred);
    const int dmn0 = __builtin_amdgcn_readfirstlane(S.dmn0);
    const int k0 = dm ? dmn0 : 0, k1 = dm ? nred : dmn0;
    const double* a = dpars + I.coff + ncol;
    double v = 0.0;
    if (!dm && k1 > 0 && k1 <= 128) {
        // PLRedNoise block: harmonics 1..dmn0 of f_1 = red_freq[0] (get_rednoise_freqs is
        // linspace(1/T, nmodes/T)), by rotations of the row's e^{i theta} (k_trig_setup) instead
        // of a double-double reduction and a sincos per harmonic; four independent chains
        // (harmonics j + 1 + 4m, j < 4, stepped by e^{4 i theta}) for instruction-level
        // parallelism
        for (int k = threadIdx.x; k < 2 * k1; k += 256) sa[k] = a[k];
        __syncthreads();
        if (i >= I.n) return;
        const double4_t z = ((gptr<double4_t>)Pd.red_cs)[i];
        const double c1 = z[0], s1 = z[1];
        double cz[4], sz[4];
        cz[0] = c1;
        sz[0] = s1;
#pragma unroll
        for (int j = 1; j < 4; j++) {
            cz[j] = cz[j - 1];
            sz[j] = sz[j - 1];
            rot(cz[j], sz[j], c1, s1);
        }
        double c4 = cz[3], s4 = sz[3];  // e^{4 i theta}
        double vj[4] = {0.0, 0.0, 0.0, 0.0};
        for (int m = 0; m < k1; m += 4) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if (m + j < k1) vj[j] += sa[2 * (m + j)] * sz[j] + sa[2 * (m + j) + 1] * cz[j];
                rot(cz[j], sz[j], c4, s4);
            }
        }
        v = (vj[0] + vj[1]) + (vj[2] + vj[3]);
    } else {
        if (i >= I.n) return;
        if (k1 > k0) {
            const dd ts = dd_mul_d(dd_make(Pd.tdb_hi[i], Pd.tdb_lo[i]), DAYSEC);
            for (int k = k0; k < k1; k++) {
                const dd x = dd_mul(ts, dd_make(Pd.red_freq[k], Pd.red_freq[nred + k]));
                const double fr = dd_to_d(dd_sub(x, dd_floor(x)));
                double sn, cs;
                sincos(TWO_PI * fr, &sn, &cs);
                v += a[2 * k] * sn + a[2 * k + 1] * cs;
            }
            if (dm) v *= dfac[I.ooff + i];
        }
    }
    out[I.roff - inst + i] = v;
}

__global__ __launch_bounds__(64) void k_noise_ecorr(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                    const double* __restrict__ dpars, const double* __restrict__ esum,
                                                    const double* __restrict__ eD, double* __restrict__ out,
                                                    int compact, const double* __restrict__ eC) {
    const int inst = blockIdx.y, e = blockIdx.x;
    const InstDev I = insts[inst];
    const PsrDev& Pd = psrs[I.psr];
    if (e >= Pd.nep) return;
    const bool cmp = compact && Pd.dsplit;
    const int K = I.K;
    const double* x = dpars + I.coff;
    double t = 0.0;
    for (int c = threadIdx.x; c < K; c += 64) t += esum_col(Pd, I, esum, eC, cmp, e, c) * x[c];
    t = wave_sum(t);
    const double ce = (esum_col(Pd, I, esum, eC, cmp, e, K) - t) / eD[I.epoff + e];
    double* o = out + (I.roff - inst);
    for (int k = Pd.ep_ptr[e] + threadIdx.x; k < Pd.ep_ptr[e + 1]; k += 64) o[Pd.ep_idx[k]] = ce;
}

// k_noise_lnl: log-likelihood of the fixed time residuals under trial white-noise parameters,
// the objective of the noise-parameter fit (fitter.py:1242-1261 _mloglike/_mloglike_grad with
// residuals.py:591-667 and :718-807).  One workgroup per instance; the residuals r stay those
// of the last evaluation, as the reference keeps Residuals.time_resids while it changes the
// noise parameters.  Per TOA N_i = (sigma0_i^2 + Q_c^2) F_c^2 (us^2 -> s^2) from the (Q^2, F) of
// its class c.  kind (meta[3k+1]): 0 diagonal N (residuals.py:638); 1 N plus one ECORR block
// per epoch, Sherman-Morrison (residuals.py:591); 2 as 1 plus the 1e40 offset column of
// _calc_gls_chi2 (residuals.py:583-587), eliminated last.  Writes (lnL, chi2, logdet C / 2) and,
// for kinds 0/1, sum_i g_i N_i and sum_i g_i per class (g_i = dlnL/dN_i) and dlnL/dw_e per epoch.
__global__ __launch_bounds__(256) void k_noise_lnl(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                  const double* __restrict__ rtime, const long* __restrict__ meta,
                                                  const double* __restrict__ qf, const double* __restrict__ epw,
                                                  double* __restrict__ epsv, double* __restrict__ out,
                                                  double* __restrict__ clsg, double* __restrict__ epg) {
    __shared__ double sh[32];  // block_sums<4, 8>
    const int inst = blockIdx.x;
    const InstDev I = insts[inst];
    const PsrDev& Pd = psrs[I.psr];
    const long q0 = meta[3 * inst];
    const int kind = (int)meta[3 * inst + 1];
    const double* ri = rtime + I.ooff;
    const double* Q = qf + 2 * q0;
    const int nep = kind ? Pd.nep : 0;
    // per epoch: s = sum r/N, v = sum 1/N over its TOAs; the Sherman-Morrison terms
    double ec = 0.0, el = 0.0, ea = 0.0, eb = 0.0;
    for (int e = threadIdx.x; e < nep; e += 256) {
        double s = 0.0, v = 0.0;
        for (int k = Pd.ep_ptr[e]; k < Pd.ep_ptr[e + 1]; k++) {
            const int i = Pd.ep_idx[k], c = Pd.toa_cls[i];
            const double s0 = Pd.sigma0[i], f = Q[2 * c + 1];
            const double iN = 1.0 / ((s0 * s0 + Q[2 * c]) * (f * f) * 1e-12);
            s += ri[i] * iN;
            v += iN;
        }
        const double w = epw[I.epoff + e], den = 1.0 + w * v;
        epsv[2 * (I.epoff + e)] = s;
        epsv[2 * (I.epoff + e) + 1] = v;
        ec += w * s * s / den;
        el += log(den);
        ea += w * s * v / den;
        eb += w * v * v / den;
        if (kind == 1) epg[I.epoff + e] = 0.5 * (s * s / (den * den) - v / den);
    }
    __syncthreads();
    double t1 = 0.0, t2 = 0.0, S = 0.0, V = 0.0;
    bool neg = false;
    for (int c = 0; c < Pd.ncls; c++) {
        const double q2 = Q[2 * c], f = Q[2 * c + 1], f2 = f * f;
        neg |= f < 0.0;
        double A = 0.0, B = 0.0;
        for (int k = Pd.cls_ptr[c] + threadIdx.x; k < Pd.cls_ptr[c + 1]; k += 256) {
            const int i = Pd.cls_idx[k];
            const double s0 = Pd.sigma0[i], N = (s0 * s0 + q2) * f2 * 1e-12, iN = 1.0 / N, r = ri[i], rn = r * iN;
            t1 += r * rn;
            t2 += log(N);
            S += rn;
            V += iN;
            double g = 0.5 * (rn * rn - iN);
            const int e = nep ? Pd.toa_ep[i] : -1;
            if (e >= 0) {
                const double s = epsv[2 * (I.epoff + e)], v = epsv[2 * (I.epoff + e) + 1];
                const double w = epw[I.epoff + e], den = 1.0 / (1.0 + w * v);
                g += (-w * s * r * den + 0.5 * w * w * s * s * den * den + 0.5 * w * den) * iN * iN;
            }
            A += g * N;
            B += g;
        }
        {
            double v[2] = {A, B};
            block_sums<4, 2>(v, sh);
            A = v[0];
            B = v[1];
        }
        if (threadIdx.x == 0 && kind < 2) {
            clsg[2 * (q0 + c)] = A;
            clsg[2 * (q0 + c) + 1] = B;
        }
    }
    {
        double v[8] = {t1, t2, S, V, ec, el, ea, eb};
        block_sums<4, 8>(v, sh);  // (one barrier pair for the eight sums, the same bits)
        t1 = v[0]; t2 = v[1]; S = v[2]; V = v[3]; ec = v[4]; el = v[5]; ea = v[6]; eb = v[7];
    }
    if (threadIdx.x == 0) {
        double chi2 = t1 - ec, ln = 0.5 * (t2 + el);
        if (kind == 2) {
            const double a = S - ea, b = 1e-40 + (V - eb);
            chi2 -= a * a / b;
            ln += 0.5 * (log(1e40) + log(b));
        }
        if (kind == 0 && neg) ln = __builtin_nan("");  // sum log sigma of a negative EFAC (residuals.py:666)
        out[3 * inst] = -(0.5 * chi2 + ln);
        out[3 * inst + 1] = chi2;
        out[3 * inst + 2] = ln;
    }
}

// Debug/parity introspection (pint_debug_gram): the assembled, unnormalised normal matrix
// [M | r]^T N^-1 [M | r] of the last pint_fit_step in the original column order (the ECORR
// block already eliminated by its Schur complement), (K+1)^2 per instance, followed by the K
// unweighted column sums of squares of M (normalize_designmatrix).
__global__ __launch_bounds__(256) void k_debug_gram(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                                    const double* __restrict__ Gpart, const double* __restrict__ colsq,
                                                    int nsplit, int compact, const double* __restrict__ Sd,
                                                    const double* __restrict__ DD, const double* __restrict__ DCS,
                                                    const double* __restrict__ esum, const double* __restrict__ eD,
                                                    int pre_ecorr, const long* __restrict__ ooff,
                                                    double* __restrict__ out, const double* __restrict__ eC) {
    const int inst = blockIdx.x;
    const InstDev I = insts[inst];
    const PsrDev& Pd = psrs[I.psr];
    const bool cmp = compact && Pd.dsplit;
    const GramView g = gram_view(Pd, I, Gpart, cmp, Sd, DD);
    const int W = I.K + 1;
    const int nep = pre_ecorr ? Pd.nep : 0;  // ECORR part added back: the Gram before elimination
    double* o = out + ooff[inst];
    for (long e = threadIdx.x; e < (long)W * W; e += blockDim.x) {
        const int i = (int)(e / W), j = (int)(e % W);
        double v = g(i, j);
        for (int q = 0; q < nep; q++)
            v += esum_col(Pd, I, esum, eC, cmp, q, i) * esum_col(Pd, I, esum, eC, cmp, q, j) / eD[I.epoff + q];
        o[e] = v;
    }
    for (int j = threadIdx.x; j < I.K; j += blockDim.x) o[(long)W * W + j] = colsq_of(Pd, I, colsq, nsplit, cmp, DCS, j);
}

// The design-matrix normalisation of the last pint_fit_step (pint_read_norms): per instance
// its K column norms squared in the fitter's original column order -- mode 1 (GLS) the
// unweighted column sums of squares of [M | F] (fitter.py:2164-2176 normalize_designmatrix),
// mode 0 (WLS) the whitened Gram's diagonal, the timing columns (fitter.py:1320-1343).
__global__ __launch_bounds__(64) void k_norms(const PsrDev* __restrict__ psrs, const InstDev* __restrict__ insts,
                                              const double* __restrict__ Gpart, const double* __restrict__ colsq,
                                              int nsplit, int compact, const double* __restrict__ Sd,
                                              const double* __restrict__ DD, const double* __restrict__ DCS, int mode,
                                              double* __restrict__ out) {
    const InstDev I = insts[blockIdx.x];
    const PsrDev& Pd = psrs[I.psr];
    const bool cmp = compact && Pd.dsplit;
    const GramView g = gram_view(Pd, I, Gpart, cmp, Sd, DD);
    for (int j = threadIdx.x; j < I.K; j += blockDim.x)
        out[I.coff + j] = mode == 1 ? colsq_of(Pd, I, colsq, nsplit, cmp, DCS, j) : g(j, j);
}

// ---------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------
// k_export: a step's fit outputs written straight into the caller's pinned host buffers by
// one kernel on the copy stream (lazy steps), instead of a runtime copy per output: the
// runtime's async D2H copies launch a blit kernel each, and twice per process one of them
// blocked the host ~7 ms (measured inside pint_step_end: with the driver's 5 warm-up steps
// both landed in the timed steps, 0.38 -> 0.75-1.1 ms per step over 20 steps).
constexpr int EXP_MAXSEG = 8;
struct ExportSeg {
    const double* src;
    double* dst;  // device-visible address of the pinned host buffer
    long n;
};
struct ExportArgs {
    ExportSeg seg[EXP_MAXSEG];
    int nseg;
    const int* st_src;  // the slot's status word (nullptr: none)
    int* st_dst;
};
__global__ __launch_bounds__(256) void k_export(ExportArgs a) {
    WgTimer wgt_(WGT_EXPORT);
    if (a.st_src && blockIdx.x == 0 && threadIdx.x == 0) *a.st_dst = *a.st_src;
    const long stride = (long)gridDim.x * 256;
    for (int k = 0; k < a.nseg; k++) {
        const double* __restrict__ s = a.seg[k].src;
        double* __restrict__ d = a.seg[k].dst;
        for (long i = blockIdx.x * 256L + threadIdx.x; i < a.seg[k].n; i += stride) d[i] = s[i];
    }
}

// Pulsar uploads (pint_add_pulsar) staged in page-locked chunks and committed a chunk at a
// time -- one device allocation and one asynchronous DMA per 16 MB chunk, the other chunk
// filled meanwhile -- with the last chunk committed at the first call that needs the device
// arrays (commit_uploads).  A PTA's 68 pulsars took 68 allocations and synchronous pageable
// copies of ~1.4 MB each (17 ms of its cold start; one pageable 95 MB copy: 16 ms).  The two
// staging chunks are a process-wide pool (StagePool), like the device allocation cache.
constexpr size_t STAGE_CHUNK = (size_t)16 << 20;
struct StagePool {
    std::mutex mu;
    char* buf[2] = {nullptr, nullptr};
    size_t cap[2] = {0, 0};
    bool busy = false;  // held by a context's pending uploads
};
static StagePool g_stage;
// page-locked host buffers of pint_host_alloc (start -> bytes): copies into them stay direct
static std::mutex g_pinned_mu;
static std::map<uintptr_t, size_t> g_pinned;
static bool host_pinned(const void* p, size_t bytes) {
    std::lock_guard<std::mutex> lk(g_pinned_mu);
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    auto it = g_pinned.upper_bound(a);
    if (it == g_pinned.begin()) return false;
    --it;
    return a + bytes <= it->first + it->second;
}
// device -> host copy.  Into pageable memory a large copy goes through the staging chunk (a
// page-locked buffer the uploads already made), synchronously, chunk by chunk: left to the
// runtime, it page-locks the caller's buffer for the copy, and registering or releasing
// such pages makes the driver evict and restore the process's queues -- a 12-33 ms stall of
// whichever synchronous call comes next (a fresh session's first fit, DESIGN §3 Round 6;
// none in 6 sessions with the runtime's own pinning turned off).  Small copies, copies into
// pint_host_alloc buffers, and a staging chunk in use by a context's uploads: direct.
constexpr size_t BOUNCE_MIN = (size_t)64 << 10;
static hipError_t d2h(void* dst, const void* src, size_t bytes, hipStream_t st) {
    if (bytes < BOUNCE_MIN || host_pinned(dst, bytes)) return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st);
    {
        std::lock_guard<std::mutex> lk(g_stage.mu);
        if (g_stage.busy || !g_stage.buf[0]) return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st);
        g_stage.busy = true;
    }
    // the two chunks alternate: chunk k's DMA runs while chunk k-1 is copied out on the host
    static hipEvent_t ev[2] = {nullptr, nullptr};  // (used under the busy flag only)
    hipError_t e = hipSuccess;
    const int nb = g_stage.buf[1] ? 2 : 1;
    const size_t cap = nb == 2 ? std::min(g_stage.cap[0], g_stage.cap[1]) : g_stage.cap[0];
    for (int b = 0; b < nb && e == hipSuccess; b++)
        if (!ev[b]) e = hipEventCreateWithFlags(&ev[b], hipEventDisableTiming);
    const size_t nch = (bytes + cap - 1) / cap;
    auto out = [&](size_t k) {  // chunk k (its DMA recorded) -> the caller's buffer
        const size_t off = k * cap, n = std::min(cap, bytes - off);
        hipError_t r = hipEventSynchronize(ev[k % nb]);
        if (r == hipSuccess) memcpy(static_cast<char*>(dst) + off, g_stage.buf[k % nb], n);
        return r;
    };
    for (size_t k = 0; k < nch && e == hipSuccess; k++) {
        const size_t off = k * cap, n = std::min(cap, bytes - off);
        if (nb == 1 && k > 0) e = out(k - 1);  // (one chunk: drained before it is refilled)
        if (e == hipSuccess)
            e = hipMemcpyAsync(g_stage.buf[k % nb], static_cast<const char*>(src) + off, n, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipEventRecord(ev[k % nb], st);
        if (e == hipSuccess && nb == 2 && k > 0) e = out(k - 1);
    }
    if (e == hipSuccess && nch > 0) e = out(nch - 1);
    std::lock_guard<std::mutex> lk(g_stage.mu);
    g_stage.busy = false;
    return e;
}
// host -> device, the same way round (blocking: hipMemcpy's semantics, else stream-ordered)
static hipError_t h2d(void* dst, const void* src, size_t bytes, hipStream_t st, bool blocking) {
    auto direct = [&]() {
        return blocking ? hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice)
                        : hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
    };
    if (bytes < BOUNCE_MIN || host_pinned(src, bytes)) return direct();
    {
        std::lock_guard<std::mutex> lk(g_stage.mu);
        if (g_stage.busy || !g_stage.buf[0]) return direct();
        g_stage.busy = true;
    }
    hipError_t e = hipSuccess;
    for (size_t off = 0; off < bytes && e == hipSuccess; off += g_stage.cap[0]) {
        const size_t n = std::min(g_stage.cap[0], bytes - off);
        memcpy(g_stage.buf[0], static_cast<const char*>(src) + off, n);
        if (blocking) {
            e = hipMemcpy(static_cast<char*>(dst) + off, g_stage.buf[0], n, hipMemcpyHostToDevice);
        } else {
            e = hipMemcpyAsync(static_cast<char*>(dst) + off, g_stage.buf[0], n, hipMemcpyHostToDevice, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
        }
    }
    std::lock_guard<std::mutex> lk(g_stage.mu);
    g_stage.busy = false;
    return e;
}
struct PendArena {
    struct Fix {
        size_t psr, field, off;  // pulsar, byte offset of the pointer field in its PsrDev, chunk offset
    };
    int cur = 0;               // the chunk being filled (g_stage.buf[cur])
    char* host = nullptr;      // == g_stage.buf[cur] while held
    size_t size = 0, cap = 0;
    std::vector<Fix> fix;
    hipEvent_t done[2] = {nullptr, nullptr};  // a chunk's DMA finished (reuse)
    bool inflight[2] = {false, false};
    long flushes = 0;
    bool held = false;
    size_t cur_idx = (size_t)-1;  // the pulsar being added (pint_add_pulsar) and its host record
    PsrDev* cur_dev = nullptr;
    std::vector<void*> bufs;      // the chunks' device allocations (freed with the context)
    ~PendArena() { release(); }
    void release() {
        for (int k = 0; k < 2; k++) {
            if (done[k]) {
                if (inflight[k]) hipEventSynchronize(done[k]);
                hipEventDestroy(done[k]);
                done[k] = nullptr;
            }
            inflight[k] = false;
        }
        if (held) {
            std::lock_guard<std::mutex> lk(g_stage.mu);
            g_stage.busy = false;
            held = false;
        }
        host = nullptr;
        cap = 0;
        size = 0;
        fix.clear();
    }
};

struct PsrHost {
    PsrDev dev;
    pint_spec_t spec;
    std::vector<int> dlo, dhi;  // row range of each DMX column's bin (compact layout)
    std::vector<int> drow_host; // DMX column of each TOA (-1: none), compact layout
    int dslot_ns = 0;           // vns the uploaded dslot was formed with (0: none)
    std::vector<void*> bufs;
    int n, K;
    double f1 = 0.0, f1_lo = 0.0;  // the red-noise fundamental (dd), k_trig_setup
};

struct pint_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t cstream = nullptr;   // copy stream: fit outputs -> host, overlapped with compute
    hipEvent_t ev_solved = nullptr, ev_copied = nullptr;
    hipStream_t sstream = nullptr;   // side stream: the Woodbury Sigma factor (k_sigma)
    hipEvent_t ev_gram = nullptr, ev_sigma = nullptr;
    bool sigma_pending = false;
    std::string err;
    std::vector<PsrHost> psrs;
    std::vector<int> setup_pending;  // pulsars whose red-noise set-up (k_trig_setup) is not run yet
    bool psrs_dirty = false;         // d_psrs lags ctx->psrs (pulsars added since the last refresh)
    PsrDev* d_psrs = nullptr;
    int npsr_dev = 0;
    // instances
    int ninst = 0;
    std::vector<InstDev> inst;
    InstDev* d_inst = nullptr;
    InstDev* d_inst_sorted = nullptr;   // instances grouped by k_gram T (full layout)
    InstDev* d_inst_sorted_c = nullptr; // ... compact layout
    InstDev* d_inst_sorted_v = nullptr; // ... compact layout, generated Fourier basis (k_gram_v)
    bool sorted_alias[3] = {false, false, false};  // a launch order equal to d_inst's: d_inst itself
    double* d_gridspec = nullptr;       // pint_set_grid: the base table and the grid axes
    std::vector<KpGroup> kp_groups, kp_groups_c, kp_groups_v;
    int vgram = 1;       // PINT_OPT_VGRAM
    int vbin = 1;        // PINT_OPT_VBIN: k_gram_v's binned DMX x Fourier tile
    int wbfit = 0;       // PINT_OPT_WBFIT: wideband DM rows in the fit step (k_wb_gram)
    int gv_pair = 1;     // PINT_GV_PAIR: k_gram_v launch order pairs heavy and light instances on a CU
    int maxn = 0;        // the batch's largest instance (rows)
    int max_ts = 0;      // the batch's largest parameter table (doubles)
    int resid12 = 1;     // PINT_RESID12: k_resid12 for batches of one-block instances without tiles
    int prep_lanes = 1;  // PINT_PREP_LANES: lane-per-instance k_prep / k_apply for small tables
    int fuse_r2 = 1;     // PINT_FUSE_R2: the fit layout's k_resid2 folded into k_gram_v's staging
    bool r2_pending = false;  // k_resid2 of the last pass deferred (the Gram formed its residuals)
    bool grid_valid = false;  // the batch is pint_set_grid's: grid_psr's points, options grid_opts
    std::vector<double> grid_spec_host;  // pint_set_grid's spec, kept while its upload may run
    int grid_psr = -1;
    long grid_opts = 0;
    int small = 1;       // PINT_OPT_SMALL: k_gram_s / one-wave k_solve_blk for small instances
    int schur = 1;       // PINT_SCHUR: k_schur forms the DMX-eliminated solve's S', U, b'_d (deferred solves)
    int evalb_wpe = 3;   // PINT_EVALB_WPE: one-model ELL1/DD batches with M at 3 waves/SIMD (0: the compiler's)
    int la_chol = 1;     // PINT_LA_CHOL: k_solve_dmx's look-ahead blocked Cholesky (0: blk_cholinv; the same bits)
    int solve_w8 = 1;    // PINT_SOLVE_W8: k_solve_dmx with 8 waves when the dense block fits (0: 16 waves)
    int eval0_wpe = 1;   // PINT_EVAL0_WPE: the isolated-model build at fixed register budgets (0: the compiler's)
    int eval_wpe = 3;    // PINT_EVAL_WPE: k_eval_mix<1>'s register budget in waves/SIMD (3: 168 VGPRs,
                         // 108 B of spills, 0.124 -> 0.105 ms; 4: 276 B of spills, slower; 0: none, 204)
    int n_vg = 0;        // instances on the k_gram_v path
    bool any_dmx_rows = false;  // compact instances still on k_dmx_rows / k_dmx
    double *d_TSp = nullptr, *d_TS = nullptr;  // k_gram_v per-split trig sums, their totals
    double* d_Sdp = nullptr;                    // k_gram_v DMX slot partials
    double* d_BFp = nullptr;                    // k_gram_v binned DMX x Fourier partials (VB)
    int vb_on = 0;                              // the batch's vg instances use VB
    double* d_xw = nullptr;     // k_solve_dmx's X, U and scalings for the deferred W, DMX errors and covariance
    int cov_defer = 1;          // PINT_COV_DEFER: the DMX-eliminated covariance in k_cov_dmx (0 never,
                                // 1 batches of >= 16 instances, 2 always)
    bool cov_pending = false;   // d_cov of the last solve not formed yet (k_cov_dmx at the read)
    int cov_mode = 0;
    size_t cov_lds = 0;
    bool ic_valid = false;  // per-instance constants (k_prep) current for the tables
    bool no_events = false; // PINT_NO_EVENTS=1: no per-kernel timing events (their cost)
    int timing_mask = 0xff; // PINT_OPT_TIMING_MASK: timing slots whose events are recorded
    int timing_every = 1;   // PINT_OPT_TIMING_EVERY: Gram events on every k-th fit step
    long gram_calls = 0;
    static constexpr int NSLOT = PINT_NSLOT;  // pipeline slots (pint_step_end / pint_check_step)
    hipGraph_t graph_s[NSLOT] = {};          // a captured launch sequence per pipeline
    hipGraphExec_t graph_exec_s[NSLOT] = {};  // slot (pint_capture_*, pint_graph_launch)
    bool capturing = false;
    int* d_blk_inst = nullptr;
    int* d_blk_row0 = nullptr;
    int* d_rblk_inst = nullptr;   // k_resid1/2 block -> instance
    double* d_rpart = nullptr;    // per residual block: sum w, sum w x, chi2 partial
    double* d_epart = nullptr;    // fused residual pass (efz): per evaluation block sum w, sum w x
    int efz = 0;                  // the batch's evaluation blocks carry k_resid1 (EF_ROWS rows + row 0 + TZR)
    int efuse = 1;                // PINT_EFUSE: fuse k_resid1 into the evaluation of large instances
    int lane_solve = 1;           // PINT_LANE_SOLVE: k_solve_lanes for small-instance batches of K <= 8
    std::vector<int> upsr;        // the batch's distinct pulsars (host plans loop over these, not instances)
    int spin_grid = 0;            // the resident grid's points differ in spin parameters only (k_eval_head/_spin)
    bool tables_fresh = false;    // ... and the tables are still pint_set_grid's (no step applied since)
    int spin_eval = 1;            // PINT_SPIN_EVAL: use the shared head for such grids
    double* d_shr = nullptr;      // its rows (EVAL_HEAD_W doubles each)
    long shr_cap = 0;
    int nrblk = 0;
    int eval_merge = 0;  // bit 0: one k_eval_mix launch without M, bit 1: with M, bit 2: also for a
                         // batch of one model (PINT_EVAL_MERGE)
    int nblk = 0;
    int blk_off[PINT_NBIN + 1] = {0};  // block ranges per binary model (PINT_BIN_*)
    long tot_table = 0, tot_rows = 0, tot_m = 0, tot_g = 0, tot_s = 0, tot_c = 0, tot_out = 0, tot_cv = 0;
    int lazy = 0;
    int blocked_solve = 1;  // k_solve_blk (MFMA, blocked) vs the column-by-column k_solve
    int refine = 1;         // PINT_OPT_REFINE: iterative refinement of ill-conditioned solves
    int gvdbg = 0;          // (experiment) k_gram_v phases switched off
    int nsplit = 1;
    double *d_tables = nullptr, *d_phhi = nullptr, *d_phlo = nullptr, *d_ftay = nullptr, *d_delay = nullptr;
    double *d_M = nullptr, *d_rt = nullptr, *d_rp = nullptr, *d_chi2 = nullptr, *d_chi2lin = nullptr;
    double *d_G = nullptr, *d_colsq = nullptr, *d_work = nullptr, *d_dpars = nullptr, *d_errs = nullptr;
    double *d_cov = nullptr, *d_sigL = nullptr, *d_lam = nullptr, *d_chi2g = nullptr;
    double *d_esum = nullptr, *d_eD = nullptr, *d_eW = nullptr, *d_ecs = nullptr, *d_wpart = nullptr;
    double* d_eC = nullptr;  // compact layout: each epoch's DMX entry c_e (k_ecorr)
    double* d_lognorm = nullptr;  // per instance: logdet(C)/2 of the last pint_chi2_gls
    double *d_eigw = nullptr, *d_degv = nullptr;  // k_eig scratch and dropped directions
    int* d_ndeg = nullptr;
    size_t eig_cap = 0;
    int degv_cap = 0;
    InstConst* d_ic = nullptr;  // per-instance constants (k_prep)
    InstConst* d_ic0 = nullptr; // the constants of the table snapshot (pint_save_tables)
    bool apply_req = false;     // pint_fit_step_apply: fuse the apply into the solve if possible
    bool apply_done = false;    //   ... and it was fused
    double apply_lam = 1.0;
    bool ic0_valid = false;
    double *d_dmxv = nullptr, *d_Sd = nullptr, *d_DD = nullptr, *d_DCS = nullptr;  // sparse-DMX layout
    double* d_dfac = nullptr;  // PLDMNoise basis scale per TOA row (only with PLDMNoise pulsars)
    int max_ndc = 0;
    int m_compact = 0;  // layout of the design matrix written by the last pint_eval(want_M)
    int red_valid[2] = {0, 0};  // red-noise columns of M already written (full, compact layout)
    size_t wpart_cap = 0;
    double *d_dmr = nullptr, *d_dmc2 = nullptr;  // wideband DM residuals / chi2 (pint_dm_resids)
    long dmr_cap = 0, dmc2_cap = 0;
    long tot_e = 0, tot_ep = 0;
    int max_nep = 0;
    int* d_status = nullptr;
    int* d_istatus = nullptr;  // per-instance status bits since the last pint_inst_status read
    double* d_rscr = nullptr;  // per-instance scratch vectors of the solves (RSCR doubles each)
    int maxK = 0;
    // HIP event pairs: 0/1 eval, 2/3 eval with design matrix, 4/5 resid, 6/7 ecorr + Gram +
    // reduction, 7/8 solve, 10/11 Woodbury chi2, 12/13 the Gram kernels alone, 14/15 k_greduce
    // (side stream)
    static constexpr int NEV = 16, NMS = 8;
    // pipelined steps (pint_step_end / pint_check_step): NSLOT slots, each with its own timing
    // events, status word and end-of-step event; non-pipelined use stays in slot 0
    int slot = 0;
    hipEvent_t ev_slot[NSLOT][NEV] = {};  // (created at their first record: most runs time nothing)
    bool rec_slot[NSLOT][NEV] = {{false}};
    hipEvent_t* ev = ev_slot[0];  // the current slot's events
    bool* rec = rec_slot[0];
    hipEvent_t ev_done[NSLOT] = {};
    hipEvent_t ev_cdone[NSLOT] = {};  // the step's output copies (copy stream)
    bool cdone_rec[NSLOT] = {};
    int* d_status_slots = nullptr;  // NSLOT status words on the device
    int* h_status = nullptr;        // their pinned host mirrors
    float ms[NMS] = {0, 0, 0, 0, 0, 0, 0, 0};
    double* d_nz = nullptr;  // pint_noise_lnlike scratch (parameters, epoch sums, outputs)
    size_t nz_cap = 0;
    double* d_noise = nullptr;  // pint_noise_resids: red and ECORR realisations (2 tot_out)
    long noise_cap = 0;
    double* d_tables0 = nullptr;  // pint_save_tables snapshot
    long tables0_cap = 0;
    bool restore_pending = false;  // pint_restore_tables not yet carried out (k_prep does it)
    double* chi2_dst = nullptr;    // lazy pint_chi2_gls: the host buffer of its deferred copy
    bool chi2_pending = false;     // d_chi2 not yet summed from the last residual pass's partials
    // fit outputs the copy stream reads, one set per pipeline slot: a step's solve writes its
    // slot's set while the copies of the previous step (the other slot) may still run, so the
    // solve need not wait for them (copy_pend[slot]: copies of that slot's set in flight)
    double *d_dpars_s[NSLOT] = {}, *d_errs_s[NSLOT] = {}, *d_cov_s[NSLOT] = {};
    double *d_chi2lin_s[NSLOT] = {}, *d_xw_s[NSLOT] = {}, *d_chi2g_s[NSLOT] = {};
    bool copy_pend[NSLOT] = {};
    bool dm_noise_pend = false;  // a copy-stream PLDMNoise realisation still reads d_dfac (lazy)
    int out_slot = -1;
    bool wfuse = false;            // the batch takes the fused Woodbury dots (k_resid2 tiles)
    bool wtile_valid = false;      // d_wpart holds the current residuals' dots (one split)
    double* d_wtile = nullptr;     // k_resid2's per-block trig tiles (256 per residual block)
    double* d_norms = nullptr;     // pint_read_norms: per-instance K vectors (coff)
    double* d_ones = nullptr;      // k_onesrow: the Woodbury ones row without an Offset column (coff)
    int wstride = 0;
    hipEvent_t ev_noise = nullptr;
    // lazy copy-stream work of the current step (pint_read_step's k_cov_dmx and copies, the
    // noise realisations): enqueued at the step's end (pint_step_end, after ev_done) or at
    // pint_check, behind the kernel stream's last kernel -- so no cross-stream event sits
    // inside the step (the solve's dispatch carried ev_solved: ~5 us of idle stream after it)
    PendArena pend;              // pulsar uploads not committed to the device yet
    // pint_add_pulsar_cols: the packed columns of the pulsar being added (reused: the pages of
    // a 10k-TOA pulsar's 1.4 MB are touched once per context, not once per pulsar)
    std::vector<double> pk_d;
    std::vector<uint64_t> pk_j;
    std::vector<uint32_t> pk_f;
    std::vector<int32_t> pk_i, pk_x;
    std::vector<std::function<int()>> cq;
    std::vector<ExportSeg> exp;  // the deferred work's host-bound outputs (k_export at the flush)
    const int* exp_st_src = nullptr;
    int* exp_st_dst = nullptr;
    // (Tried: holding a closed step's cq back until the next step's solve starts -- an event
    // on k_schur's dispatch -- so its kernels and blit copies run beside the one-workgroup-
    // per-instance solve: the event cost a ~6 us gap and the copy-stream workgroups slowed the
    // solve itself, 0.226 vs 0.193 ms per 9-pulsar step; dropped.)
};

static bool any_copy_pend(const pint_ctx* ctx) {
    for (int sl = 0; sl < pint_ctx::NSLOT; sl++)
        if (ctx->copy_pend[sl]) return true;
    return false;
}
static void clear_copy_pend(pint_ctx* ctx) {
    for (int sl = 0; sl < pint_ctx::NSLOT; sl++) ctx->copy_pend[sl] = false;
}
// a host-bound output of the deferred work: a k_export segment when it is small and the
// destination pinned (device-visible), else a runtime copy on the copy stream now (the
// runtime's blit copy streams large outputs over PCIe faster than a kernel's stores: k_export
// for everything, 7.4 MB of covariances and 5.4 MB of noise realisations per 68-pulsar step,
// took the step from 0.38 to 0.50-0.77 ms)
constexpr long EXP_MAX_BYTES = 1L << 20;
static int export_seg(pint_ctx* ctx, double* dst, const double* src, long n) {
    if (!dst || n <= 0) return PINT_OK;
    void* dd = nullptr;
    static const long max_bytes = getenv("PINT_EXPORT_MAX") ? atol(getenv("PINT_EXPORT_MAX")) : EXP_MAX_BYTES;
    if (n * (long)sizeof(double) <= max_bytes && (int)ctx->exp.size() < EXP_MAXSEG &&
        hipHostGetDevicePointer(&dd, dst, 0) == hipSuccess && dd) {
        ctx->exp.push_back(ExportSeg{src, static_cast<double*>(dd), n});
        return PINT_OK;
    }
    (void)hipGetLastError();
    HIPCHK(d2h(dst, src, sizeof(double) * n, ctx->cstream));
    return PINT_OK;
}
static int launch_export(pint_ctx* ctx) {
    if (ctx->exp.empty() && !ctx->exp_st_src) return PINT_OK;
    ExportArgs a{};
    a.nseg = (int)ctx->exp.size();
    long tot = 0;
    for (int k = 0; k < a.nseg; k++) {
        a.seg[k] = ctx->exp[k];
        tot += a.seg[k].n;
    }
    a.st_src = ctx->exp_st_src;
    a.st_dst = ctx->exp_st_dst;
    // a few workgroups: the writes are posted over PCIe (~50 GB/s), and workgroups on every
    // CU waiting on them slowed the step's kernels beside them (256: 0.60 ms per step)
    static const int wg = getenv("PINT_EXPORT_WG") ? std::max(1, atoi(getenv("PINT_EXPORT_WG"))) : 4;
    const int nb = (int)std::max<long>(1, std::min<long>(wg, (tot + 4095) / 4096));
    hipLaunchKernelGGL(k_export, dim3(nb), dim3(256), 0, ctx->cstream, a);
    HIPCHK(hipGetLastError());
    ctx->exp.clear();
    ctx->exp_st_src = nullptr;
    ctx->exp_st_dst = nullptr;
    return PINT_OK;
}

// PINT_TRACE_ENQ=1: host-side stalls (> 1 ms) of single runtime calls on the step path
struct HostLap {
    const char* where;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    static bool on() {
        static const bool v = getenv("PINT_TRACE_ENQ") && atoi(getenv("PINT_TRACE_ENQ"));
        return v;
    }
    void operator()(const char* what) {
        if (!on()) return;
        const auto n = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(n - t).count();
        if (ms > 1.0) fprintf(stderr, "[pint %s] %s took %.3f ms\n", where, what, ms);
        t = n;
    }
};

// enqueue the deferred copy-stream work behind `after` (an event just recorded on the kernel
// stream); ev_copied then covers it, and copy_pend marks the current slot's outputs in flight
static int flush_cq(pint_ctx* ctx, hipEvent_t after) {
    if (ctx->cq.empty() && ctx->exp.empty() && !ctx->exp_st_src) return PINT_OK;
    HostLap lap{"flush_cq"};
    HIPCHK(hipStreamWaitEvent(ctx->cstream, after, 0));
    lap("wait event");
    std::vector<std::function<int()>> ops;
    ops.swap(ctx->cq);
    for (auto& op : ops) {
        if (int rc = op()) return rc;
        lap("an op");
    }
    if (int rc = launch_export(ctx)) return rc;
    lap("export");
    HIPCHK(hipEventRecord(ctx->ev_copied, ctx->cstream));
    lap("record ev_copied");
    ctx->copy_pend[ctx->slot] = true;
    return PINT_OK;
}
// ... behind everything enqueued on the kernel stream so far (a marker event): before a launch
// rewrites what the deferred work reads (a second fit step in the same slot, the DM-noise scale)
static int flush_cq_now(pint_ctx* ctx) {
    if (ctx->cq.empty()) return PINT_OK;
    HIPCHK(hipEventRecord(ctx->ev_solved, ctx->stream));
    return flush_cq(ctx, ctx->ev_solved);
}

// Point the context's fit-output buffers at pipeline slot sl's set.
static void select_out_slot(pint_ctx* ctx, int sl) {
    if (ctx->out_slot == sl) return;
    ctx->out_slot = sl;
    ctx->d_dpars = ctx->d_dpars_s[sl];
    ctx->d_errs = ctx->d_errs_s[sl];
    ctx->d_cov = ctx->d_cov_s[sl];
    ctx->d_chi2lin = ctx->d_chi2lin_s[sl];
    ctx->d_xw = ctx->d_xw_s[sl];
    ctx->d_chi2g = ctx->d_chi2g_s[sl];
}

// Per-instance buffers (eval rows, design matrices, Gram partials: tens of GB for a large
// grid batch) go through a process-wide cache per device: hipMalloc/hipFree of that much
// memory costs ~0.3 s per batch, while grid_chisq / Session re-creation re-requests the same
// sizes.  Freed buffers stay mapped and are handed out again to a request of <= their size
// (within 25%); a failed hipMalloc releases the cache and retries.  pint_release_cache()
// returns it all to the runtime.  PINT_CACHE_POISON=1 fills every handed-out buffer with
// NaN bytes (checks that no kernel reads memory it did not write).
struct DevCache {
    std::multimap<size_t, void*> idle;
    std::map<void*, size_t> live;
    size_t idle_bytes = 0;
};
static std::mutex g_cache_mu;
static DevCache g_cache[64];
static const size_t CACHE_MAX_IDLE = (size_t)128 << 30;
static int g_poison = -1;

static size_t cache_round(size_t b) {
    if (b == 0) b = 8;
    if (b >= ((size_t)1 << 20)) return (b + ((size_t)2 << 20) - 1) & ~(((size_t)2 << 20) - 1);
    return (b + 255) & ~(size_t)255;
}

static void cache_trim(int dev, size_t keep) {  // caller holds g_cache_mu
    DevCache& c = g_cache[dev & 63];
    while (c.idle_bytes > keep && !c.idle.empty()) {
        auto it = std::prev(c.idle.end());  // largest first
        hipFree(it->second);
        c.idle_bytes -= it->first;
        c.idle.erase(it);
    }
}

static hipError_t cmalloc(void** p, size_t bytes) {
    int dev = 0;
    hipGetDevice(&dev);
    size_t b = cache_round(bytes);
    if (g_poison < 0) {
        const char* e = getenv("PINT_CACHE_POISON");
        g_poison = (e && e[0] == '1') ? 1 : 0;
    }
    std::lock_guard<std::mutex> lk(g_cache_mu);
    DevCache& c = g_cache[dev & 63];
    *p = nullptr;
    auto it = c.idle.lower_bound(b);
    if (it != c.idle.end() && it->first <= b + b / 4) {
        *p = it->second;
        c.live[*p] = it->first;
        c.idle_bytes -= it->first;
        c.idle.erase(it);
    } else {
        hipError_t e = hipMalloc(p, b);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            cache_trim(dev, 0);
            e = hipMalloc(p, b);
            if (e != hipSuccess) return e;
        }
        c.live[*p] = b;
    }
    if (g_poison == 1) {
        hipError_t e = hipMemset(*p, 0xff, b);
        return e != hipSuccess ? e : hipDeviceSynchronize();  // ordered before any stream's use
    }
    return hipSuccess;
}

static void dfree(void*& p) {
    if (!p) return;
    int dev = 0;
    hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(g_cache_mu);
    DevCache& c = g_cache[dev & 63];
    auto it = c.live.find(p);
    if (it == c.live.end()) {
        hipFree(p);
    } else {
        c.idle.emplace(it->second, p);
        c.idle_bytes += it->second;
        c.live.erase(it);
        cache_trim(dev, CACHE_MAX_IDLE);
    }
    p = nullptr;
}

extern "C" void pint_release_cache(void) {
    int n = 0;
    hipGetDeviceCount(&n);
    std::lock_guard<std::mutex> lk(g_cache_mu);
    int cur = 0;
    hipGetDevice(&cur);
    for (int d = 0; d < n && d < 64; d++) {
        if (g_cache[d].idle.empty()) continue;
        hipSetDevice(d);
        cache_trim(d, 0);
    }
    hipSetDevice(cur);
}

// k_trig_setup + k_trig_sum over a list of jobs (one sync at the end)
static int run_trig_jobs(pint_ctx* ctx, std::vector<TrigJob>& jobs) {
    if (jobs.empty()) return 0;
    int nb = 0;
    for (auto& J : jobs) {
        J.b0 = nb;
        J.nb = (J.n + TRIG_RB - 1) / TRIG_RB;
        nb += J.nb;
    }
    void *part = nullptr, *dj = nullptr;
    HIPCHK(cmalloc(&part, sizeof(double) * 512 * (size_t)std::max(1, nb)));
    HIPCHK(cmalloc(&dj, sizeof(TrigJob) * jobs.size()));
    HIPCHK(h2d(dj, jobs.data(), sizeof(TrigJob) * jobs.size(), ctx->stream, false));
    hipLaunchKernelGGL(k_trig_setup, dim3(nb), dim3(256), sizeof(double) * 4 * 48 * WT_CS, ctx->stream,
                       (const TrigJob*)dj, (int)jobs.size(), (double*)part);
    hipLaunchKernelGGL(k_trig_sum, dim3((unsigned)jobs.size()), dim3(256), 0, ctx->stream, (const TrigJob*)dj,
                       (const double*)part);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(ctx->stream));
    dfree(part);
    dfree(dj);
    return 0;
}

static TrigJob trig_job(const PsrHost& ph, bool base) {
    const PsrDev& d = ph.dev;
    TrigJob J{};
    J.tdb_hi = d.tdb_hi;
    J.tdb_lo = d.tdb_lo;
    J.isig = d.isig;
    J.cs = (double*)d.red_cs;
    J.trigU = base ? (double*)d.trigU : nullptr;
    J.trigW = (double*)d.trigW;
    J.f1 = ph.f1;
    J.f1_lo = ph.f1_lo;
    J.n = ph.n;
    J.base = base ? 1 : 0;
    return J;
}

// the red-noise set-up of every pulsar added since the last flush, batched: e^{i theta},
// e^{i 8 theta} per TOA and the trig sums U_m, V_m, C_m, S_m (k_trig_setup + k_trig_sum)
static int commit_uploads(pint_ctx* ctx);
static int flush_setup(pint_ctx* ctx) {
    if (commit_uploads(ctx)) return 1;
    if (ctx->setup_pending.empty()) return 0;
    std::vector<TrigJob> jobs;
    for (int p : ctx->setup_pending) jobs.push_back(trig_job(ctx->psrs[p], true));
    ctx->setup_pending.clear();
    return run_trig_jobs(ctx, jobs);
}

// the weighted trig sums of a pulsar with red noise (PsrDev::trigW) from its current isig
static int form_trigw(pint_ctx* ctx, const PsrHost& ph) {
    if (!ph.dev.trigW || !ph.dev.red_cs || ph.n <= 0) return 0;
    if (flush_setup(ctx)) return 1;  // red_cs first
    std::vector<TrigJob> jobs{trig_job(ph, false)};
    return run_trig_jobs(ctx, jobs);
}

template <typename T>
static int upload(pint_ctx* ctx, PsrHost& ph, const T* src, size_t count, const T*& dst) {
    void* p = nullptr;
    size_t bytes = count * sizeof(T);
    if (bytes == 0) bytes = sizeof(T);
    HIPCHK(hipMalloc(&p, bytes));
    if (src && count) HIPCHK(h2d(p, src, count * sizeof(T), nullptr, true));
    else HIPCHK(hipMemset(p, 0, bytes));
    ph.bufs.push_back(p);
    dst = (const T*)p;
    return 0;
}

// the current chunk to the device: its allocation, an asynchronous DMA, its pointers set
static int flush_chunk(pint_ctx* ctx) {
    PendArena& pa = ctx->pend;
    if (pa.fix.empty()) return PINT_OK;
    void* p = nullptr;
    HIPCHK(hipMalloc(&p, std::max<size_t>(pa.size, 256)));
    HIPCHK(h2d(p, pa.host, pa.size, ctx->stream, false));
    if (!pa.done[pa.cur]) HIPCHK(hipEventCreateWithFlags(&pa.done[pa.cur], hipEventDisableTiming));
    HIPCHK(hipEventRecord(pa.done[pa.cur], ctx->stream));
    pa.inflight[pa.cur] = true;
    for (auto& f : pa.fix) {
        PsrDev* tgt = f.psr < ctx->psrs.size() ? &ctx->psrs[f.psr].dev : (f.psr == pa.cur_idx ? pa.cur_dev : nullptr);
        if (tgt)
            *reinterpret_cast<const void**>(reinterpret_cast<char*>(tgt) + f.field) =
                static_cast<const void*>(static_cast<char*>(p) + f.off);
    }
    pa.bufs.push_back(p);
    pa.fix.clear();
    pa.size = 0;
    pa.flushes++;
    // the other chunk next (once its own DMA has finished)
    pa.cur ^= 1;
    if (pa.inflight[pa.cur]) {
        HIPCHK(hipEventSynchronize(pa.done[pa.cur]));
        pa.inflight[pa.cur] = false;
    }
    pa.host = g_stage.buf[pa.cur];
    pa.cap = g_stage.cap[pa.cur];
    return PINT_OK;
}
// commit every staged pulsar upload; the device arrays are complete when the stream reaches
// here (kernels on ctx->stream follow the DMAs), and the staging chunks go back to the pool
static int commit_uploads(pint_ctx* ctx) {
    PendArena& pa = ctx->pend;
    if (!pa.held) return PINT_OK;
    if (int rc = flush_chunk(ctx)) return rc;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    pa.release();
    return PINT_OK;
}
// hold the process's staging chunks (page-locked, STAGE_CHUNK each) for this context
static bool stage_hold(pint_ctx* ctx) {
    PendArena& pa = ctx->pend;
    if (pa.held) return true;
    std::lock_guard<std::mutex> lk(g_stage.mu);
    if (g_stage.busy) return false;  // (another context is staging: it uses the pageable path)
    for (int k = 0; k < 2; k++)
        if (!g_stage.buf[k]) {
            if (hipHostMalloc((void**)&g_stage.buf[k], STAGE_CHUNK, hipHostMallocDefault) != hipSuccess) {
                g_stage.buf[k] = nullptr;
                return false;
            }
            {
                std::lock_guard<std::mutex> pk(g_pinned_mu);
                g_pinned[reinterpret_cast<uintptr_t>(g_stage.buf[k])] = STAGE_CHUNK;
            }
            g_stage.cap[k] = STAGE_CHUNK;
        }
    g_stage.busy = true;
    pa.held = true;
    pa.cur = 0;
    pa.host = g_stage.buf[0];
    pa.cap = g_stage.cap[0];
    pa.size = 0;
    return true;
}
// stage count elements (zeros when src is null) for the PsrDev pointer field dst of pulsar psr;
// false: not staged (no pool chunk, or larger than a chunk) -- the caller uploads it itself
template <typename T>
static bool stage(pint_ctx* ctx, size_t psr, PsrDev& d, const T* src, size_t count, const T*& dst) {
    PendArena& pa = ctx->pend;
    const size_t bytes = std::max(count * sizeof(T), sizeof(T));
    if (bytes > STAGE_CHUNK || !stage_hold(ctx)) return false;
    size_t off = (pa.size + 255) & ~(size_t)255;
    if (off + bytes > pa.cap) {
        if (flush_chunk(ctx)) return false;
        off = 0;
    }
    if (src && count) memcpy(pa.host + off, src, count * sizeof(T));
    else memset(pa.host + off, 0, bytes);
    pa.size = off + bytes;
    pa.fix.push_back(PendArena::Fix{psr, (size_t)(reinterpret_cast<const char*>(&dst) - reinterpret_cast<const char*>(&d)), off});
    return true;
}

extern "C" {
static int set_instances_impl(pint_ctx* ctx, int ninst, const int32_t* inst_psr, const double* tables);
}

// pint_set_grid: tables[k] = base with each grid variable's (hi, lo) pair set (see there)
__global__ __launch_bounds__(256) void k_grid_tables(const double* __restrict__ spec, int ts, int nvar, int npts,
                                                     long k0, double* __restrict__ tables) {
    const long total = (long)npts * ts;
    const double* hdr = spec + ts;
    const double* vals = hdr + 4 * nvar;
    for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
        const long k = e / ts;
        const int i = (int)(e - k * ts);
        double v = spec[i];
        for (int j = 0; j < nvar; j++) {
            const int o = (int)hdr[4 * j];
            if (i != o && i != o + 1) continue;
            const long st = (long)hdr[4 * j + 1], sz = (long)hdr[4 * j + 2], vo = (long)hdr[4 * j + 3];
            const long q = ((k0 + k) / st) % sz;
            v = vals[2 * (vo + q) + (i - o)];
        }
        tables[e] = v;
    }
}

static int refresh_psrs(pint_ctx* ctx) {
    if (int rc = commit_uploads(ctx)) return rc;
    ctx->psrs_dirty = false;
    if (ctx->d_psrs) hipFree(ctx->d_psrs);
    ctx->d_psrs = nullptr;
    std::vector<PsrDev> all;
    for (auto& p : ctx->psrs) all.push_back(p.dev);
    HIPCHK(hipMalloc(&ctx->d_psrs, sizeof(PsrDev) * all.size()));
    HIPCHK(h2d(ctx->d_psrs, all.data(), sizeof(PsrDev) * all.size(), nullptr, true));
    return 0;
}

extern "C" {

int pint_nslot(void) { return pint_ctx::NSLOT; }

int pint_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// Streams outlive their contexts: a destroyed context's streams go back to per-device pools,
// one per role (kernel, copy, side stream), and a later context takes the oldest (first
// created) of each role, so the k-th context alive on a device always runs on the streams the k-th context
// ever created had -- on the same hardware queues.  HIP maps each new stream onto one of
// GPU_MAX_HW_QUEUES hardware queues as it is created; with streams destroyed and recreated
// the mapping of a later context's streams changed from context to context, and so did the
// speed of several contexts' steps run concurrently (bench.py --pipes: 2 x 9-pulsar
// pipelines 0.105 or 0.138 ms per step by which streams a shard's sessions had got).
static std::mutex g_stream_mu;
static std::map<int, std::map<long, hipStream_t>> g_stream_pool[3];  // per role: creation rank -> idle stream
static std::map<hipStream_t, long> g_stream_rank;
static long g_stream_made = 0;
enum { STREAM_KERNEL = 0, STREAM_COPY = 1, STREAM_SIDE = 2 };
static int g_stream_pool_on = -1;  // PINT_STREAM_POOL=0: every context creates and destroys its own
static bool stream_pool_on() {
    if (g_stream_pool_on < 0) g_stream_pool_on = getenv("PINT_STREAM_POOL") ? (atoi(getenv("PINT_STREAM_POOL")) != 0) : 1;
    return g_stream_pool_on != 0;
}
static hipStream_t stream_get(int device, int role) {
    std::lock_guard<std::mutex> lk(g_stream_mu);
    auto& v = g_stream_pool[role][device];
    if (stream_pool_on() && !v.empty()) {  // the oldest idle stream of the role
        hipStream_t s = v.begin()->second;
        v.erase(v.begin());
        return s;
    }
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    g_stream_rank[s] = g_stream_made++;
    return s;
}
static void stream_put(int device, int role, hipStream_t s) {
    if (!s) return;
    hipStreamSynchronize(s);
    if (!stream_pool_on()) {
        hipStreamDestroy(s);
        return;
    }
    std::lock_guard<std::mutex> lk(g_stream_mu);
    g_stream_pool[role][device][g_stream_rank[s]] = s;
}

pint_ctx* pint_ctx_create(int device) {
    pint_ctx* ctx = new pint_ctx();
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess) {
        ctx->err = "hipSetDevice failed";
        return ctx;
    }
    // (stream priorities -- the kernel stream highest, the copy stream lowest -- measured no
    // different in round 4: 0.376-0.384 vs 0.380-0.387 ms per 68-pulsar step)
    ctx->stream = stream_get(device, STREAM_KERNEL);
    ctx->cstream = stream_get(device, STREAM_COPY);
    // the cross-stream events are waited on by the device (and ev_done by the host only for
    // completion: everything the host reads comes through copies covered by ev_cdone), so they
    // release to device scope: the default system-scope release writes back the caches and
    // idled the stream ~4-8 us at each such event, measured (PINT_EV_SYSTEM=1 restores it)
    const unsigned evf = hipEventDisableTiming |
                         ((getenv("PINT_EV_SYSTEM") && atoi(getenv("PINT_EV_SYSTEM"))) ? 0u : hipEventReleaseToDevice);
    hipEventCreateWithFlags(&ctx->ev_solved, evf);
    hipEventCreateWithFlags(&ctx->ev_copied, evf);
    hipEventCreateWithFlags(&ctx->ev_noise, evf);
    // PINT_SERIAL=1 (profiling aid): side-stream kernels run on the main stream, so
    // rocprof's per-kernel durations are not inflated by concurrent kernels
    if (getenv("PINT_SERIAL") && atoi(getenv("PINT_SERIAL"))) ctx->sstream = ctx->stream;
    else ctx->sstream = stream_get(device, STREAM_SIDE);
    ctx->no_events = getenv("PINT_NO_EVENTS") && atoi(getenv("PINT_NO_EVENTS"));
    ctx->eval_merge = getenv("PINT_EVAL_MERGE") ? atoi(getenv("PINT_EVAL_MERGE")) : 3;
    ctx->vbin = getenv("PINT_VBIN") ? (atoi(getenv("PINT_VBIN")) ? 1 : 0) : 1;  // PINT_OPT_VBIN default
    ctx->cov_defer = getenv("PINT_COV_DEFER") ? atoi(getenv("PINT_COV_DEFER")) : 1;  // 0 off, 1 batches, 2 always
    ctx->eval_wpe = getenv("PINT_EVAL_WPE") ? atoi(getenv("PINT_EVAL_WPE")) : 3;
    ctx->gv_pair = getenv("PINT_GV_PAIR") ? atoi(getenv("PINT_GV_PAIR")) : 1;
    ctx->schur = getenv("PINT_SCHUR") ? atoi(getenv("PINT_SCHUR")) : 1;
    ctx->fuse_r2 = getenv("PINT_FUSE_R2") ? atoi(getenv("PINT_FUSE_R2")) : 1;
    ctx->eval0_wpe = getenv("PINT_EVAL0_WPE") ? atoi(getenv("PINT_EVAL0_WPE")) : 1;
    ctx->prep_lanes = getenv("PINT_PREP_LANES") ? atoi(getenv("PINT_PREP_LANES")) : 1;
    ctx->resid12 = getenv("PINT_RESID12") ? atoi(getenv("PINT_RESID12")) : 1;
    ctx->evalb_wpe = getenv("PINT_EVALB_WPE") ? atoi(getenv("PINT_EVALB_WPE")) : 3;
    ctx->la_chol = getenv("PINT_LA_CHOL") ? atoi(getenv("PINT_LA_CHOL")) : 1;
    ctx->solve_w8 = getenv("PINT_SOLVE_W8") ? atoi(getenv("PINT_SOLVE_W8")) : 1;
    ctx->efuse = getenv("PINT_EFUSE") ? atoi(getenv("PINT_EFUSE")) : 1;
    ctx->lane_solve = getenv("PINT_LANE_SOLVE") ? atoi(getenv("PINT_LANE_SOLVE")) : 1;
    ctx->spin_eval = getenv("PINT_SPIN_EVAL") ? atoi(getenv("PINT_SPIN_EVAL")) : 1;
    hipEventCreateWithFlags(&ctx->ev_gram, evf);
    hipEventCreateWithFlags(&ctx->ev_sigma, evf);
    for (int sl = 0; sl < pint_ctx::NSLOT; sl++) {
        hipEventCreateWithFlags(&ctx->ev_done[sl], evf);
        hipEventCreateWithFlags(&ctx->ev_cdone[sl], hipEventDisableTiming);
    }
    hipMalloc(&ctx->d_status_slots, pint_ctx::NSLOT * sizeof(int));
    hipMemset(ctx->d_status_slots, 0, pint_ctx::NSLOT * sizeof(int));
    ctx->d_status = ctx->d_status_slots;
    hipHostMalloc(&ctx->h_status, pint_ctx::NSLOT * sizeof(int), hipHostMallocDefault);
    if (ctx->h_status)
        for (int sl = 0; sl < pint_ctx::NSLOT; sl++) ctx->h_status[sl] = 0;
    return ctx;
}

const char* pint_last_error(pint_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

static void free_instances(pint_ctx* ctx) {
    // the buffers go back to the device cache, where another context may take them
    if (ctx->stream) hipStreamSynchronize(ctx->stream);
    if (ctx->cstream) hipStreamSynchronize(ctx->cstream);
    if (ctx->sstream) hipStreamSynchronize(ctx->sstream);
    InstDev** sorted[3] = {&ctx->d_inst_sorted, &ctx->d_inst_sorted_c, &ctx->d_inst_sorted_v};
    for (int l = 0; l < 3; l++) {  // (aliases of d_inst: freed once, below)
        if (ctx->sorted_alias[l]) *sorted[l] = nullptr;
        ctx->sorted_alias[l] = false;
    }
    dfree((void*&)ctx->d_gridspec);
    dfree((void*&)ctx->d_shr);
    ctx->shr_cap = 0;
    ctx->spin_grid = 0;
    for (int sl = 0; sl < pint_ctx::NSLOT; sl++) {
        void** pss[] = {(void**)&ctx->d_chi2lin_s[sl], (void**)&ctx->d_dpars_s[sl], (void**)&ctx->d_errs_s[sl],
                        (void**)&ctx->d_cov_s[sl], (void**)&ctx->d_chi2g_s[sl], (void**)&ctx->d_xw_s[sl]};
        for (auto p : pss) dfree(*p);
    }
    void** ps[] = {(void**)&ctx->d_inst, (void**)&ctx->d_inst_sorted, (void**)&ctx->d_blk_inst, (void**)&ctx->d_blk_row0, (void**)&ctx->d_tables,
                   (void**)&ctx->d_phhi, (void**)&ctx->d_phlo, (void**)&ctx->d_ftay, (void**)&ctx->d_delay,
                   (void**)&ctx->d_M, (void**)&ctx->d_rt, (void**)&ctx->d_rp, (void**)&ctx->d_chi2, (void**)&ctx->d_istatus, (void**)&ctx->d_rscr,
                   (void**)&ctx->d_G, (void**)&ctx->d_colsq,
                   (void**)&ctx->d_work, (void**)&ctx->d_sigL,
                   (void**)&ctx->d_lam, (void**)&ctx->d_lognorm,
                   (void**)&ctx->d_eigw,
                   (void**)&ctx->d_degv, (void**)&ctx->d_ndeg, (void**)&ctx->d_esum, (void**)&ctx->d_eD,
                   (void**)&ctx->d_eW, (void**)&ctx->d_eC, (void**)&ctx->d_ecs, (void**)&ctx->d_wpart, (void**)&ctx->d_ic, (void**)&ctx->d_ic0,
                   (void**)&ctx->d_dmxv, (void**)&ctx->d_Sd, (void**)&ctx->d_DD, (void**)&ctx->d_DCS,
                   (void**)&ctx->d_dfac, (void**)&ctx->d_inst_sorted_c, (void**)&ctx->d_inst_sorted_v, (void**)&ctx->d_Sdp,
                   (void**)&ctx->d_BFp, (void**)&ctx->d_TSp, (void**)&ctx->d_TS, (void**)&ctx->d_rblk_inst, (void**)&ctx->d_rpart, (void**)&ctx->d_epart,
                   (void**)&ctx->d_noise, (void**)&ctx->d_tables0,
                   (void**)&ctx->d_wtile, (void**)&ctx->d_norms, (void**)&ctx->d_ones};
    for (auto p : ps) dfree(*p);
    ctx->d_dpars = ctx->d_errs = ctx->d_cov = ctx->d_chi2lin = ctx->d_xw = ctx->d_chi2g = nullptr;
    clear_copy_pend(ctx);
    ctx->noise_cap = 0;
    ctx->tables0_cap = 0;
    ctx->ic0_valid = false;
    ctx->restore_pending = false;
    ctx->wfuse = ctx->wtile_valid = false;
    for (int k = 0; k < pint_ctx::NSLOT; k++) {
        if (ctx->graph_exec_s[k]) hipGraphExecDestroy(ctx->graph_exec_s[k]);
        if (ctx->graph_s[k]) hipGraphDestroy(ctx->graph_s[k]);
        ctx->graph_exec_s[k] = nullptr;
        ctx->graph_s[k] = nullptr;
    }
    ctx->ninst = 0;
    ctx->wpart_cap = 0;
    ctx->eig_cap = 0;
    ctx->degv_cap = 0;
}

void pint_ctx_destroy(pint_ctx* ctx) {
    if (!ctx) return;
    hipSetDevice(ctx->device);
    ctx->cq.clear();  // deferred reads never enqueued: their host buffers are not filled
    hipStreamSynchronize(ctx->stream);
    free_instances(ctx);
    ctx->pend.release();
    for (auto b : ctx->pend.bufs) hipFree(b);
    for (auto& p : ctx->psrs) {
        for (auto b : p.bufs) hipFree(b);
    }
    if (ctx->d_psrs) hipFree(ctx->d_psrs);
    if (ctx->d_dmr) hipFree(ctx->d_dmr);
    if (ctx->d_dmc2) hipFree(ctx->d_dmc2);
    if (ctx->d_nz) hipFree(ctx->d_nz);
    if (ctx->d_status_slots) hipFree(ctx->d_status_slots);
    if (ctx->h_status) hipHostFree(ctx->h_status);
    for (int sl = 0; sl < pint_ctx::NSLOT; sl++) {
        for (int i = 0; i < pint_ctx::NEV; i++)
            if (ctx->ev_slot[sl][i]) hipEventDestroy(ctx->ev_slot[sl][i]);
        if (ctx->ev_done[sl]) hipEventDestroy(ctx->ev_done[sl]);
        if (ctx->ev_cdone[sl]) hipEventDestroy(ctx->ev_cdone[sl]);
    }
    if (ctx->cstream) hipStreamSynchronize(ctx->cstream);
    if (ctx->ev_solved) hipEventDestroy(ctx->ev_solved);
    if (ctx->ev_copied) hipEventDestroy(ctx->ev_copied);
    if (ctx->ev_noise) hipEventDestroy(ctx->ev_noise);
    if (ctx->sstream) hipStreamSynchronize(ctx->sstream);
    if (ctx->ev_gram) hipEventDestroy(ctx->ev_gram);
    if (ctx->ev_sigma) hipEventDestroy(ctx->ev_sigma);
    if (ctx->sstream && ctx->sstream != ctx->stream) stream_put(ctx->device, STREAM_SIDE, ctx->sstream);
    stream_put(ctx->device, STREAM_COPY, ctx->cstream);
    stream_put(ctx->device, STREAM_KERNEL, ctx->stream);
    delete ctx;
}

// engine.pack_toas in native code, bit-identical to it: every column with the TZR row appended,
// flags = is_bary | all(ssb_obs_pos != 0) << 1, sigma_s = sigma_us * 1e-6, and each TOA's DMX
// bins in parameter order (toa_select.py:101, inclusive ranges; dispersion_model.py:659-678 sums
// every selecting bin): the first two in dmx_a/dmx_b, any further ones in the dmx_x CSR.  Ranges
// that sorted by start have non-decreasing ends hold MJD t in the sorted positions lo..hi
// (lo = #(ends < t), hi = #(starts <= t) - 1): a two-pointer sweep over time-ordered TOAs, a
// binary search otherwise; other ranges are tested one by one.
int64_t pint_pack_toas(const pint_toa_cols_t* c, pint_toas_t* o, int32_t* dmx_x, int64_t cap) {
    if (!c || !o || c->n <= 0 || o->n != c->n) return -PINT_E_INVALID;
    if (!c->tdb_hi || !c->tdb_lo || !c->freq_mhz || !c->pos_km || !c->vel_kms || !c->sun_km || !c->mjd ||
        !c->is_bary || !c->sigma_us || (c->ndmx > 0 && (!c->dmx_r1 || !c->dmx_r2)))
        return -PINT_E_INVALID;
    if (!o->tdb_hi || !o->tdb_lo || !o->freq_mhz || !o->sigma_s || !o->pos_km || !o->vel_kms || !o->sun_km ||
        !o->pulse_number || !o->delta_pn || !o->flags || !o->jump_mask || !o->dmx_a || !o->dmx_b)
        return -PINT_E_INVALID;
    const int n = c->n;
    const double* tz = c->tzr;
    auto col = [&](const double* src, int w, const double* tail, const double* dst_c) {
        double* dst = const_cast<double*>(dst_c);
        if (src) memcpy(dst, src, sizeof(double) * w * n);
        else memset(dst, 0, sizeof(double) * w * n);
        memcpy(dst + (size_t)w * n, tail, sizeof(double) * w);
    };
    col(c->tdb_hi, 1, tz + 0, o->tdb_hi);
    col(c->tdb_lo, 1, tz + 1, o->tdb_lo);
    col(c->freq_mhz, 1, tz + 2, o->freq_mhz);
    col(c->pos_km, 3, tz + 3, o->pos_km);
    col(c->vel_kms, 3, tz + 6, o->vel_kms);
    col(c->sun_km, 3, tz + 9, o->sun_km);
    col(c->delta_pn, 1, tz + 12, o->delta_pn);
    double* sg = const_cast<double*>(o->sigma_s);
    for (int i = 0; i < n; i++) sg[i] = c->sigma_us[i] * 1e-6;
    double* pn = const_cast<double*>(o->pulse_number);
    if (c->pulse_number) memcpy(pn, c->pulse_number, sizeof(double) * n);
    else memset(pn, 0, sizeof(double) * n);
    uint64_t* jm = const_cast<uint64_t*>(o->jump_mask);
    if (c->jump_mask) memcpy(jm, c->jump_mask, sizeof(uint64_t) * (n + 1));
    else memset(jm, 0, sizeof(uint64_t) * (n + 1));
    uint32_t* fl = const_cast<uint32_t*>(o->flags);
    auto allpos = [](const double* p) { return (uint32_t)(p[0] != 0.0 && p[1] != 0.0 && p[2] != 0.0); };
    for (int i = 0; i < n; i++) fl[i] = (uint32_t)(c->is_bary[i] != 0) | (allpos(c->pos_km + 3 * i) << 1);
    fl[n] = (uint32_t)(tz[14] != 0.0) | (allpos(tz + 3) << 1);
    o->planet_km = c->planet_km;

    int32_t* da = const_cast<int32_t*>(o->dmx_a);
    int32_t* db = const_cast<int32_t*>(o->dmx_b);
    const int m = c->ndmx > 0 ? c->ndmx : 0;
    auto tmjd = [&](int i) { return i < n ? c->mjd[i] : tz[13]; };
    std::vector<int> order(m);
    std::vector<double> s1(m), s2(m);
    bool vec = m > 0;
    for (int j = 0; j < m; j++) {
        order[j] = j;
        vec = vec && !std::isnan(c->dmx_r1[j]) && !std::isnan(c->dmx_r2[j]);
    }
    if (vec) {
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return c->dmx_r1[a] < c->dmx_r1[b]; });
        for (int k = 0; k < m; k++) {
            s1[k] = c->dmx_r1[order[k]];
            s2[k] = c->dmx_r2[order[k]];
            vec = vec && s1[k] <= s2[k] && (k == 0 || s2[k] >= s2[k - 1]);
        }
    }
    auto search = [&](double t, int& lo, int& hi) {  // lo = #(s2 < t), hi = #(s1 <= t) - 1
        lo = (int)(std::lower_bound(s2.begin(), s2.end(), t) - s2.begin());
        hi = (int)(std::upper_bound(s1.begin(), s1.end(), t) - s1.begin()) - 1;
        if (std::isnan(t)) { lo = m; hi = m - 1; }  // (numpy orders NaN last: no bin)
    };
    // the bins of TOA i in parameter order
    std::vector<int> tmp;
    auto bins_of = [&](int i, int lo, int hi) -> const std::vector<int>& {
        tmp.clear();
        if (vec) {
            for (int k = lo; k <= hi; k++) tmp.push_back(order[k]);
            std::sort(tmp.begin(), tmp.end());
        } else {
            const double t = tmjd(i);
            for (int j = 0; j < m; j++)
                if (t >= c->dmx_r1[j] && t <= c->dmx_r2[j]) tmp.push_back(j);
        }
        return tmp;
    };
    bool tord = vec;
    for (int i = 1; i < n && tord; i++) tord = c->mjd[i] >= c->mjd[i - 1];
    int64_t extra = 0;
    int lo = 0, hi = -1;
    for (int i = 0; i <= n; i++) {
        da[i] = db[i] = -1;
        if (m == 0) continue;
        if (vec) {
            if (tord && i < n) {  // a sweep: both counts only grow with t
                const double t = c->mjd[i];
                while (lo < m && s2[lo] < t) lo++;
                while (hi + 1 < m && s1[hi + 1] <= t) hi++;
            } else {
                search(tmjd(i), lo, hi);
            }
            const int cnt = hi - lo + 1;
            if (cnt == 1) {
                da[i] = order[lo];
                continue;
            }
            if (cnt == 2) {
                da[i] = std::min(order[lo], order[hi]);
                db[i] = std::max(order[lo], order[hi]);
                continue;
            }
            if (cnt <= 0) continue;
        }
        const std::vector<int>& b = bins_of(i, lo, hi);
        if (b.size() > 0) da[i] = b[0];
        if (b.size() > 1) db[i] = b[1];
        if (b.size() > 2) extra += (int64_t)b.size() - 2;
    }
    o->dmx_x = nullptr;
    if (extra == 0) return 0;
    const int64_t need = (int64_t)(n + 2) + extra;
    if (!dmx_x || need > cap) return need;
    int64_t off = n + 2;
    for (int i = 0; i <= n; i++) {
        dmx_x[i] = (int32_t)off;
        if (vec) search(tmjd(i), lo, hi);
        const std::vector<int>& b = bins_of(i, lo, hi);
        for (size_t k = 2; k < b.size(); k++) dmx_x[off++] = b[k];
    }
    dmx_x[n + 1] = (int32_t)off;
    o->dmx_x = dmx_x;
    return need;
}

int pint_add_pulsar_cols(pint_ctx* ctx, const pint_toa_cols_t* c, const pint_spec_t* spec, const double* red_freq,
                         const double* red_phi) {
    if (!ctx || !c || !spec || c->n <= 0) return -PINT_E_INVALID;
    const size_t n = (size_t)c->n;
    ctx->pk_d.resize(15 * (n + 1));  // tdb_hi, tdb_lo, freq, delta_pn, sigma, pulse_number: n+1 each; pos, vel, sun: 3(n+1)
    ctx->pk_j.resize(n + 1);
    ctx->pk_f.resize(n + 1);
    ctx->pk_i.resize(2 * (n + 1));
    double* D = ctx->pk_d.data();
    pint_toas_t t;
    memset(&t, 0, sizeof(t));
    t.n = c->n;
    t.tdb_hi = D;
    t.tdb_lo = D + (n + 1);
    t.freq_mhz = D + 2 * (n + 1);
    t.delta_pn = D + 3 * (n + 1);
    t.sigma_s = D + 4 * (n + 1);
    t.pulse_number = D + 5 * (n + 1);
    t.pos_km = D + 6 * (n + 1);
    t.vel_kms = D + 9 * (n + 1);
    t.sun_km = D + 12 * (n + 1);
    t.flags = ctx->pk_f.data();
    t.jump_mask = ctx->pk_j.data();
    t.dmx_a = ctx->pk_i.data();
    t.dmx_b = ctx->pk_i.data() + (n + 1);
    int64_t need = pint_pack_toas(c, &t, ctx->pk_x.data(), (int64_t)ctx->pk_x.size());
    if (need > (int64_t)ctx->pk_x.size()) {
        ctx->pk_x.resize((size_t)need);
        need = pint_pack_toas(c, &t, ctx->pk_x.data(), need);
    }
    if (need < 0) { ctx->err = "pint_add_pulsar_cols: missing TOA column"; return (int)need; }
    return pint_add_pulsar(ctx, &t, spec, red_freq, red_phi);
}

int pint_add_pulsar(pint_ctx* ctx, const pint_toas_t* t, const pint_spec_t* spec, const double* red_freq,
                    const double* red_phi) {
    if (!ctx || !t || !spec) return -PINT_E_INVALID;
    hipSetDevice(ctx->device);
    int n = t->n;
    if (n <= 0) { ctx->err = "pulsar has no TOAs"; return -PINT_E_INVALID; }
    if (spec->nf < 1 || spec->o_F < 0 || spec->o_PEPOCH < 0) { ctx->err = "Spindown F0/PEPOCH required"; return -PINT_E_INVALID; }
    if (spec->ncol < 1 || spec->ncol > PINT_MAX_COLS) { ctx->err = "bad column count"; return -PINT_E_INVALID; }
    int K = spec->ncol + 2 * spec->nred;
    int Kp = (K + 1 + 15) / 16 * 16;
    if (Kp > GMAXKP) { ctx->err = "design matrix too wide for k_gram (K+1 > 256)"; return -PINT_E_INVALID; }
    if (spec->njump > PINT_MAX_JUMP) { ctx->err = "too many JUMPs"; return -PINT_E_INVALID; }
    if (spec->ndmjump < 0 || spec->ndmjump > 64) { ctx->err = "too many DMJUMPs"; return -PINT_E_INVALID; }
    if (spec->binary < 0 || spec->binary > PINT_BIN_DDK) { ctx->err = "unsupported binary model"; return -PINT_E_INVALID; }
    if (spec->binary == PINT_BIN_ELL1H &&
        (spec->ell1h < 1 || spec->ell1h > 3 || (spec->ell1h == 2 && (spec->nharms < 3 || spec->nharms > 64)))) {
        ctx->err = "bad ELL1H Shapiro form";
        return -PINT_E_INVALID;
    }
    PsrHost ph;
    // every array of the pulsar staged on the host (ctx->pend), committed with the other
    // pulsars of the batch by commit_uploads
    const size_t pidx = ctx->psrs.size();
    PendArena& pa = ctx->pend;
    const size_t mark_size = pa.size, mark_fix = pa.fix.size();
    const long mark_flush = pa.flushes;
    // staged (pool chunk) or, failing that, uploaded now into its own allocation
    auto stg = [&](auto src, size_t count, auto& dst) {
        if (stage(ctx, pidx, ph.dev, src, count, dst)) return 0;
        return upload(ctx, ph, src, count, dst);
    };
    auto unstage = [&]() {  // (a rejected pulsar leaves nothing staged; what a flush already
                            // committed of it stays allocated, unreferenced, until the context ends)
        if (pa.flushes == mark_flush) {
            pa.size = mark_size;
            pa.fix.resize(mark_fix);
        } else {
            pa.size = 0;
            pa.fix.clear();
        }
        pa.cur_idx = (size_t)-1;
        pa.cur_dev = nullptr;
    };
    pa.cur_idx = pidx;
    pa.cur_dev = &ph.dev;
    ph.spec = *spec;
    ph.n = n;
    ph.K = K;
    PsrDev& d = ph.dev;
    memset(&d, 0, sizeof(d));
    int rc = 0;
    rc |= stg(t->tdb_hi, n + 1, d.tdb_hi);
    rc |= stg(t->tdb_lo, n + 1, d.tdb_lo);
    rc |= stg(t->freq_mhz, n + 1, d.freq);
    rc |= stg(t->sigma_s, n, d.sigma);
    {
        std::vector<double> is(n);
        double ls = 0.0, sw = 0.0;
        for (int i = 0; i < n; i++) {
            if (!(t->sigma_s[i] > 0.0)) { ctx->err = "TOA uncertainty must be > 0"; unstage(); return -PINT_E_INVALID; }
            is[i] = 1.0 / t->sigma_s[i];
            ls += std::log(t->sigma_s[i]);
            sw += is[i] * is[i];
        }
        d.logsig = ls;
        d.sumw = sw;
        rc |= stg(is.data(), n, d.isig);
    }
    rc |= stg(t->pos_km, 3 * (n + 1), d.pos);
    rc |= stg(t->vel_kms, 3 * (n + 1), d.vel);
    rc |= stg(t->sun_km, 3 * (n + 1), d.sun);
    if (spec->shapiro == 2) {
        if (!t->planet_km) { ctx->err = "PLANET_SHAPIRO needs the planet positions (planet_km)"; unstage(); return -PINT_E_INVALID; }
        rc |= stg(t->planet_km, (size_t)15 * (n + 1), d.planet);
    }
    rc |= stg(t->pulse_number, n, d.pn);
    rc |= stg(t->delta_pn, n + 1, d.dpn);
    rc |= stg(t->flags, n + 1, d.flags);
    rc |= stg(t->jump_mask, n + 1, d.jmask);
    rc |= stg(t->dmx_a, n + 1, d.dmx_a);
    rc |= stg(t->dmx_b, n + 1, d.dmx_b);
    if (t->dmx_x) {
        // the CSR overflow of the DMX bin ids: n+2 non-decreasing offsets starting at n+2,
        // then bin indices in [0, ndmx) (the kernels index the table with them unchecked)
        const int32_t* x = t->dmx_x;
        bool ok = x[0] == n + 2;
        for (int i = 0; ok && i <= n; i++) ok = x[i + 1] >= x[i];
        for (int k = ok ? n + 2 : 0; ok && k < x[n + 1]; k++) ok = x[k] >= 0 && x[k] < spec->ndmx;
        if (!ok) { ctx->err = "dmx_x: malformed DMX overflow CSR (offsets or bin indices)"; unstage(); return -PINT_E_INVALID; }
        rc |= stg(t->dmx_x, (size_t)x[n + 1], d.dmx_x);
    }
    rc |= stg(red_freq, (size_t)2 * spec->nred, d.red_freq);
    rc |= stg(red_phi, (size_t)2 * spec->nred, d.red_phi);
    rc |= stg((const double*)nullptr, (size_t)4 * n, d.red_cs);
    rc |= stg((const double*)nullptr, (size_t)2 * VTRIG, d.trigU);
    rc |= stg((const double*)nullptr, (size_t)2 * VTRIG, d.trigW);
    const bool trig_setup = spec->nred > 0;  // red_cs and the trig sums: flush_setup, batched
    if (trig_setup) {
        ph.f1 = red_freq[0];
        ph.f1_lo = red_freq[spec->nred];
    }
    {
        // compact fit layout: DMX columns out of M when there are enough of them and no TOA
        // lies in two free bins (bins do not overlap), ECORR checked in pint_set_ecorr
        const int ncol = spec->ncol;
        std::vector<int> colOfBin(spec->ndmx > 0 ? spec->ndmx : 1, -1);
        int ndc = 0;
        for (int c = 0; c < ncol; c++)
            if (spec->col_kind[c] == PINT_COL_DMX) {
                const int bin = spec->col_index[c];
                if (bin >= 0 && bin < spec->ndmx) colOfBin[bin] = ndc;
                ndc++;
            }
        bool ok = ndc >= 8;
        std::vector<std::vector<int>> lists(ndc);
        auto colof = [&](int bin) { return bin >= 0 && bin < spec->ndmx ? colOfBin[bin] : -1; };
        for (int i = 0; ok && i < n; i++) {
            int c = -1, nfree = 0;
            for (int bin : {t->dmx_a[i], t->dmx_b[i]})
                if (colof(bin) >= 0) { c = colof(bin); nfree++; }
            if (t->dmx_x)
                for (int k = t->dmx_x[i]; k < t->dmx_x[i + 1]; k++)
                    if (colof(t->dmx_x[k]) >= 0) { c = colof(t->dmx_x[k]); nfree++; }
            if (nfree > 1) ok = false;
            else if (c >= 0) lists[c].push_back(i);
        }
        std::vector<int32_t> cmap(K + 1), dptr(ndc + 1, 0), didx;
        int kd = 0, ad = 0;
        for (int c = 0; c < ncol; c++) cmap[c] = (spec->col_kind[c] == PINT_COL_DMX) ? -(++ad) : kd++;
        const int red0c = kd;
        for (int c = ncol; c < K; c++) cmap[c] = kd++;
        cmap[K] = kd;  // residual column
        for (int a = 0; a < ndc; a++) {
            dptr[a + 1] = dptr[a] + (int)lists[a].size();
            didx.insert(didx.end(), lists[a].begin(), lists[a].end());
        }
        std::vector<int32_t> drow(n, -1);
        bool contig = true;
        for (int a = 0; a < ndc; a++) {
            for (size_t k = 0; k < lists[a].size(); k++) {
                drow[lists[a][k]] = a;
                if (k > 0 && lists[a][k] != lists[a][k - 1] + 1) contig = false;
            }
        }
        rc |= stg(drow.data(), drow.size(), d.drow);
        ph.drow_host.assign(drow.begin(), drow.end());
        ph.dlo.assign(ndc, 0);
        ph.dhi.assign(ndc, 0);
        for (int a = 0; a < ndc; a++)
            if (!lists[a].empty()) { ph.dlo[a] = lists[a].front(); ph.dhi[a] = lists[a].back() + 1; }
        d.dcontig = (ok && contig) ? 1 : 0;
        d.dsplit = ok ? 1 : 0;
        d.ndc = ndc;
        d.Kd = kd;
        d.Kpd = (kd + 1 + 15) / 16 * 16;
        d.red0c = red0c;
        {
            std::vector<int32_t> dorig(kd > 0 ? kd : 1), xorig(ndc > 0 ? ndc : 1);
            for (int c = 0; c < K; c++) {
                if (cmap[c] >= 0) dorig[cmap[c]] = c;
                else xorig[-cmap[c] - 1] = c;
            }
            rc |= stg(dorig.data(), dorig.size(), d.dorig);
            rc |= stg(xorig.data(), xorig.size(), d.xorig);
        }
        rc |= stg(cmap.data(), cmap.size(), d.cmap);
        rc |= stg(dptr.data(), dptr.size(), d.dptr);
        rc |= stg(didx.data(), didx.size(), d.didx);
        // design-matrix column runs: same kind, consecutive indices (BIN: same kind only)
        std::vector<ColRun> runs;
        for (int c = 0; c < ncol; c++) {
            const int k = spec->col_kind[c], ix = spec->col_index[c];
            if (!runs.empty()) {
                ColRun& R = runs.back();
                if (R.kind == k && (k == PINT_COL_BIN || R.idx0 + R.cnt == ix)) { R.cnt++; continue; }
            }
            runs.push_back(ColRun{k, c, 1, ix, k == PINT_COL_DMX ? -1 : cmap[c], {0, 0, 0}});
        }
        rc |= stg(runs.data(), runs.size(), d.runs);
        d.nrun = (int)runs.size();
    }
    rc |= stg(spec, 1, d.spec);
    if (rc) {
        unstage();
        ctx->err = "pint_add_pulsar: host staging allocation failed";
        return -PINT_E_HIP;
    }
    d.n = n;
    d.K = K;
    d.Kp = Kp;
    ctx->psrs.push_back(ph);
    pa.cur_idx = (size_t)-1;
    pa.cur_dev = nullptr;
    if (trig_setup) ctx->setup_pending.push_back((int)ctx->psrs.size() - 1);
    ctx->psrs_dirty = true;  // the device descriptor array is rebuilt once, at pint_set_instances
    return (int)ctx->psrs.size() - 1;
}

int pint_fit_layout(pint_ctx* ctx, int psr, int32_t* out4) {
    if (!ctx || psr < 0 || psr >= (int)ctx->psrs.size() || !out4) return PINT_E_INVALID;
    const PsrDev& d = ctx->psrs[psr].dev;
    out4[0] = d.dsplit;
    out4[1] = d.dsplit ? d.Kd : d.K;
    out4[2] = d.dsplit ? d.ndc : 0;
    out4[3] = d.dsplit ? d.Kpd : d.Kp;
    return PINT_OK;
}

int pint_vgram_layout(pint_ctx* ctx, int psr, int32_t* out4) {
    if (!ctx || psr < 0 || psr >= (int)ctx->psrs.size() || !out4) return PINT_E_INVALID;
    const PsrDev& d = ctx->psrs[psr].dev;
    out4[0] = d.vg + 2 * d.vb;  // bit 1: the binned DMX x Fourier tile (PINT_OPT_VBIN)
    out4[1] = d.vns;
    out4[2] = d.vkp;
    out4[3] = d.red0c;
    return PINT_OK;
}

int pint_set_ecorr(pint_ctx* ctx, int psr, int nep, const int32_t* ep_ptr, const int32_t* ep_idx,
                   const double* ep_phi) {
    if (!ctx || psr < 0 || psr >= (int)ctx->psrs.size() || nep < 0) return PINT_E_INVALID;
    hipSetDevice(ctx->device);
    if (int rc_ = commit_uploads(ctx)) return rc_;  // (staged pulsar uploads first)
    PsrHost& ph = ctx->psrs[psr];
    if (nep == 0) { ph.dev.nep = 0; return refresh_psrs(ctx) ? PINT_E_HIP : PINT_OK; }
    if (!ep_ptr || !ep_idx || !ep_phi || ep_ptr[0] != 0) { ctx->err = "bad ECORR epoch lists"; return PINT_E_INVALID; }
    for (int e = 0; e < nep; e++) {
        if (ep_ptr[e + 1] < ep_ptr[e] || !(ep_phi[e] > 0.0)) { ctx->err = "bad ECORR epoch"; return PINT_E_INVALID; }
    }
    for (int k = 0; k < ep_ptr[nep]; k++) {
        if (ep_idx[k] < 0 || ep_idx[k] >= ph.n) { ctx->err = "ECORR TOA index out of range"; return PINT_E_INVALID; }
    }
    int rc = 0;
    rc |= upload(ctx, ph, ep_ptr, (size_t)nep + 1, ph.dev.ep_ptr);
    rc |= upload(ctx, ph, ep_idx, (size_t)ep_ptr[nep], ph.dev.ep_idx);
    rc |= upload(ctx, ph, ep_phi, (size_t)nep, ph.dev.ep_phi);
    {
        std::vector<int32_t> te(ph.n, -1);
        int overlap = 0;
        for (int e = 0; e < nep; e++)
            for (int k = ep_ptr[e]; k < ep_ptr[e + 1]; k++) {
                overlap |= te[ep_idx[k]] >= 0;
                te[ep_idx[k]] = e;
            }
        ph.dev.ep_overlap = overlap;
        rc |= upload(ctx, ph, te.data(), (size_t)ph.n, ph.dev.toa_ep);
    }
    if (rc) return PINT_E_HIP;
    ph.dev.nep = nep;
    if (ph.dev.dsplit) {
        // the compact layout stays when no TOA is in two epochs and each epoch's TOAs lie in at
        // most one DMX column (the epoch-by-DMX block then has one entry per epoch); otherwise
        // the Schur rows couple DMX columns: the full layout
        const int ndc = ph.dev.ndc;
        std::vector<int32_t> eb(nep, -1), bptr(ndc + 1, 0), bidx;
        bool ok = !ph.dev.ep_overlap;
        for (int e = 0; ok && e < nep; e++)
            for (int k = ep_ptr[e]; k < ep_ptr[e + 1]; k++) {
                const int a = ph.drow_host[ep_idx[k]];
                if (a < 0) continue;
                if (eb[e] >= 0 && eb[e] != a) { ok = false; break; }
                eb[e] = a;
            }
        if (ok) {
            std::vector<std::vector<int32_t>> lists(ndc);
            for (int e = 0; e < nep; e++)
                if (eb[e] >= 0) lists[eb[e]].push_back(e);
            for (int a = 0; a < ndc; a++) {
                bptr[a + 1] = bptr[a] + (int)lists[a].size();
                bidx.insert(bidx.end(), lists[a].begin(), lists[a].end());
            }
            rc |= upload(ctx, ph, eb.data(), eb.size(), ph.dev.ep_bin);
            rc |= upload(ctx, ph, bptr.data(), bptr.size(), ph.dev.bep_ptr);
            rc |= upload(ctx, ph, bidx.data(), bidx.size(), ph.dev.bep_idx);
            if (rc) return PINT_E_HIP;
        } else {
            ph.dev.dsplit = 0;
        }
    }
    return refresh_psrs(ctx) ? PINT_E_HIP : PINT_OK;
}

int pint_set_instances(pint_ctx* ctx, int ninst, const int32_t* inst_psr, const double* tables) {
    if (!ctx || ninst <= 0 || !tables) return PINT_E_INVALID;
    return set_instances_impl(ctx, ninst, inst_psr, tables);
}

// A grid of npts points of one pulsar (gridutils.grid_chisq and friends): every point's table
// is the base table with nvar entries replaced, formed on the device (k_grid_tables) from the
// base table and the grid axes instead of npts host-built tables: variable j of point k takes
// the value (hi, lo) = vals_j[((k0 + k) / stride[j]) % size[j]] (vals: the variables' value
// pairs concatenated, size[j] pairs each) -- a meshgrid's axes, or every point's own value
// (stride 1, size npts).
static int flush_chi2(pint_ctx* ctx);
int pint_set_grid(pint_ctx* ctx, int psr, int npts, const double* base, int nvar, const int32_t* var_toff,
                  const int64_t* var_stride, const int64_t* var_size, const double* vals, int64_t k0) {
    if (!ctx || npts <= 0 || !base || nvar < 0 || nvar > 16 || (nvar && (!var_toff || !var_stride || !var_size || !vals)))
        return PINT_E_INVALID;
    if (psr < 0 || psr >= (int)ctx->psrs.size()) { ctx->err = "bad pulsar id"; return PINT_E_INVALID; }
    const int ts = ctx->psrs[psr].spec.tstride;
    long nv = 0;
    for (int j = 0; j < nvar; j++) {
        if (var_toff[j] < 0 || var_toff[j] + 1 >= ts || var_stride[j] < 1 || var_size[j] < 1) {
            ctx->err = "pint_set_grid: bad grid variable (table offset, stride or size)";
            return PINT_E_INVALID;
        }
        nv += var_size[j];
    }
    // the same pulsar and point count as the resident batch (the next grid over the same
    // TOAs, or the next chunk of one): every instance array, launch group and buffer is the
    // same, only the tables differ -- reset the batch's state as a fresh batch has it and
    // form the new tables, instead of ~3 ms of host set-up and InstDev uploads at 65,536 points
    const long gkey = ((long)ctx->small << 2) | ((long)ctx->vgram << 1) | (long)ctx->vbin;
    if (ctx->grid_valid && ctx->grid_psr == psr && ctx->ninst == npts && ctx->grid_opts == gkey && !ctx->psrs_dirty &&
        ctx->setup_pending.empty()) {
        if (flush_chi2(ctx)) return PINT_E_HIP;  // (a lazy pint_chi2_gls of the previous points is delivered)
        if (int rc = flush_cq_now(ctx)) return rc;
        HIPCHK(hipStreamSynchronize(ctx->cstream));
        HIPCHK(hipStreamSynchronize(ctx->sstream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        clear_copy_pend(ctx);
        dfree((void*&)ctx->d_tables0);  // (a snapshot of the previous points)
        ctx->tables0_cap = 0;
        ctx->ic_valid = ctx->ic0_valid = false;
        ctx->restore_pending = ctx->chi2_pending = ctx->cov_pending = false;
        ctx->wtile_valid = false;
        ctx->chi2_dst = nullptr;
        for (int k = 0; k < pint_ctx::NSLOT; k++) {
            if (ctx->graph_exec_s[k]) hipGraphExecDestroy(ctx->graph_exec_s[k]);
            if (ctx->graph_s[k]) hipGraphDestroy(ctx->graph_s[k]);
            ctx->graph_exec_s[k] = nullptr;
            ctx->graph_s[k] = nullptr;
        }
        HIPCHK(hipMemsetAsync(ctx->d_istatus, 0, sizeof(int) * ctx->ninst, ctx->stream));
        HIPCHK(hipMemsetAsync(ctx->d_cov, 0, sizeof(double) * std::max<long>(1, ctx->tot_cv), ctx->stream));
    } else {
        std::vector<int32_t> ip(npts, psr);
        if (int rc = set_instances_impl(ctx, npts, ip.data(), nullptr)) return rc;
        ctx->grid_valid = true;
        ctx->grid_psr = psr;
        ctx->grid_opts = gkey;
    }
    // the spec: base table, then per variable (toff, stride, size, value offset) as doubles
    // (exact: all < 2^53), then the value pairs
    // (the spec stays in the context until the next pint_set_grid, which synchronises the
    // streams before it is rewritten: no wait here for its upload)
    std::vector<double>& spec = ctx->grid_spec_host;
    spec.assign((size_t)ts + 4 * nvar + 2 * nv, 0.0);
    for (int i = 0; i < ts; i++) spec[i] = base[i];
    long vo = 0;
    for (int j = 0; j < nvar; j++) {
        double* h = spec.data() + ts + 4 * j;
        h[0] = var_toff[j];
        h[1] = (double)var_stride[j];
        h[2] = (double)var_size[j];
        h[3] = (double)vo;
        vo += var_size[j];
    }
    for (long i = 0; i < 2 * nv; i++) spec[ts + 4 * nvar + i] = vals[i];
    dfree((void*&)ctx->d_gridspec);  // (the previous grid's: its tables were formed, the streams synchronised)
    HIPCHK(cmalloc((void**)&ctx->d_gridspec, sizeof(double) * spec.size()));
    HIPCHK(h2d(ctx->d_gridspec, spec.data(), sizeof(double) * spec.size(), ctx->stream, false));
    const long total = (long)npts * ts;
    const int nb = (int)std::min<long>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(k_grid_tables, dim3(nb), dim3(256), 0, ctx->stream, ctx->d_gridspec, ts, nvar, npts, (long)k0,
                       ctx->d_tables);
    HIPCHK(hipGetLastError());
    // points that differ in spin frequencies only share the evaluation's head (k_eval_head)
    {
        const PsrHost& ph = ctx->psrs[psr];
        const pint_spec_t& sp = ph.spec;
        bool spin = nvar > 0 && sp.binary == 0 && sp.nred == 0 && !ph.dev.dsplit && !ctx->efz;
        for (int j = 0; j < nvar; j++) spin = spin && var_toff[j] >= sp.o_F && var_toff[j] < sp.o_F + 2 * sp.nf;
        ctx->spin_grid = spin;
        if (spin && (long)(ph.n + 1) * EVAL_HEAD_W > ctx->shr_cap) {
            dfree((void*&)ctx->d_shr);
            ctx->shr_cap = (long)(ph.n + 1) * EVAL_HEAD_W;
            HIPCHK(cmalloc((void**)&ctx->d_shr, sizeof(double) * ctx->shr_cap));
        }
        ctx->tables_fresh = true;
    }
    if (!ctx->lazy) HIPCHK(hipStreamSynchronize(ctx->stream));
    return PINT_OK;
}

static int set_instances_impl(pint_ctx* ctx, int ninst, const int32_t* inst_psr, const double* tables) {
    if (!ctx || ninst <= 0) return PINT_E_INVALID;
    ctx->grid_valid = false;  // (pint_set_grid marks its own batch afterwards)
    ctx->tables_fresh = false;
    ctx->r2_pending = false;
    hipSetDevice(ctx->device);
    if (ctx->psrs_dirty && refresh_psrs(ctx)) return PINT_E_HIP;
    if (flush_setup(ctx)) return PINT_E_HIP;  // the uploads' red-noise set-up, one batch
    if (int rc = flush_cq_now(ctx)) return rc;  // (their buffers are freed below, after the streams drain)
    free_instances(ctx);
    ctx->inst.resize(ninst);
    long toff = 0, roff = 0, moff = 0, goff = 0, soff = 0, coff = 0, out = 0, cvoff = 0, eoff = 0, epoff = 0;
    long sdoff = 0, ddoff = 0;
    int max_nep = 0, max_ndc = 0;
    std::vector<int> bti[PINT_NBIN], btr[PINT_NBIN];
    std::vector<int> rbi;
    int maxK = 0, maxN = 0;
    for (int k = 0; k < ninst; k++) {
        int p = inst_psr[k];
        if (p < 0 || p >= (int)ctx->psrs.size()) { ctx->err = "bad pulsar id"; return PINT_E_INVALID; }
        if (ctx->psrs[p].n > maxN) maxN = ctx->psrs[p].n;
    }
    // the fused residual pass for batches off the small-instance path (whose one-wave
    // residual kernels serve instances of <= RES_SMALLN rows)
    ctx->efz = ctx->efuse && !(ctx->small && maxN <= RES_SMALLN);
    long ebn = 0;
    // N-split for the Gram so the launch fills the 256 CUs
    // choose the split count that minimises (workgroup rounds) / nsplit, i.e. the k_gram
    // makespan with one 1024-thread workgroup resident per CU, with >= 4 chunks per split
    int ncu = 256;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, ctx->device) == hipSuccess && prop.multiProcessorCount > 0)
            ncu = prop.multiProcessorCount;
    }
    int maxsplit = (maxN + 4 * GCH - 1) / (4 * GCH);
    if (maxsplit < 1) maxsplit = 1;
    // Resident Gram workgroups per CU: k_gram runs one per CU, k_gram_v GWG; the batch's
    // majority path decides
    long nvgc = 0;
    for (int k = 0; k < ninst; k++) {
        const PsrHost& ph = ctx->psrs[inst_psr[k]];
        const PsrDev& d = ph.dev;
        nvgc += (ctx->vgram && d.dsplit && d.dcontig && d.nep == 0 && ph.spec.nred <= VTRIG / 2 - 1 &&
                 d.red0c + 1 <= VMAXR0) ? 1 : 0;
    }
    const long slots = (long)ncu * (2 * nvgc > ninst ? GWG : 1);
    // A batch too small to fill the chip even at the finest split (a single fit, a few
    // pulsars) is latency-bound: splits of 128 rows leave each workgroup two chunks while
    // k_greduce sums hundreds of partials per Gram element.  Keep >= 512 rows per split there.
    if ((long)ninst * maxsplit < slots) maxsplit = std::max(1, std::min(maxsplit, (maxN + 511) / 512));
    // (smallest split count within 3% of the best makespan: each split adds a partial
    // Gram that k_greduce must sum)
    double best = 1e30;
    for (int ns = 1; ns <= maxsplit && ns <= 4096; ns++) {
        long blocks = (long)ninst * ns;
        double cost = (double)((blocks + slots - 1) / slots) / ns;
        if (cost < best) best = cost;
    }
    int nsplit = 1;
    for (int ns = 1; ns <= maxsplit && ns <= 4096; ns++) {
        long blocks = (long)ninst * ns;
        double cost = (double)((blocks + slots - 1) / slots) / ns;
        if (cost <= best * 1.03) { nsplit = ns; break; }
    }
    // (measured on the 68-pulsar PTA, round 4: 7 splits -- one round of workgroups, many CUs
    // with one -- 0.120 ms of k_gram_v, 8: 0.147, 11: 0.104, this model's 15: 0.089-0.093)
    if (const char* e = getenv("PINT_NSPLIT")) {  // (diagnostic sweeps: a fixed split count)
        const int v = atoi(e);
        if (v >= 1) nsplit = std::min(v, std::max(1, (maxN + 63) / 64));
    }
    ctx->nsplit = nsplit;
    ctx->red_valid[0] = ctx->red_valid[1] = 0;
    ctx->ic_valid = false;
    // vg compact path (k_gram_v): contiguous DMX bins, no ECORR, nred <= 31, <= 47
    // timing columns; the DMX slots fill the [T | r] row tiles (+16 if needed) such that the
    // bins of every N-split are distinct mod vns; LDS width <= VMAXKP
    auto vg_ok = [&](const PsrHost& ph) {
        const PsrDev& d = ph.dev;
        return ctx->vgram && d.dsplit && d.dcontig && d.nep == 0 && ph.spec.nred <= VTRIG / 2 - 1 &&
               ph.spec.dmn0 >= ph.spec.nred &&  // PLDMNoise: stored, per-TOA scaled basis
               d.red0c + 1 <= VMAXR0;
    };
    auto slots_ok = [&](const PsrHost& ph, int ntr) {  // bins of every split distinct mod ns
        const PsrDev& d = ph.dev;
        const int wt = d.red0c + 1, R = d.Kd - d.red0c;
        const int ns = 16 * ntr - wt, kpv = (16 * ntr + R + 15) / 16 * 16;
        if (ns < 1 || kpv > VMAXKP) return false;
        long per = (ph.n + nsplit - 1) / nsplit;
        per = (per + 3) / 4 * 4;
        for (int sp = 0; sp < nsplit; sp++) {
            const long i0 = sp * per, i1 = std::min<long>(i0 + per, ph.n);
            std::vector<char> seen(ns, 0);
            for (int a = 0; a < d.ndc; a++) {
                if (ph.dhi[a] <= ph.dlo[a] || ph.dlo[a] >= i1 || ph.dhi[a] <= i0) continue;
                if (seen[a % ns]) return false;
                seen[a % ns] = 1;
            }
        }
        return true;
    };
    // A batch whose Gram workgroups fit one resident round (a few pulsars: the per-rank shard
    // of a PTA over several GPUs) is latency-bound, and every distinct k_gram_v tile shape is
    // a launch of its own, in sequence: there all vg pulsars take the largest row-tile count
    // any of them needs (more padding MFMAs, one launch)
    int force_ntr = 0;
    if ((long)ninst * nsplit <= slots) {
        std::vector<char> inb(ctx->psrs.size(), 0);
        for (int k = 0; k < ninst; k++) inb[inst_psr[k]] = 1;
        for (size_t p = 0; p < ctx->psrs.size(); p++) {
            const PsrHost& ph = ctx->psrs[p];
            if (!inb[p] || !vg_ok(ph)) continue;
            const int wt = ph.dev.red0c + 1;
            for (int ntr = (wt + 15) / 16; ntr <= std::min(3, (wt + 15) / 16 + 2); ntr++)
                if (slots_ok(ph, ntr)) { force_ntr = std::max(force_ntr, ntr); break; }
        }
    }
    // the rows' DMX slot ids of every pulsar whose slot count changed, staged into one
    // allocation and one copy after the loop (a PTA: 68 uploads of 40 KB each, ~0.1 ms apiece)
    std::vector<std::pair<size_t, size_t>> slot_up;  // (pulsar, offset in slot_host)
    std::vector<int32_t> slot_host;
    for (size_t pi = 0; pi < ctx->psrs.size(); pi++) {
        PsrHost& ph = ctx->psrs[pi];
        PsrDev& d = ph.dev;
        d.vg = 0;
        d.vb = 0;
        if (!vg_ok(ph)) continue;
        long per = (ph.n + nsplit - 1) / nsplit;
        per = (per + 3) / 4 * 4;
        const int wt = d.red0c + 1, R = d.Kd - d.red0c;
        const int ntr0 = std::max((wt + 15) / 16, std::min(3, force_ntr));
        for (int ntr = ntr0; ntr <= std::min(3, (wt + 15) / 16 + 2); ntr++) {
            const int ns = 16 * ntr - wt, kpv = (16 * ntr + R + 15) / 16 * 16;
            if (!slots_ok(ph, ntr)) continue;
            {
                d.vg = 1;
                d.vns = ns;
                d.vkp = kpv;
                if (ph.dslot_ns != ns) {  // the rows' slots, so k_gram_v does no modulo
                    const size_t o = (slot_host.size() + 63) & ~(size_t)63;
                    slot_host.resize(o + ph.n);
                    for (int i = 0; i < ph.n; i++) slot_host[o + i] = ph.drow_host[i] >= 0 ? ph.drow_host[i] % ns : -1;
                    slot_up.push_back({pi, o});
                    ph.dslot_ns = ns;
                }
                break;
            }
        }
        d.vb = 0;
        // VB only with an all-slot row tile to drop (the [T | r] columns leave >= 16 slots)
        if (d.vg && ctx->vbin && d.vkp <= 96 && d.vns >= 16) {
            // VB (binned DMX x F): the 16 rows a wave takes from one chunk (split sp, quarter w,
            // rows i0 + w QV + 16 c ..) hold at most two bins, of distinct parity (drow)
            // (a pulsar that fails it leaves the vg path: with an all-slot row tile k_gram_v
            // takes the binned body, so vg without VB is not a layout the kernel knows)
            const std::vector<int>& dr = ph.drow_host;
            for (int sp = 0; d.vg && sp < nsplit; sp++) {
                const long i0 = std::min<long>((long)sp * per, ph.n), i1 = std::min<long>(i0 + per, ph.n);
                const long QV = (i1 - i0 + VCH - 1) / VCH * 16;
                for (long g = 0; d.vg && g < i1 - i0; g += 16) {  // g = w QV + 16 c
                    const long gend = std::min<long>(g + 16, (g / QV + 1) * QV);
                    int b0 = -1, b1 = -1;
                    for (long r = g; r < gend && r < i1 - i0; r++) {
                        const int b = dr[i0 + r];
                        if (b < 0 || b == b0 || b == b1) continue;
                        if (b0 < 0) b0 = b;
                        else if (b1 < 0 && ((b ^ b0) & 1)) b1 = b;
                        else d.vg = 0;
                    }
                }
            }
            d.vb = d.vg;
        }
    }
    if (!slot_up.empty()) {
        void* p = nullptr;
        HIPCHK(hipMalloc(&p, sizeof(int32_t) * slot_host.size()));
        HIPCHK(h2d(p, slot_host.data(), sizeof(int32_t) * slot_host.size(), nullptr, true));
        ctx->psrs[slot_up[0].first].bufs.push_back(p);  // (freed with the first pulsar's buffers)
        for (auto& u : slot_up) ctx->psrs[u.first].dev.dslot = static_cast<const int32_t*>(p) + u.second;
    }
    if (refresh_psrs(ctx)) return PINT_E_HIP;
    long vgoff = 0, vboff = 0, xwoff = 0;
    ctx->n_vg = 0;
    ctx->cov_pending = false;
    ctx->vb_on = ctx->vbin;
    ctx->any_dmx_rows = false;
    for (int k = 0; k < ninst; k++) {
        int p = inst_psr[k];
        PsrHost& ph = ctx->psrs[p];
        InstDev& I = ctx->inst[k];
        I.psr = p;
        I.n = ph.n;
        I.spec = ph.dev.spec;
        I.runs = ph.dev.runs;
        I.ts = ph.spec.tstride;
        I.nrun = ph.dev.nrun;
        I.K = ph.K;
        I.Kp = ph.dev.Kp;
        I.toff = toff;
        I.roff = roff;
        I.moff = moff;
        I.goff = goff;
        I.soff = soff;
        I.coff = coff;
        I.cvoff = cvoff;
        I.eoff = eoff;
        I.epoff = epoff;
        I.ooff = out;
        I.sdoff = sdoff;
        I.ddoff = ddoff;
        I.vgoff = vgoff;
        I.vboff = vboff;
        I.xwoff = xwoff;
        if (ph.dev.vg) {
            vgoff += (long)nsplit * ph.dev.vns * (ph.dev.Kd + 3);
            if (ph.dev.vb) vboff += (long)nsplit * GW * ph.dev.vns * 128;
            ctx->n_vg++;
        } else if (ph.dev.dsplit) {
            ctx->any_dmx_rows = true;
        }
        if (ph.dev.dsplit) {
            sdoff += (long)ph.dev.ndc * ph.dev.Kpd;
            ddoff += ph.dev.ndc;
            const long nbd = (ph.dev.Kd + 15) / 16, nbk = (ph.dev.ndc + 15) / 16;
            xwoff += (nbd * (nbd + 1) / 2 + nbd * nbk) * 256 + (nbd + 3 * nbk) * 16 + schur_xw_extra(nbd, nbk);
            if (ph.dev.ndc > max_ndc) max_ndc = ph.dev.ndc;
        }
        I.self = k;
        I.rb0 = (long)rbi.size();
        I.nrb = std::max(1, (ph.n + RES_RB - 1) / RES_RB);
        for (int b = 0; b < I.nrb; b++) rbi.push_back(k);
        eoff += (long)ph.dev.nep * I.Kp;
        epoff += ph.dev.nep;
        if (ph.dev.nep > max_nep) max_nep = ph.dev.nep;
        cvoff += (long)ph.spec.ncol * ph.spec.ncol;
        toff += ph.spec.tstride;
        int bt = ph.spec.binary;
        if (bt < 0 || bt >= PINT_NBIN) { ctx->err = "bad binary model"; return PINT_E_INVALID; }
        if (ctx->efz) {  // EF_ROWS rows per block (+ row 0 and the TZR row on its last lanes)
            I.eb0 = ebn;
            I.neb = std::max(1, (ph.n + EF_ROWS - 1) / EF_ROWS);
            ebn += I.neb;
            for (int r0 = 0; r0 < std::max(1, ph.n); r0 += EF_ROWS) {
                bti[bt].push_back(k);
                btr[bt].push_back(r0);
            }
        } else {
            I.eb0 = 0;
            I.neb = 0;
            for (int r0 = 0; r0 <= ph.n; r0 += 256) {
                bti[bt].push_back(k);
                btr[bt].push_back(r0);
            }
        }
        roff += ph.n + 1;
        moff += (long)ph.n * ph.K;
        goff += (long)(nsplit + 1) * I.Kp * I.Kp;  // + ECORR Schur partial
        soff += (long)(ph.K + 1) * (ph.K + 1);
        coff += ph.K + 1;
        out += ph.n;
        if (ph.K > maxK) maxK = ph.K;
    }
    ctx->ninst = ninst;
    ctx->tot_table = toff;
    ctx->tot_rows = roff;
    ctx->tot_m = moff;
    ctx->tot_g = goff;
    ctx->tot_s = soff;
    ctx->tot_c = coff;
    ctx->tot_out = out;
    ctx->tot_cv = cvoff;
    ctx->maxK = maxK;
    ctx->maxn = 0;
    ctx->max_ts = 0;
    for (const InstDev& I : ctx->inst) {
        ctx->maxn = std::max(ctx->maxn, I.n);
        ctx->max_ts = std::max(ctx->max_ts, ctx->psrs[I.psr].spec.tstride);
    }
    {
        std::vector<char> seen(ctx->psrs.size(), 0);
        ctx->upsr.clear();
        for (int k = 0; k < ninst; k++)
            if (!seen[inst_psr[k]]) {
                seen[inst_psr[k]] = 1;
                ctx->upsr.push_back(inst_psr[k]);
            }
    }
    ctx->tot_e = eoff;
    ctx->tot_ep = epoff;
    ctx->max_nep = max_nep;
    ctx->max_ndc = max_ndc;
    std::vector<int> bi, br;
    for (int t = 0; t < PINT_NBIN; t++) {
        ctx->blk_off[t] = (int)bi.size();
        bi.insert(bi.end(), bti[t].begin(), bti[t].end());
        br.insert(br.end(), btr[t].begin(), btr[t].end());
    }
    ctx->blk_off[PINT_NBIN] = (int)bi.size();
    ctx->nblk = ctx->blk_off[3];  // k_eval_mix covers the isolated, ELL1 and DD blocks
    HIPCHK(cmalloc((void**)&ctx->d_inst, sizeof(InstDev) * ninst));
    HIPCHK(h2d(ctx->d_inst, ctx->inst.data(), sizeof(InstDev) * ninst, nullptr, true));
    for (int lay = 0; lay < 3; lay++) {  // k_gram launch groups: full, compact, compact + vg
        std::vector<InstDev> sorted;
        std::vector<KpGroup>& groups = lay == 0 ? ctx->kp_groups : (lay == 1 ? ctx->kp_groups_c : ctx->kp_groups_v);
        groups.clear();
        // bucket the instances by launch key in one pass (a grid batch has ~10^5 instances)
        const int maxT = lay == 2 ? 29 : GMAXT_ALL;
        std::vector<std::vector<int>> bucket(maxT + 1);
        std::vector<int> bkp(maxT + 1, 16);
        for (int k = 0; k < ninst; k++) {
            const InstDev& I = ctx->inst[k];
            const PsrDev& pd = ctx->psrs[I.psr].dev;
            if (lay == 1 && pd.dsplit && pd.vg) continue;
            if (lay == 2 && !(pd.dsplit && pd.vg)) continue;
            const int kp = lay == 2 ? pd.vkp : ((lay && pd.dsplit) ? pd.Kpd : I.Kp);
            const int nt = kp / 16;
            int tT = (nt * (nt + 1) / 2 + GWAVES - 1) / GWAVES;
            if (lay == 2) {  // k_gram_v template key: row tiles (1..3) x column tiles (ntr..7)
                const int ntr = (pd.red0c + 1 + pd.vns) / 16;
                tT = 10 * (ntr - 1) + nt;
            }
            if (lay < 2 && ctx->small && kp <= 32 && I.n <= GS_MAXN) tT = 0;  // k_gram_s
            if (tT < (lay < 2 ? 0 : 1) || tT > maxT) continue;
            bucket[tT].push_back(k);
            if (kp > bkp[tT]) bkp[tT] = kp;
        }
        if (lay == 2) {
            // heaviest first within a launch (MFMAs per k-step x rows): the light blocks fill
            // the tail of the second resident round
            auto cost = [&](int k) {
                const PsrDev& pd = ctx->psrs[ctx->inst[k].psr].dev;
                const int ntr = (pd.red0c + 1 + pd.vns) / 16, ntc = pd.vkp / 16;
                const int nsk = ntr - (pd.red0c + 1 + 15) / 16;
                int t = pd.vb ? 1 : 0;
                for (int ti = 0; ti < ntr; ti++)
                    for (int tj = ti; tj < ntc; tj++)
                        if (!(ti >= ntr - nsk && (tj < ntr || pd.vb))) t++;
                // MFMA tiles per k-step, and the timing columns loaded and staged (measured on
                // the bench PTA: ~4 columns cost one tile)
                return (long)(4 * t + pd.red0c + 1) * ctx->inst[k].n;
            };
            std::vector<long> ck(ninst, 0);
            for (auto& b : bucket) {
                for (int k : b) ck[k] = cost(k);
                std::stable_sort(b.begin(), b.end(), [&](int x, int y) { return ck[x] > ck[y]; });
                // two k_gram_v workgroups share a CU, and the dispatcher gives workgroup w and
                // w + ncu (roughly) the same CU in the first resident round: pair the heaviest
                // instances (first ncu workgroups) with the lightest (next ncu), then the rest
                // heaviest first (PINT_GV_PAIR=0: plain heaviest-first order)
                const int k1 = ncu / std::max(1, nsplit);
                const bool uniform = b.empty() || ck[b.front()] == ck[b.back()];  // (nothing to pair)
                if (ctx->gv_pair && !uniform && k1 > 0 && (int)b.size() > 2 * k1) {
                    std::vector<int> o(b.begin(), b.begin() + k1);
                    o.insert(o.end(), b.rbegin(), b.rbegin() + k1);
                    o.insert(o.end(), b.begin() + k1, b.end() - k1);
                    b.swap(o);
                }
            }
        }
        bool ident = true;  // the launch order is the instance order (e.g. a grid's points)
        int nxt = 0;
        for (int T = 0; T <= maxT; T++) {
            if (bucket[T].empty()) continue;
            KpGroup g{T, (int)sorted.size(), (int)bucket[T].size(), bkp[T]};
            for (int k : bucket[T]) {
                ident = ident && k == nxt++;
                sorted.push_back(ctx->inst[k]);
            }
            groups.push_back(g);
        }
        InstDev*& dst = lay == 0 ? ctx->d_inst_sorted : (lay == 1 ? ctx->d_inst_sorted_c : ctx->d_inst_sorted_v);
        if (ident && (int)sorted.size() == ninst) {
            // one upload of the instance array serves this launch order too (a 65,536-point
            // grid batch moved ~10 MB of InstDev per order from pageable memory, ~1 ms each)
            dst = ctx->d_inst;
            ctx->sorted_alias[lay] = true;
            continue;
        }
        HIPCHK(cmalloc((void**)&dst, sizeof(InstDev) * std::max<size_t>(1, sorted.size())));
        if (!sorted.empty())
            HIPCHK(h2d(dst, sorted.data(), sizeof(InstDev) * sorted.size(), nullptr, true));
    }
    if (getenv("PINT_VERBOSE")) {
        for (auto& g : ctx->kp_groups_v) fprintf(stderr, "[pint] k_gram_v group key %d: %d instances, max width %d\n", g.T, g.count, g.maxKp);
        for (size_t k = 0; k < ctx->psrs.size() && k < 4; k++) {
            const PsrDev& d = ctx->psrs[k].dev;
            fprintf(stderr, "[pint] psr %zu: vg %d r0 %d Kd %d ns %d kpv %d ndc %d nsplit %d\n", k, d.vg, d.red0c, d.Kd, d.vns, d.vkp, d.ndc, nsplit);
        }
    }
    HIPCHK(cmalloc((void**)&ctx->d_Sdp, sizeof(double) * std::max<long>(1, vgoff)));
    HIPCHK(cmalloc((void**)&ctx->d_BFp, sizeof(double) * std::max<long>(1, vboff)));
    if (xwoff > 0 && xwoff <= (1L << 28)) {
        for (int sl = 0; sl < pint_ctx::NSLOT; sl++) HIPCHK(cmalloc((void**)&ctx->d_xw_s[sl], sizeof(double) * xwoff));
    }
    HIPCHK(cmalloc((void**)&ctx->d_TSp, sizeof(double) * std::max<long>(1, (long)ninst * nsplit * 4 * VTRIG)));
    HIPCHK(cmalloc((void**)&ctx->d_TS, sizeof(double) * std::max<long>(1, (long)ninst * 4 * VTRIG)));
    HIPCHK(cmalloc((void**)&ctx->d_blk_inst, sizeof(int) * bi.size()));
    HIPCHK(cmalloc((void**)&ctx->d_blk_row0, sizeof(int) * br.size()));
    HIPCHK(h2d(ctx->d_blk_inst, bi.data(), sizeof(int) * bi.size(), nullptr, true));
    HIPCHK(h2d(ctx->d_blk_row0, br.data(), sizeof(int) * br.size(), nullptr, true));
    ctx->nrblk = (int)rbi.size();
    HIPCHK(cmalloc((void**)&ctx->d_rblk_inst, sizeof(int) * std::max<size_t>(1, rbi.size())));
    if (!rbi.empty())
        HIPCHK(h2d(ctx->d_rblk_inst, rbi.data(), sizeof(int) * rbi.size(), nullptr, true));
    HIPCHK(cmalloc((void**)&ctx->d_rpart, sizeof(double) * 3 * std::max<size_t>(1, rbi.size())));
    HIPCHK(cmalloc((void**)&ctx->d_epart, sizeof(double) * 2 * std::max<long>(1, ebn)));
    // the post-fit Woodbury dots fused into the residual pass (k_resid2 tiles, k_rsum): every
    // instance's noise basis a PLRedNoise harmonic series of < 64 modes (no PLDMNoise)
    {
        bool fuse = true;
        int R = 0;
        for (int k = 0; k < ninst; k++) {
            const pint_spec_t& sp = ctx->psrs[inst_psr[k]].spec;
            R = std::max(R, 2 * sp.nred);
            if (sp.dmn0 < sp.nred || sp.nred > 63) fuse = false;
        }
        // (R = 0: no tile to form -- a WLS batch's post-fit pass would write 2 KB of zeros per
        // residual block; 1^T W r then comes from k_wdot if a GLS chi2 is asked for)
        ctx->wfuse = fuse && R > 0 && !rbi.empty();
        ctx->wtile_valid = false;
        if (ctx->wfuse) {
            HIPCHK(cmalloc((void**)&ctx->d_wtile, sizeof(double) * 256 * rbi.size()));
            const size_t need = (size_t)ninst * (R + 2);
            if (need > ctx->wpart_cap) {
                dfree((void*&)ctx->d_wpart);
                HIPCHK(cmalloc((void**)&ctx->d_wpart, sizeof(double) * need));
                ctx->wpart_cap = need;
            }
            ctx->wstride = R + 2;
        }
    }

    HIPCHK(cmalloc((void**)&ctx->d_tables, sizeof(double) * toff));
    if (tables) HIPCHK(h2d(ctx->d_tables, tables, sizeof(double) * toff, nullptr, true));
    HIPCHK(cmalloc((void**)&ctx->d_phhi, sizeof(double) * roff));
    HIPCHK(cmalloc((void**)&ctx->d_phlo, sizeof(double) * roff));
    HIPCHK(cmalloc((void**)&ctx->d_ftay, sizeof(double) * roff));
    HIPCHK(cmalloc((void**)&ctx->d_delay, sizeof(double) * roff));
    HIPCHK(cmalloc((void**)&ctx->d_M, sizeof(double) * (moff > 0 ? moff : 1)));
    HIPCHK(cmalloc((void**)&ctx->d_rt, sizeof(double) * out));
    HIPCHK(cmalloc((void**)&ctx->d_rp, sizeof(double) * out));
    HIPCHK(cmalloc((void**)&ctx->d_chi2, sizeof(double) * ninst));
    HIPCHK(cmalloc((void**)&ctx->d_istatus, sizeof(int) * ninst));
    HIPCHK(cmalloc((void**)&ctx->d_rscr, sizeof(double) * RSCR * (size_t)ninst));
    HIPCHK(hipMemsetAsync(ctx->d_istatus, 0, sizeof(int) * ninst, ctx->stream));
    for (int sl = 0; sl < pint_ctx::NSLOT; sl++) HIPCHK(cmalloc((void**)&ctx->d_chi2g_s[sl], sizeof(double) * ninst));
    HIPCHK(cmalloc((void**)&ctx->d_lognorm, sizeof(double) * ninst));
    for (int sl = 0; sl < pint_ctx::NSLOT; sl++) HIPCHK(cmalloc((void**)&ctx->d_chi2lin_s[sl], sizeof(double) * ninst));
    HIPCHK(cmalloc((void**)&ctx->d_G, sizeof(double) * goff));
    HIPCHK(cmalloc((void**)&ctx->d_colsq, sizeof(double) * coff * nsplit));
    HIPCHK(cmalloc((void**)&ctx->d_work, sizeof(double) * soff));
    for (int sl = 0; sl < pint_ctx::NSLOT; sl++)
        HIPCHK(cmalloc((void**)&ctx->d_cov_s[sl], sizeof(double) * (cvoff > 0 ? cvoff : 1)));
    HIPCHK(cmalloc((void**)&ctx->d_sigL, sizeof(double) * soff));
    for (int sl = 0; sl < pint_ctx::NSLOT; sl++) {
        HIPCHK(cmalloc((void**)&ctx->d_dpars_s[sl], sizeof(double) * coff));
        HIPCHK(cmalloc((void**)&ctx->d_errs_s[sl], sizeof(double) * coff));
        // the per-instance slot past the last column (K+1 stride) is never written by a solve
        HIPCHK(hipMemsetAsync(ctx->d_dpars_s[sl], 0, sizeof(double) * coff, ctx->stream));
        HIPCHK(hipMemsetAsync(ctx->d_errs_s[sl], 0, sizeof(double) * coff, ctx->stream));
    }
    ctx->out_slot = -1;
    select_out_slot(ctx, ctx->slot);
    HIPCHK(cmalloc((void**)&ctx->d_lam, sizeof(double) * ninst));
    HIPCHK(cmalloc((void**)&ctx->d_norms, sizeof(double) * coff));
    HIPCHK(cmalloc((void**)&ctx->d_ones, sizeof(double) * coff));
    HIPCHK(cmalloc((void**)&ctx->d_esum, sizeof(double) * (eoff > 0 ? eoff : 1)));
    HIPCHK(cmalloc((void**)&ctx->d_eD, sizeof(double) * (epoff > 0 ? epoff : 1)));
    HIPCHK(cmalloc((void**)&ctx->d_eW, sizeof(double) * (epoff > 0 ? epoff : 1)));
    HIPCHK(cmalloc((void**)&ctx->d_eC, sizeof(double) * (epoff > 0 ? epoff : 1)));
    HIPCHK(cmalloc((void**)&ctx->d_ecs, sizeof(double) * (epoff > 0 ? epoff : 1)));
    HIPCHK(cmalloc((void**)&ctx->d_ic, sizeof(InstConst) * ninst));
    HIPCHK(cmalloc((void**)&ctx->d_dmxv, sizeof(double) * (out > 0 ? out : 1)));
    {
        bool any_dmn = false;
        for (int k = 0; k < ninst; k++) any_dmn |= ctx->psrs[ctx->inst[k].psr].spec.dmn0 < ctx->psrs[ctx->inst[k].psr].spec.nred;
        HIPCHK(cmalloc((void**)&ctx->d_dfac, sizeof(double) * (any_dmn && out > 0 ? out : 1)));
    }
    HIPCHK(cmalloc((void**)&ctx->d_Sd, sizeof(double) * (sdoff > 0 ? sdoff : 1)));
    HIPCHK(cmalloc((void**)&ctx->d_DD, sizeof(double) * (ddoff > 0 ? ddoff : 1)));
    HIPCHK(cmalloc((void**)&ctx->d_DCS, sizeof(double) * (ddoff > 0 ? ddoff : 1)));
    HIPCHK(hipMemsetAsync(ctx->d_cov, 0, sizeof(double) * (cvoff > 0 ? cvoff : 1), ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PINT_OK;
}

static int flush_restore(pint_ctx* ctx);

// a lazy pint_chi2_gls copy not yet enqueued: on the kernel stream, in order
static int flush_chi2(pint_ctx* ctx) {
    if (!ctx->chi2_dst) return PINT_OK;
    double* dst = ctx->chi2_dst;
    ctx->chi2_dst = nullptr;
    HIPCHK(d2h(dst, ctx->d_chi2g, sizeof(double) * ctx->ninst, ctx->stream));
    return PINT_OK;
}

int pint_get_tables(pint_ctx* ctx, double* out) {
    if (flush_restore(ctx)) return PINT_E_HIP;
    HIPCHK(d2h(out, ctx->d_tables, sizeof(double) * ctx->tot_table, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PINT_OK;
}

int pint_set_tables(pint_ctx* ctx, const double* tables) {
    ctx->ic_valid = false;
    ctx->tables_fresh = false;
    ctx->restore_pending = false;  // overwritten anyway
    if (ctx->sigma_pending) HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_sigma, 0));  // k_sigma reads F0
    HIPCHK(h2d(ctx->d_tables, tables, sizeof(double) * ctx->tot_table, ctx->stream, false));
    if (!ctx->lazy) HIPCHK(hipStreamSynchronize(ctx->stream));
    return PINT_OK;
}

static const int kTimingPairs[pint_ctx::NMS][2] = {{0, 1}, {4, 5}, {6, 7}, {7, 8}, {2, 3}, {10, 11}, {12, 13}, {14, 15}};

static void record(pint_ctx* ctx, int i, hipStream_t st = nullptr) {
    if (ctx->no_events || ctx->capturing) return;  // no timing events inside a graph
    bool on = false;  // only the events of the enabled timing slots (each costs device time)
    for (int k = 0; k < pint_ctx::NMS; k++)
        if ((ctx->timing_mask >> k) & 1) on |= kTimingPairs[k][0] == i || kTimingPairs[k][1] == i;
    if (!on) return;
    if (!ctx->ev[i] && hipEventCreate(&ctx->ev[i]) != hipSuccess) return;
    hipEventRecord(ctx->ev[i], st ? st : ctx->stream);
    ctx->rec[i] = true;
}

static void update_timings(pint_ctx* ctx, bool zero_missing = false) {
    const auto& pairs = kTimingPairs;
    for (int k = 0; k < pint_ctx::NMS; k++) {
        if (!((ctx->timing_mask >> k) & 1)) continue;
        float t = 0.0f;
        if (ctx->rec[pairs[k][0]] && ctx->rec[pairs[k][1]] &&
            hipEventElapsedTime(&t, ctx->ev[pairs[k][0]], ctx->ev[pairs[k][1]]) == hipSuccess)
            ctx->ms[k] = t;
        else if (zero_missing)
            ctx->ms[k] = 0.0f;  // not recorded in this step (e.g. an unsampled Gram, PINT_OPT_TIMING_EVERY)
    }
}

static int decode_status(pint_ctx* ctx, int st);

static int flush_chi2(pint_ctx* ctx);

static int check_status(pint_ctx* ctx) {
    int st = 0;
    if (int rc = flush_cq_now(ctx)) return rc;
    if (flush_chi2(ctx)) return PINT_E_HIP;
    HIPCHK(hipStreamSynchronize(ctx->cstream));
    clear_copy_pend(ctx);
    HIPCHK(hipStreamSynchronize(ctx->sstream));
    HIPCHK(d2h(&st, ctx->d_status, sizeof(int), ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    // the status word accumulates error bits of everything enqueued since the last check
    if (st) HIPCHK(hipMemsetAsync(ctx->d_status, 0, sizeof(int), ctx->stream));
    return decode_status(ctx, st);
}

static int decode_status(pint_ctx* ctx, int st) {
    if (st & (1 << PINT_E_KEPLER)) { ctx->err = "Kepler equation: eccentricity outside [0,1) or no convergence"; return PINT_E_KEPLER; }
    if (st & (1 << PINT_E_SIGMA)) { ctx->err = "Woodbury Sigma (noise basis) not positive definite"; return PINT_E_SIGMA; }
    if (st & (1 << PINT_E_NOT_PD)) { ctx->err = "normal matrix not positive definite"; return PINT_E_NOT_PD; }
    if (st) { ctx->err = "device status " + std::to_string(st); return PINT_E_PARAM; }
    return PINT_OK;
}

// Evaluate phases/delays (+ design matrix) and residuals for every instance.
// k_prep / k_apply, or their lane-per-instance forms for a batch of small tables
static bool prep_lanes(const pint_ctx* ctx) { return ctx->prep_lanes && ctx->max_ts <= PREP_LANE_TAB; }
static void launch_prep(pint_ctx* ctx, double* tables, const double* tables0, InstConst* ic) {
    if (prep_lanes(ctx))
        hipLaunchKernelGGL(k_prep_lanes, dim3((ctx->ninst + 63) / 64), dim3(64), 0, ctx->stream, ctx->d_psrs,
                           ctx->d_inst, ctx->ninst, tables, tables0, ic);
    else
        hipLaunchKernelGGL(k_prep, dim3(ctx->ninst), dim3(PREP_T), 0, ctx->stream, ctx->d_psrs, ctx->d_inst, tables,
                           tables0, ic);
}
static void launch_apply(pint_ctx* ctx, const double* lam, double lam_u) {
    ctx->tables_fresh = false;
    if (prep_lanes(ctx))
        hipLaunchKernelGGL(k_apply_lanes, dim3((ctx->ninst + 63) / 64), dim3(64), 0, ctx->stream, ctx->d_psrs,
                           ctx->d_inst, ctx->ninst, ctx->d_tables, ctx->d_dpars, lam, ctx->d_ic, lam_u);
    else
        hipLaunchKernelGGL(k_apply, dim3(ctx->ninst), dim3(PREP_T), 0, ctx->stream, ctx->d_psrs, ctx->d_inst,
                           ctx->d_tables, ctx->d_dpars, lam, ctx->d_ic, lam_u);
}

// k_resid2 of the last residual pass (with wt, the Woodbury trig tiles)
static void launch_resid2(pint_ctx* ctx, bool wt) {
    const size_t wlds = wt ? sizeof(double) * std::max((RES_BT / 64) * 32 * WT_CS2, 4 * 256) : 0;
    const double* ep = ctx->efz ? ctx->d_epart : nullptr;
    if (!ctx->efz && ctx->small && ctx->maxn <= RES_SMALLN)
        hipLaunchKernelGGL(k_resid2<64>, dim3((ctx->nrblk + 3) / 4), dim3(RES_BT), wlds, ctx->stream, ctx->d_psrs,
                           ctx->d_inst, ctx->d_rblk_inst, ctx->nrblk, ctx->d_ftay, ctx->d_rt, ctx->d_rp, ctx->d_rpart,
                           wt ? ctx->d_wtile : nullptr, ep);
    else
        hipLaunchKernelGGL(k_resid2<RES_BT>, dim3(ctx->nrblk), dim3(RES_BT), wlds, ctx->stream, ctx->d_psrs,
                           ctx->d_inst, ctx->d_rblk_inst, ctx->nrblk, ctx->d_ftay, ctx->d_rt, ctx->d_rp, ctx->d_rpart,
                           wt ? ctx->d_wtile : nullptr, ep);
}

// The fit layout's residual pass may leave k_resid2 to the Gram (GvResid) when every instance
// takes k_gram_v and nothing else of the fit step reads the time residuals: no ECORR epochs
// (k_ecorr), no wideband rows (k_wb_gram), and <= 64 residual blocks per instance (the mean
// summed on one wave as k_resid2 sums it).  PINT_FUSE_R2=0 keeps k_resid2 in the pass.
static bool can_defer_r2(const pint_ctx* ctx) {
    return ctx->fuse_r2 && ctx->m_compact && ctx->n_vg == ctx->ninst && ctx->max_nep == 0 && !ctx->wbfit &&
           ctx->maxn <= 64 * (ctx->efz ? EF_ROWS : RES_RB);
}

// a reader of the time/phase residuals or their chi2 partials after a deferred pass
static void flush_r2(pint_ctx* ctx) {
    if (!ctx->r2_pending) return;
    ctx->r2_pending = false;
    launch_resid2(ctx, false);
}

int pint_eval(pint_ctx* ctx, int want_M) {
    if (!ctx || ctx->ninst <= 0) return PINT_E_INVALID;
    hipSetDevice(ctx->device);
    if (want_M < 0 || want_M > 2) return PINT_E_INVALID;
    ctx->r2_pending = false;  // (this pass replaces the residuals a deferred k_resid2 would form)
    if (want_M) ctx->m_compact = (want_M == 2) ? 1 : 0;
    // the full and compact layouts place the red-noise columns differently; each is written
    // once after pint_set_instances (M is reallocated there)
    int write_red = 0;
    if (want_M) {
        write_red = ctx->red_valid[want_M == 2] ? 0 : 1;
        ctx->red_valid[want_M == 2] = 1;
        ctx->red_valid[want_M != 2] = 0;  // the other layout's red columns get overwritten
        if (ctx->dm_noise_pend) {  // the evaluation with M rewrites the DM-noise scale d_dfac
            if (int rc = flush_cq_now(ctx)) return rc;
            HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_copied, 0));
            ctx->dm_noise_pend = false;
        }
    }
    record(ctx, want_M ? 2 : 0);
    const double* tabs = ctx->d_tables;
    const InstConst* icp = ctx->d_ic;
    EvalRestore rs{nullptr, nullptr, nullptr, nullptr};
    if (!ctx->ic_valid) {  // (k_apply refreshes them itself)
        if (ctx->restore_pending && ctx->ic0_valid) {
            // restore: the evaluation reads the snapshot and its constants (pint_save_tables) and
            // each instance's first block writes them back -- no k_prep launch in a refit step
            tabs = ctx->d_tables0;
            icp = ctx->d_ic0;
            rs.tables = ctx->d_tables;
            rs.ic = ctx->d_ic;
        } else {
            launch_prep(ctx, ctx->d_tables, ctx->restore_pending ? (const double*)ctx->d_tables0 : nullptr, ctx->d_ic);
            HIPCHK(hipGetLastError());
        }
        ctx->restore_pending = false;
        ctx->ic_valid = true;
    }
    if (ctx->efz && ctx->nrblk > 0) {  // the residual pass's first half in the evaluation's blocks
        rs.rph = ctx->d_rp;
        rs.epart = ctx->d_epart;
    }
    // a spin-only grid's first evaluation with the design matrix: the shared head, then each
    // point's spin part
    const bool spin_pass = want_M && ctx->spin_grid && ctx->tables_fresh && ctx->spin_eval && rs.tables == nullptr &&
                           !ctx->efz && ctx->d_shr && ctx->blk_off[PINT_NBIN] == ctx->blk_off[1];
    if (spin_pass) {
        const int n1 = ctx->inst[0].n + 1;
        hipLaunchKernelGGL(k_eval_head, dim3((n1 + 255) / 256), dim3(256), 0, ctx->stream, ctx->d_psrs, ctx->d_inst,
                           tabs, icp, ctx->d_shr);
        hipLaunchKernelGGL(k_eval_spin, dim3((ctx->ninst + 3) / 4), dim3(256), 0, ctx->stream, ctx->d_psrs, ctx->d_inst,
                           ctx->ninst, tabs, icp, ctx->d_shr, ctx->d_phhi, ctx->d_phlo, ctx->d_ftay, ctx->d_delay,
                           ctx->d_M);
        HIPCHK(hipGetLastError());
    }
    // a batch of one model (a grid's points, an all-isolated PTA) takes that model's own
    // build, whose register set the other models do not raise (k_eval<WM, 0>: 48 instead
    // of 84 VGPRs + spills with M for an isolated pulsar); PINT_EVAL_MERGE bit 2 merges anyway
    int ntyp = 0;
    for (int t = 0; t < 3; t++) ntyp += ctx->blk_off[t + 1] > ctx->blk_off[t];
    const bool mix = ((ctx->eval_merge >> (want_M ? 1 : 0)) & 1) && (ntyp > 1 || (ctx->eval_merge & 4));
    if (!spin_pass && mix && ctx->nblk > 0) {
#define PINT_EVAL_MIX(WM)                                                                                      \
        hipLaunchKernelGGL((k_eval_mix<WM>), dim3(ctx->nblk), dim3(256), 0, ctx->stream, ctx->d_psrs, ctx->d_inst, \
                           ctx->d_blk_inst, ctx->d_blk_row0, ctx->blk_off[1], ctx->blk_off[2], ctx->blk_off[3],   \
                           tabs, icp, ctx->d_phhi, ctx->d_phlo, ctx->d_ftay, ctx->d_delay, ctx->d_M, \
                           ctx->d_dmxv, want_M == 2 ? 1 : 0, write_red, ctx->d_status, ctx->d_istatus, ctx->d_dfac, rs)
        // the 3-waves/SIMD register budget (spills) pays when the blocks fill the SIMDs more
        // than twice; a small batch (<= 2 waves per SIMD) runs the unconstrained build (203
        // VGPRs, no spills) at its own occupancy
        const bool small = ctx->nblk <= 2 * 256;
        if (want_M && ctx->eval_wpe == 3 && !small) {
            hipLaunchKernelGGL((k_eval_mix_w<1, 3>), dim3(ctx->nblk), dim3(256), 0, ctx->stream, ctx->d_psrs, ctx->d_inst,
                               ctx->d_blk_inst, ctx->d_blk_row0, ctx->blk_off[1], ctx->blk_off[2], ctx->blk_off[3],
                               tabs, icp, ctx->d_phhi, ctx->d_phlo, ctx->d_ftay, ctx->d_delay, ctx->d_M,
                               ctx->d_dmxv, want_M == 2 ? 1 : 0, write_red, ctx->d_status, ctx->d_istatus, ctx->d_dfac, rs);
        } else if (want_M && ctx->eval_wpe == 4) {
            hipLaunchKernelGGL((k_eval_mix_w<1, 4>), dim3(ctx->nblk), dim3(256), 0, ctx->stream, ctx->d_psrs, ctx->d_inst,
                               ctx->d_blk_inst, ctx->d_blk_row0, ctx->blk_off[1], ctx->blk_off[2], ctx->blk_off[3],
                               tabs, icp, ctx->d_phhi, ctx->d_phlo, ctx->d_ftay, ctx->d_delay, ctx->d_M,
                               ctx->d_dmxv, want_M == 2 ? 1 : 0, write_red, ctx->d_status, ctx->d_istatus, ctx->d_dfac, rs);
        } else if (want_M) PINT_EVAL_MIX(1); else PINT_EVAL_MIX(0);
#undef PINT_EVAL_MIX
        HIPCHK(hipGetLastError());
    }
    // one launch per binary model, back to back on the stream: all models without the merged
    // launch; ELL1H/BT/DDK always (they stay out of k_eval_mix so its register set, which
    // every block of the merged launch carries, is not raised by the rarer models)
    for (int t = spin_pass ? PINT_NBIN : (mix ? 3 : 0); t < PINT_NBIN; t++) {
        int nb = ctx->blk_off[t + 1] - ctx->blk_off[t];
        if (nb == 0) continue;
        const int* bi = ctx->d_blk_inst + ctx->blk_off[t];
        const int* br = ctx->d_blk_row0 + ctx->blk_off[t];
#define PINT_EVAL_LAUNCH(WM, BT, ...)                                                                     \
        hipLaunchKernelGGL((k_eval<WM, BT, ##__VA_ARGS__>), dim3(nb), dim3(256), 0, ctx->stream, ctx->d_psrs, ctx->d_inst, bi, br, \
                           tabs, icp, ctx->d_phhi, ctx->d_phlo, ctx->d_ftay, ctx->d_delay, ctx->d_M, \
                           ctx->d_dmxv, want_M == 2 ? 1 : 0, write_red, ctx->d_status, ctx->d_istatus, ctx->d_dfac, rs)
        // the isolated build at a register budget of 6 waves/SIMD with M (80 VGPRs, no spills:
        // 0.28 vs 0.31 ms on the 65,536-point NGC6440E grid) and 8 without (64 VGPRs, 36 B of
        // spills: 0.143 vs 0.162 ms); 8 with M spilled 76 B and lost (0.35 ms).
        // PINT_EVAL0_WPE=0: the compiler's own allocation (84 / 74 VGPRs, 5 / 6 waves)
        if (t == 0 && ctx->eval0_wpe) {
            if (want_M) PINT_EVAL_LAUNCH(1, 0, 6); else PINT_EVAL_LAUNCH(0, 0, 8);
        } else if (want_M && (t == 1 || t == 2) && ctx->evalb_wpe == 3 && nb > 2 * 256) {
            // a large one-model ELL1 or DD batch (a J0740 grid) with M at the merged build's
            // budget of 3 waves/SIMD (168 VGPRs + spills) instead of 2 (174 / 202 VGPRs)
            if (t == 1) PINT_EVAL_LAUNCH(1, 1, 3); else PINT_EVAL_LAUNCH(1, 2, 3);
        } else if (want_M) {
            switch (t) {
                case 0: PINT_EVAL_LAUNCH(1, 0); break;
                case 1: PINT_EVAL_LAUNCH(1, 1); break;
                case 2: PINT_EVAL_LAUNCH(1, 2); break;
                case 3: PINT_EVAL_LAUNCH(1, 3); break;
                case 4: PINT_EVAL_LAUNCH(1, 4); break;
                default: PINT_EVAL_LAUNCH(1, 5); break;
            }
        } else {
            switch (t) {
                case 0: PINT_EVAL_LAUNCH(0, 0); break;
                case 1: PINT_EVAL_LAUNCH(0, 1); break;
                case 2: PINT_EVAL_LAUNCH(0, 2); break;
                case 3: PINT_EVAL_LAUNCH(0, 3); break;
                case 4: PINT_EVAL_LAUNCH(0, 4); break;
                default: PINT_EVAL_LAUNCH(0, 5); break;
            }
        }
#undef PINT_EVAL_LAUNCH
        HIPCHK(hipGetLastError());
    }
    record(ctx, want_M ? 3 : 1);
    record(ctx, 4);
    if (ctx->nrblk > 0) {
        // without the design matrix (the post-fit evaluation a GLS chi2 follows): the Woodbury
        // dot products come with the residual pass (k_resid2 tiles, k_rsum)
        const bool wt = ctx->wfuse && want_M == 0;
        // (256-row blocks for small batches were measured: resid1 faster, resid2 and k_wsolve's
        // longer tile sums slower, the step ~1.4 us slower at 9 pulsars)
        // the fit layout's pass on the k_gram_v path: k_resid1 only, the Gram stages the time
        // residuals itself and k_resid2 waits for a reader of them (flush_r2)
        const bool defer2 = want_M == 2 && can_defer_r2(ctx);
        const bool fused12 = !ctx->efz && ctx->small && ctx->maxn <= RES_SMALLN && !wt && !defer2 && ctx->resid12;
        if (ctx->efz) {
            // (k_resid1's work done by the evaluation's blocks)
        } else if (fused12) {  // one wave per instance does both passes
            hipLaunchKernelGGL(k_resid12, dim3((ctx->nrblk + 3) / 4), dim3(RES_BT), 0, ctx->stream, ctx->d_psrs,
                               ctx->d_inst, ctx->d_rblk_inst, ctx->nrblk, ctx->d_phhi, ctx->d_phlo, ctx->d_ftay,
                               ctx->d_rt, ctx->d_rp, ctx->d_rpart);
        } else if (ctx->small && ctx->maxn <= RES_SMALLN) {  // a wave per residual block
            const int nb4 = (ctx->nrblk + 3) / 4;
            hipLaunchKernelGGL(k_resid1<64>, dim3(nb4), dim3(RES_BT), 0, ctx->stream, ctx->d_psrs, ctx->d_inst,
                               ctx->d_rblk_inst, ctx->nrblk, ctx->d_phhi, ctx->d_phlo, ctx->d_rp, ctx->d_rpart);
        } else {
            hipLaunchKernelGGL(k_resid1<RES_BT>, dim3(ctx->nrblk), dim3(RES_BT), 0, ctx->stream, ctx->d_psrs,
                               ctx->d_inst, ctx->d_rblk_inst, ctx->nrblk, ctx->d_phhi, ctx->d_phlo, ctx->d_rp,
                               ctx->d_rpart);
        }
        if (defer2) ctx->r2_pending = true;
        else if (!fused12) launch_resid2(ctx, wt);
        // the chi2 partials are summed when the chi2 is read (pint_read_resids) or by k_wsolve,
        // which needs them anyway: no launch of its own in a fit step
        ctx->chi2_pending = true;
        ctx->wtile_valid = wt;
    }
    HIPCHK(hipGetLastError());
    record(ctx, 5);
    if (ctx->lazy) return PINT_OK;
    int rc = check_status(ctx);
    update_timings(ctx);
    return rc;
}

int pint_read_resids(pint_ctx* ctx, double* time_resid, double* phase_resid, double* chi2) {
    flush_r2(ctx);
    if (chi2 && ctx->chi2_pending) {
        hipLaunchKernelGGL(k_rsum, dim3(ctx->ninst), dim3(64), 0, ctx->stream, ctx->d_inst, ctx->d_rpart, ctx->d_chi2);
        HIPCHK(hipGetLastError());
        ctx->chi2_pending = false;
    }
    if (time_resid) HIPCHK(d2h(time_resid, ctx->d_rt, sizeof(double) * ctx->tot_out, ctx->stream));
    if (phase_resid) HIPCHK(d2h(phase_resid, ctx->d_rp, sizeof(double) * ctx->tot_out, ctx->stream));
    if (chi2) HIPCHK(d2h(chi2, ctx->d_chi2, sizeof(double) * ctx->ninst, ctx->stream));
    if (!ctx->lazy) HIPCHK(hipStreamSynchronize(ctx->stream));  // lazy: valid after pint_check
    return PINT_OK;
}

int pint_set_wideband(pint_ctx* ctx, int psr, const double* pp_dm, const double* pp_dme, const double* dm_sigma,
                      const uint64_t* dmjump_mask) {
    if (!ctx || psr < 0 || psr >= (int)ctx->psrs.size() || !pp_dm || !pp_dme || !dm_sigma) return PINT_E_INVALID;
    hipSetDevice(ctx->device);
    if (int rc_ = commit_uploads(ctx)) return rc_;  // (staged pulsar uploads first)
    PsrHost& ph = ctx->psrs[psr];
    if (ph.spec.ndmjump > 0 && !dmjump_mask) { ctx->err = "DMJUMPs without masks"; return PINT_E_INVALID; }
    for (int i = 0; i < ph.n; i++)
        if (!(dm_sigma[i] > 0.0) || !(pp_dme[i] > 0.0)) {
            ctx->err = "Some DM errors are zero - cannot calculate the weighted residuals.";
            return PINT_E_INVALID;
        }
    int rc = 0;
    rc |= upload(ctx, ph, pp_dm, (size_t)ph.n, ph.dev.pp_dm);
    rc |= upload(ctx, ph, pp_dme, (size_t)ph.n, ph.dev.pp_dme);
    rc |= upload(ctx, ph, dm_sigma, (size_t)ph.n, ph.dev.dm_sig);
    if (ph.spec.ndmjump > 0) rc |= upload(ctx, ph, dmjump_mask, (size_t)ph.n, ph.dev.dmjmask);
    if (rc) return PINT_E_HIP;
    ph.dev.wb = 1;
    return refresh_psrs(ctx) ? PINT_E_HIP : PINT_OK;
}

int pint_dm_resids(pint_ctx* ctx, int subtract_mean, int use_weighted_mean, double* resid_out, double* chi2_out) {
    if (!ctx || ctx->ninst <= 0) return PINT_E_INVALID;
    if (flush_restore(ctx)) return PINT_E_HIP;
    hipSetDevice(ctx->device);
    if (ctx->tot_out > ctx->dmr_cap) {
        if (ctx->d_dmr) hipFree(ctx->d_dmr);
        ctx->d_dmr = nullptr;
        HIPCHK(hipMalloc((void**)&ctx->d_dmr, sizeof(double) * std::max<long>(1, ctx->tot_out)));
        ctx->dmr_cap = ctx->tot_out;
    }
    if (ctx->ninst > ctx->dmc2_cap) {
        if (ctx->d_dmc2) hipFree(ctx->d_dmc2);
        ctx->d_dmc2 = nullptr;
        HIPCHK(hipMalloc((void**)&ctx->d_dmc2, sizeof(double) * ctx->ninst));
        ctx->dmc2_cap = ctx->ninst;
    }
    hipLaunchKernelGGL(k_dm_resid, dim3(ctx->ninst), dim3(DMR_T), 0, ctx->stream, ctx->d_psrs, ctx->d_inst,
                       ctx->d_tables, subtract_mean, use_weighted_mean, ctx->d_dmr, ctx->d_dmc2);
    HIPCHK(hipGetLastError());
    if (resid_out) HIPCHK(d2h(resid_out, ctx->d_dmr, sizeof(double) * ctx->tot_out, ctx->stream));
    if (chi2_out) HIPCHK(d2h(chi2_out, ctx->d_dmc2, sizeof(double) * ctx->ninst, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PINT_OK;
}

int pint_read_eval(pint_ctx* ctx, double* ph_hi, double* ph_lo, double* ftaylor, double* delay) {
    size_t b = sizeof(double) * ctx->tot_rows;
    if (ph_hi) HIPCHK(d2h(ph_hi, ctx->d_phhi, b, ctx->stream));
    if (ph_lo) HIPCHK(d2h(ph_lo, ctx->d_phlo, b, ctx->stream));
    if (ftaylor) HIPCHK(d2h(ftaylor, ctx->d_ftay, b, ctx->stream));
    if (delay) HIPCHK(d2h(delay, ctx->d_delay, b, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PINT_OK;
}

int pint_read_designmatrix(pint_ctx* ctx, double* M) {
    HIPCHK(d2h(M, ctx->d_M, sizeof(double) * ctx->tot_m, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PINT_OK;
}

// Gram + solve for every instance; requires pint_eval(want_M=1) on the current state.
int pint_fit_step(pint_ctx* ctx, int mode) {
    if (!ctx || ctx->ninst <= 0) return PINT_E_INVALID;
    if (flush_restore(ctx)) return PINT_E_HIP;
    hipSetDevice(ctx->device);
    // deferred reads of this slot's outputs enqueued since the last step_end go first (this
    // solve rewrites them)
    if (int rc = flush_cq_now(ctx)) return rc;
    if (ctx->r2_pending && !can_defer_r2(ctx)) flush_r2(ctx);  // (a kernel below reads d_rt)
    const GvResid gvr{ctx->d_rp, ctx->d_ftay, ctx->d_rpart, ctx->r2_pending ? 1 : 0, ctx->efz ? ctx->d_epart : nullptr};
    if (ctx->wbfit) {
        // k_wb_gram carries at most WB_MAXC free DM-type columns (DM Taylor terms + DMJUMPs):
        // refuse more instead of leaving the extra columns without their DM rows
        for (int pi : ctx->upsr) {
            const pint_spec_t& sp = ctx->psrs[pi].spec;
            if (!ctx->psrs[pi].dev.wb) continue;
            int m = 0;
            for (int c = 0; c < sp.ncol; c++) m += (sp.col_kind[c] == PINT_COL_DM || sp.col_kind[c] == PINT_COL_ZERO);
            if (m > WB_MAXC) {
                ctx->err = "wideband fit: more than 8 free DM-type columns (DM Taylor terms + DMJUMPs)";
                return PINT_E_INVALID;
            }
        }
    }
    const int nparts = ctx->nsplit + ((mode == 1 && ctx->max_nep > 0) ? 1 : 0);
    if (ctx->sigma_pending) {  // the previous k_sigma reads the Gram buffer this step overwrites
        HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_sigma, 0));
        ctx->sigma_pending = false;
    }
    record(ctx, 6);
    if (mode == 1 && ctx->max_nep > 0) {
        if (any_copy_pend(ctx)) {  // the copy stream's noise realisations read esum / eD
            HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_copied, 0));
            clear_copy_pend(ctx);
        }
        hipLaunchKernelGGL(k_ecorr, dim3((ctx->max_nep + 3) / 4, ctx->ninst), dim3(256), 0, ctx->stream, ctx->d_psrs,
                           ctx->d_inst, ctx->d_M, ctx->d_rt, ctx->d_esum, ctx->d_eD, ctx->d_eW, ctx->m_compact,
                           ctx->d_dmxv, ctx->d_eC);
        HIPCHK(hipGetLastError());
    }
    const int cmp = ctx->m_compact;
    const bool vgp = cmp && ctx->n_vg > 0;  // k_gram_v path for the vg instances
    // PhaseOffset with a frozen PHOFF and correlated noise: the Woodbury ones row (k_onesrow)
    const double* ones = nullptr;
    if (mode == 1) {
        for (int pi : ctx->upsr) {
            const PsrHost& ph = ctx->psrs[pi];
            if (ph.spec.o_PHOFF >= 0 && !ph.spec.wb_noones && (ph.spec.nred > 0 || ph.dev.nep > 0)) ones = ctx->d_ones;
        }
        if (ones) {
            hipLaunchKernelGGL(k_onesrow, dim3(ctx->ninst), dim3(64), 0, ctx->stream, ctx->d_psrs, ctx->d_inst,
                               ctx->d_esum, ctx->d_eD, ctx->d_eW, ctx->d_eC, cmp, ctx->d_M, ctx->d_ones);
            HIPCHK(hipGetLastError());
        }
    }
    if (cmp && ctx->max_ndc > 0 && ctx->any_dmx_rows) {
        int maxKd = 0;
        bool any_gather = false;
        for (int pi : ctx->upsr) {
            const PsrDev& pd = ctx->psrs[pi].dev;
            if (pd.dsplit) maxKd = std::max(maxKd, pd.Kd);
            if (pd.dsplit && !pd.dcontig) any_gather = true;
        }
        size_t lds = sizeof(double) * (DMX_RS * ((maxKd + 2) | 1) + 2 * DMX_RS);
        hipLaunchKernelGGL(k_dmx_rows, dim3(ctx->max_ndc, ctx->ninst), dim3(256), lds, ctx->stream, ctx->d_psrs,
                           ctx->d_inst, ctx->d_M, ctx->d_rt, ctx->d_dmxv, ctx->d_Sd, ctx->d_DD, ctx->d_DCS);
        HIPCHK(hipGetLastError());
        if (any_gather) {
            hipLaunchKernelGGL(k_dmx, dim3(ctx->max_ndc, ctx->ninst), dim3(256), 0, ctx->stream, ctx->d_psrs,
                               ctx->d_inst, ctx->d_M, ctx->d_rt, ctx->d_dmxv, ctx->d_Sd, ctx->d_DD, ctx->d_DCS);
            HIPCHK(hipGetLastError());
        }
        if (mode == 1 && ctx->max_nep > 0) {  // the ECORR elimination's share of the DMX rows
            hipLaunchKernelGGL(k_ecorr_dmx, dim3(ctx->max_ndc, ctx->ninst), dim3(64), 0, ctx->stream, ctx->d_psrs,
                               ctx->d_inst, ctx->d_esum, ctx->d_eD, ctx->d_eC, ctx->d_Sd, ctx->d_DD);
            HIPCHK(hipGetLastError());
        }
    }
    // Gram-kernel timing: when the whole Gram is k_gram_v launches, the slot's start/stop
    // events ride on the first/last dispatch packet (hipExtLaunchKernel) instead of marker
    // packets between kernels, which cost the stream ~10 us each
    // PINT_OPT_TIMING_EVERY k: the Gram events ride on every k-th fit step only (each event
    // pair still costs the stream a few us; the average over the sampled launches is the
    // kernel's time)
    const bool sampled = ctx->timing_every <= 1 || (ctx->gram_calls++ % ctx->timing_every) == 0;
    const bool gram_t = !ctx->no_events && !ctx->capturing && ((ctx->timing_mask >> 6) & 1) && sampled;
    const bool ext_t = gram_t && vgp && (cmp ? ctx->kp_groups_c : ctx->kp_groups).empty() &&
                       !ctx->kp_groups_v.empty();
    const bool gram_mark = sampled && !ext_t;  // marker-packet events (the other Gram paths)
    if (gram_mark) record(ctx, 12);
    {
        // instances are launched in groups of equal tiles-per-wave T (template parameter);
        // per-instance tile counts are recomputed in-kernel from their own Kp.
        const std::vector<KpGroup>& groups = cmp ? ctx->kp_groups_c : ctx->kp_groups;
        for (int g = 0; g < (int)groups.size(); g++) {
            const KpGroup& kg = groups[g];
            const int T = kg.T;
            const InstDev* di = (cmp ? ctx->d_inst_sorted_c : ctx->d_inst_sorted) + kg.first;
            if (T == 0) {  // small instances: k_gram_s (the ECORR rows, if any, by k_gram<1> below)
                hipLaunchKernelGGL(k_gram_s, dim3(ctx->nsplit, (kg.count + 3) / 4), dim3(256), 0, ctx->stream,
                                   ctx->d_psrs, di, kg.count, ctx->d_M, ctx->d_rt, ctx->nsplit, cmp, ctx->d_G,
                                   ctx->d_colsq);
                if (mode == 1 && ctx->max_nep > 0)
                    hipLaunchKernelGGL((k_gram<1, gram_ch(1), true>), dim3(1, kg.count), dim3(GTHREADS),
                                       sizeof(double) * ((size_t)kg.maxKp * (gram_ch(1) + 2) + gram_ch(1)),
                                       ctx->stream, ctx->d_psrs, di, ctx->d_M, ctx->d_rt, ctx->d_esum, ctx->d_eD,
                                       ctx->nsplit, cmp, ctx->d_G, ctx->d_colsq);
                continue;
            }
            const int CH = gram_ch(T);
            size_t lds = sizeof(double) * ((size_t)kg.maxKp * (CH + 2) + CH);
            for (int virt = 0; virt < 2; virt++) {
                if (virt && !(mode == 1 && ctx->max_nep > 0)) break;
                dim3 grid(virt ? 1 : ctx->nsplit, kg.count);
#define PINT_GRAM_CASE(TT)                                                                                         \
                case TT:                                                                                           \
                    if (virt) hipLaunchKernelGGL((k_gram<TT, gram_ch(TT), true>), grid, dim3(GTHREADS), lds,      \
                                                 ctx->stream, ctx->d_psrs, di, ctx->d_M, ctx->d_rt, ctx->d_esum,  \
                                                 ctx->d_eD, ctx->nsplit, cmp, ctx->d_G, ctx->d_colsq);            \
                    else hipLaunchKernelGGL((k_gram<TT, gram_ch(TT), false>), grid, dim3(GTHREADS), lds,         \
                                            ctx->stream, ctx->d_psrs, di, ctx->d_M, ctx->d_rt, ctx->d_esum,       \
                                            ctx->d_eD, ctx->nsplit, cmp, ctx->d_G, ctx->d_colsq);                 \
                    break;
                switch (T) {
                    PINT_GRAM_CASE(1) PINT_GRAM_CASE(2) PINT_GRAM_CASE(3) PINT_GRAM_CASE(4) PINT_GRAM_CASE(5)
                    PINT_GRAM_CASE(6) PINT_GRAM_CASE(7) PINT_GRAM_CASE(8) PINT_GRAM_CASE(9)
                    default: ctx->err = "Kp out of range"; return PINT_E_INVALID;
                }
#undef PINT_GRAM_CASE
            }
        }
    }
    if (ext_t)  // (the timing events are created at first use)
        for (int i : {12, 13})
            if (!ctx->ev[i]) HIPCHK(hipEventCreate(&ctx->ev[i]));
    if (vgp) {
        for (size_t gi = 0; gi < ctx->kp_groups_v.size(); gi++) {
            const KpGroup& kg = ctx->kp_groups_v[gi];
            const InstDev* di = ctx->d_inst_sorted_v + kg.first;
            hipEvent_t e0 = (ext_t && gi == 0) ? ctx->ev[12] : nullptr;
            hipEvent_t e1 = (ext_t && gi + 1 == ctx->kp_groups_v.size()) ? ctx->ev[13] : nullptr;
            dim3 grid(ctx->nsplit, kg.count);
            const size_t lds = sizeof(double) * std::max<size_t>((size_t)GVB * (kg.maxKp + (ctx->vb_on && kg.maxKp <= 96 ? 33 : 17)) * (VCH + 2),
                                                                 std::max(GW * VTG * 256, GW * 256 + 256));
#define PINT_GRAMV(R_, C_)                                                                                       \
            if (ctx->vb_on && C_ <= 6)                                                                               \
                hipExtLaunchKernelGGL((k_gram_v<R_, C_, true>), grid, dim3(GW * 64), (uint32_t)lds, ctx->stream, e0, e1, \
                                      0u, (const PsrDev*)ctx->d_psrs, di, (const double*)ctx->d_M,                    \
                                      (const double*)ctx->d_rt, (const double*)ctx->d_dmxv, ctx->nsplit, ctx->d_G,     \
                                      ctx->d_Sdp, ctx->d_colsq, ctx->d_TSp, ctx->d_BFp, ctx->gvdbg, gvr);              \
            else                                                                                                     \
                hipExtLaunchKernelGGL((k_gram_v<R_, C_, false>), grid, dim3(GW * 64), (uint32_t)lds, ctx->stream, e0, e1, \
                                      0u, (const PsrDev*)ctx->d_psrs, di, (const double*)ctx->d_M,                    \
                                      (const double*)ctx->d_rt, (const double*)ctx->d_dmxv, ctx->nsplit, ctx->d_G,     \
                                      ctx->d_Sdp, ctx->d_colsq, ctx->d_TSp, ctx->d_BFp, ctx->gvdbg, gvr)
            switch (kg.T) {
                case 1: PINT_GRAMV(1, 1); break;
                case 2: PINT_GRAMV(1, 2); break;
                case 3: PINT_GRAMV(1, 3); break;
                case 4: PINT_GRAMV(1, 4); break;
                case 5: PINT_GRAMV(1, 5); break;
                case 6: PINT_GRAMV(1, 6); break;
                case 7: PINT_GRAMV(1, 7); break;
                case 12: PINT_GRAMV(2, 2); break;
                case 13: PINT_GRAMV(2, 3); break;
                case 14: PINT_GRAMV(2, 4); break;
                case 15: PINT_GRAMV(2, 5); break;
                case 16: PINT_GRAMV(2, 6); break;
                case 17: PINT_GRAMV(2, 7); break;
                case 23: PINT_GRAMV(3, 3); break;
                case 24: PINT_GRAMV(3, 4); break;
                case 25: PINT_GRAMV(3, 5); break;
                case 26: PINT_GRAMV(3, 6); break;
                case 27: PINT_GRAMV(3, 7); break;
                default: ctx->err = "k_gram_v layout out of range"; return PINT_E_INVALID;
            }
#undef PINT_GRAMV
        }
        if (ext_t) ctx->rec[12] = ctx->rec[13] = true;
        else if (gram_mark) record(ctx, 13);
    } else if (gram_mark) {
        record(ctx, 13);
    }
    HIPCHK(hipGetLastError());
    // solve plan: the DMX-eliminated solve (k_solve_dmx) for compact-layout instances when
    // every such instance fits its LDS budget; the others (and everything in the full
    // layout) go to the blocked MFMA solve, or the column-by-column one beyond its budget.
    int Ks = 0, Kn = 0, ndmx_inst = 0;
    bool dmx_ok = cmp && ctx->blocked_solve;
    size_t lds_x = 0;
    for (int pi : ctx->upsr) {
        const PsrHost& ph = ctx->psrs[pi];
        const pint_spec_t& sp = ph.spec;
        const int kn = mode == 1 ? 2 * sp.nred + 1 : 0;
        Kn = std::max(Kn, kn);
        if (cmp && ph.dev.dsplit) {
            ndmx_inst++;
            const int kd = mode == 0 ? ph.dev.red0c : ph.dev.Kd;
            const int nbd = (kd + 15) / 16, nbk = (ph.dev.ndc + 15) / 16, nbs = (kn + 15) / 16;
            const int blk = nbd * (nbd + 1) / 2 + nbd * nbk;
            if (blk > SD_MAXBLK || nbd > 17 || nbs > BS_MAXNB) dmx_ok = false;
            lds_x = std::max(lds_x, sizeof(double) * ((size_t)std::max(blk, nbs * (nbs + 1) / 2) * 256 +
                                                      (size_t)(5 * nbd + 6 * nbk) * 16));
            if (lds_x > 160 * 1024 - 512) dmx_ok = false;  // (the kernel's static LDS beside it)
        } else {
            Ks = std::max(Ks, mode == 0 ? sp.ncol : ph.K);
        }
    }
    if (!dmx_ok) {  // every instance through the general solve
        for (int pi : ctx->upsr) Ks = std::max(Ks, mode == 0 ? ctx->psrs[pi].spec.ncol : ctx->psrs[pi].K);
        ndmx_inst = 0;
    }
    const int skip = ndmx_inst > 0 ? 1 : 0;
    // Woodbury Sigma factor: in k_solve_dmx's grid when every instance is solved there, else
    // on the side stream, concurrent with the per-instance solve
    int do_sigma = 0, fuse_sigma = 0, side_sigma = 0, nbs_sig = 0;
    size_t lds_s = 0;
    if (mode == 1) {
        int kn = 0;
        bool any = false;
        for (int pi : ctx->upsr) {
            const PsrHost& ph = ctx->psrs[pi];
            if (ph.spec.nred > 0 || ph.dev.nep > 0) { any = true; kn = std::max(kn, 2 * ph.spec.nred + 1); }
        }
        nbs_sig = (kn + 15) / 16;
        lds_s = sizeof(double) * (size_t)nbs_sig * (nbs_sig + 1) / 2 * 256;
        if (any && nbs_sig <= BS_MAXNB && ctx->blocked_solve && skip && Ks == 0) fuse_sigma = 1;
        else if (any && nbs_sig <= BS_MAXNB && ctx->blocked_solve) side_sigma = 1;
        else if (any) do_sigma = 1;  // the column-by-column solve factors it (beyond the blocked LDS budget)
    }
    GredArgs gra{ctx->nsplit, nparts, cmp, ctx->vb_on, ctx->d_G, ctx->d_colsq, ctx->d_Sdp, ctx->d_dmxv,
                 ctx->d_Sd, ctx->d_DD, ctx->d_DCS, ctx->d_BFp};
    if (nparts > 1 || vgp) {
        int maxKp = 16;
        for (int pi : ctx->upsr) {
            const PsrDev& pd = ctx->psrs[pi].dev;
            maxKp = std::max(maxKp, (cmp && pd.dsplit) ? pd.Kpd : pd.Kp);
        }
        // (round 4: the column sums of squares on threads of their own, beside the Gram's
        // chains, measured no faster -- 11.3-11.9 vs 10.5-10.9 us at 9 pulsars)
        const int nbg = (maxKp * maxKp + 255) / 256;
        record(ctx, 14);
        hipLaunchKernelGGL(k_greduce, dim3(nbg + (vgp ? (ctx->max_ndc + 3) / 4 : 0), ctx->ninst), dim3(256), 0, ctx->stream,
                           ctx->d_psrs, ctx->d_inst, nbg, gra);
        HIPCHK(hipGetLastError());
        record(ctx, 15);
    }
    if (ctx->wbfit && cmp) {  // WidebandTOAFitter: the DM rows join the normal equations
        hipLaunchKernelGGL(k_wb_gram, dim3(ctx->ninst), dim3(256), 0, ctx->stream, ctx->d_psrs, ctx->d_inst,
                           ctx->d_tables, ctx->nsplit, ctx->d_G, ctx->d_colsq, ctx->d_Sd, ctx->d_DD, ctx->d_DCS);
        HIPCHK(hipGetLastError());
    }
    record(ctx, 7);
    if (side_sigma) {
        HIPCHK(hipEventRecord(ctx->ev_gram, ctx->stream));
        HIPCHK(hipStreamWaitEvent(ctx->sstream, ctx->ev_gram, 0));
        if (nbs_sig <= 5)
            hipLaunchKernelGGL(k_sigma<4>, dim3(ctx->ninst), dim3(256), lds_s, ctx->sstream, ctx->d_psrs, ctx->d_inst,
                               ctx->d_tables, ctx->d_G, cmp, ctx->d_Sd, ctx->d_DD, ctx->d_sigL, ctx->d_status, ones);
        else
            hipLaunchKernelGGL(k_sigma<16>, dim3(ctx->ninst), dim3(1024), lds_s, ctx->sstream, ctx->d_psrs,
                               ctx->d_inst, ctx->d_tables, ctx->d_G, cmp, ctx->d_Sd, ctx->d_DD, ctx->d_sigL,
                               ctx->d_status, ones);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(ctx->ev_sigma, ctx->sstream));
        ctx->sigma_pending = true;
    }
    if (ctx->copy_pend[ctx->slot]) {  // this slot's outputs may still be in flight to the host
        HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_copied, 0));  // (the latest copies: covers them)
        clear_copy_pend(ctx);
    }
    ctx->cov_pending = false;
    if (skip) {
        // deferred covariance for batches (a single fit would pay a launch on its read instead)
        // (and in lazy, pipelined steps of any size: the read runs k_cov_dmx on the copy stream,
        // beside the next kernels, so a small batch's solve does not carry it either)
        double* xw = (ctx->d_xw && (ctx->cov_defer == 2 || (ctx->cov_defer == 1 && (ctx->ninst >= 16 || ctx->lazy))))
                         ? ctx->d_xw : nullptr;
        // (no event on the solve's dispatch: lazy copy-stream readers of the step are enqueued
        // at its end (flush_cq); in a graph capture a plain ev_solved record after the solve is
        // the capture's cross-stream edge.  Round 4 carried ev_solved on this packet: ~5 us of
        // idle stream after the solve in every step.)
        // pint_fit_step_apply: the apply at the end of the solve when every instance is solved
        // here on the generated-Fourier path (whose Woodbury Sigma does not read F0 from the
        // table the apply rewrites)
        double* apply_tab = nullptr;
        InstConst* apply_ic = nullptr;
        size_t lds_dyn = fuse_sigma ? std::max(lds_x, lds_s) : lds_x;
        if (ctx->apply_req && Ks == 0 && !side_sigma && !do_sigma) {
            bool ok = true;
            int maxts = 0;
            for (int pi : ctx->upsr) {
                const PsrHost& ph = ctx->psrs[pi];
                ok = ok && cmp && ph.dev.dsplit && ph.dev.vg;
                maxts = std::max(maxts, ph.spec.tstride);
            }
            // the staging region follows each instance's own solve data (lds_x bounds it)
            if (ok && lds_x + apply_tail_lds(maxts) <= 160 * 1024 - 512) {
                apply_tab = ctx->d_tables;
                apply_ic = ctx->d_ic;
                lds_dyn = std::max(lds_dyn, lds_x + apply_tail_lds(maxts));
                ctx->apply_done = true;
                ctx->tables_fresh = false;
            }
        }
        // the build phase (norms, S and U, S -= U U^T, b'_d) spread over the chip by k_schur
        // when the solve exports to xw (deferred solves); PINT_SCHUR=0 keeps it in the solve
        int pre = 0;
        if (xw && ctx->schur) {
            int mnb = 0, mnk = 0;
            for (int pi : ctx->upsr) {
                const PsrDev& pd = ctx->psrs[pi].dev;
                if (!pd.dsplit) continue;
                const int kd = mode == 0 ? pd.red0c : pd.Kd, nbd = (kd + 15) / 16;
                mnb = std::max(mnb, nbd * (nbd + 1) / 2);
                mnk = std::max(mnk, (pd.ndc + 15) / 16);
            }
            if (mnb > 0) {
                hipLaunchKernelGGL(k_schur, dim3(mnb, ctx->ninst), dim3(SCHUR_T), schur_lds(mnk), ctx->stream,
                                   (const PsrDev*)ctx->d_psrs, (const InstDev*)ctx->d_inst, (const double*)ctx->d_G,
                                   (const double*)ctx->d_colsq, ctx->nsplit, mode, (const double*)ctx->d_Sd,
                                   (const double*)ctx->d_DD, (const double*)ctx->d_DCS, xw);
                HIPCHK(hipGetLastError());
                pre = 1;
            }
        }
        // 8 waves (256 VGPRs per lane) when the dense block fits them (nbd <= 8 and, for the
        // fused Woodbury Sigma, nbs <= 9): the 16-wave form's 128-VGPR budget made the
        // diagonal factor spill its pivot columns to SGPRs and sink each column's updates to
        // its pivot, serialising them (a chain of j FMAs before pivot j)
        int mnbd = 0;
        for (int pi : ctx->upsr) {
            const PsrDev& pd = ctx->psrs[pi].dev;
            if (pd.dsplit) mnbd = std::max(mnbd, ((mode == 0 ? pd.red0c : pd.Kd) + 15) / 16);
        }
        const bool w8 = ctx->solve_w8 && mnbd <= 8 && (!fuse_sigma || nbs_sig <= 9);
#define PINT_SOLVE_DMX(NWS)                                                                                          \
        hipExtLaunchKernelGGL((k_solve_dmx<NWS>), dim3(ctx->ninst * (fuse_sigma ? 2 : 1)), dim3(NWS * 64),           \
                              (uint32_t)lds_dyn, ctx->stream, nullptr, nullptr, 0u,                                  \
                              (const PsrDev*)ctx->d_psrs, (const InstDev*)ctx->d_inst, (const double*)ctx->d_tables, \
                              (const double*)ctx->d_G, (const double*)ctx->d_colsq, ctx->nsplit, mode,               \
                              (const double*)ctx->d_Sd, (const double*)ctx->d_DD, (const double*)ctx->d_DCS,         \
                              ctx->d_dpars, ctx->d_errs, ctx->d_cov, ctx->d_chi2lin, ctx->d_sigL, ctx->d_status,     \
                              fuse_sigma, ctx->refine, xw, ones, apply_tab, apply_ic, ctx->apply_lam, pre,           \
                              ctx->la_chol)
        if (w8) PINT_SOLVE_DMX(8); else PINT_SOLVE_DMX(16);
#undef PINT_SOLVE_DMX
        HIPCHK(hipGetLastError());
        ctx->cov_pending = xw != nullptr;
        ctx->cov_mode = mode;
        ctx->cov_lds = lds_x;
    }
    const int nbx = std::max((Ks + 15) / 16, (Kn + 15) / 16);
    if (skip && Ks == 0) {
        // every instance went through k_solve_dmx
    } else if (nbx <= BS_MAXNB && ctx->blocked_solve) {
        const int ldsw = nbx * (nbx + 1) / 2 * 256 + 2 * 16 * nbx;  // doubles per instance
        const int ldsw1 = ldsw + 3 * 16 * nbx;  // (+ the three scratch vectors: one-wave form)
        size_t lds_b = sizeof(double) * (size_t)ldsw;
        // K <= 32 (a grid's points): a wave per instance, four per workgroup -- the 4-wave
        // form spent ~27 us of barriers and idle waves on each such instance
        if (nbx <= 1 && ctx->small && ctx->lane_solve && !skip && Ks <= 8) {
            // K <= 8 (a grid's points): a lane per instance
            const int KT = Ks <= 4 ? 4 : 8;
            if (KT == 4)
                hipLaunchKernelGGL(k_solve_lanes<4>, dim3((ctx->ninst + 63) / 64), dim3(64), 0, ctx->stream, ctx->d_psrs,
                                   ctx->d_inst, ctx->d_G, ctx->d_colsq, ctx->nsplit, mode, ctx->d_dpars, ctx->d_errs,
                                   ctx->d_cov, ctx->d_chi2lin, ctx->d_status, ctx->refine, ctx->ninst);
            else
                hipLaunchKernelGGL(k_solve_lanes<8>, dim3((ctx->ninst + 63) / 64), dim3(64), 0, ctx->stream, ctx->d_psrs,
                                   ctx->d_inst, ctx->d_G, ctx->d_colsq, ctx->nsplit, mode, ctx->d_dpars, ctx->d_errs,
                                   ctx->d_cov, ctx->d_chi2lin, ctx->d_status, ctx->refine, ctx->ninst);
        } else if (nbx <= 2 && ctx->small)
            hipLaunchKernelGGL(k_solve_blk<1>, dim3((ctx->ninst + 3) / 4), dim3(256), 4 * sizeof(double) * ldsw1,
                               ctx->stream, ctx->d_psrs, ctx->d_inst, ctx->d_tables, ctx->d_G, ctx->d_colsq,
                               ctx->nsplit, mode, cmp, ctx->d_Sd, ctx->d_DD, ctx->d_DCS, ctx->d_dpars, ctx->d_errs,
                               ctx->d_cov, ctx->d_chi2lin, ctx->d_sigL, ctx->d_status, skip, ctx->d_rscr, ctx->refine,
                               ctx->ninst, ldsw1);
        else if (nbx <= 5)
            hipLaunchKernelGGL(k_solve_blk<4>, dim3(ctx->ninst), dim3(256), lds_b, ctx->stream, ctx->d_psrs, ctx->d_inst,
                               ctx->d_tables, ctx->d_G, ctx->d_colsq, ctx->nsplit, mode, cmp, ctx->d_Sd, ctx->d_DD,
                               ctx->d_DCS, ctx->d_dpars, ctx->d_errs,
                               ctx->d_cov, ctx->d_chi2lin, ctx->d_sigL, ctx->d_status, skip, ctx->d_rscr, ctx->refine,
                               ctx->ninst, ldsw);
        else
            hipLaunchKernelGGL(k_solve_blk<16>, dim3(ctx->ninst), dim3(1024), lds_b, ctx->stream, ctx->d_psrs, ctx->d_inst,
                               ctx->d_tables, ctx->d_G, ctx->d_colsq, ctx->nsplit, mode, cmp, ctx->d_Sd, ctx->d_DD,
                               ctx->d_DCS, ctx->d_dpars, ctx->d_errs,
                               ctx->d_cov, ctx->d_chi2lin, ctx->d_sigL, ctx->d_status, skip, ctx->d_rscr, ctx->refine,
                               ctx->ninst, ldsw);
    } else {
        int K = ctx->maxK;
        size_t lds_s = sizeof(double) * ((size_t)K * (K + 1) / 2 + 5 * K + 8);
        if (lds_s > 160 * 1024) { ctx->err = "normal matrix too large for LDS solve"; return PINT_E_INVALID; }
        hipLaunchKernelGGL(k_solve, dim3(ctx->ninst), dim3(SOLVE_T), lds_s, ctx->stream, ctx->d_psrs, ctx->d_inst,
                           ctx->d_tables, ctx->d_G, ctx->d_colsq, ctx->nsplit, nparts, mode, cmp, ctx->d_Sd, ctx->d_DD,
                           ctx->d_DCS, ctx->d_work, ctx->d_dpars,
                           ctx->d_errs, ctx->d_cov, ctx->d_chi2lin, ctx->d_sigL, ctx->d_status, skip, do_sigma, ones);
    }
    if (do_sigma && !(nbx > BS_MAXNB || !ctx->blocked_solve)) {
        // Sigma too large for k_sigma but the main solve went to the blocked kernels
        ctx->err = "Woodbury Sigma too large for the LDS factorisation";
        return PINT_E_INVALID;
    }
    HIPCHK(hipGetLastError());
    record(ctx, 8);
    if (ctx->capturing) HIPCHK(hipEventRecord(ctx->ev_solved, ctx->stream));
    if (ctx->lazy) return PINT_OK;
    int rc = check_status(ctx);
    update_timings(ctx);
    return rc;
}

// The SVD path of the fitters (k_eig) on the Gram of the last pint_fit_step: replaces the
// step, errors, covariance and linearised chi2 of every instance; ndeg[i] dropped directions
// of instance i (<= PINT_EIG_MAXDEG), degvec[(i * PINT_EIG_MAXDEG + d) * (K_i) ...] their
// components over the instance's columns (stride degstride >= max K).
int pint_solve_eig(pint_ctx* ctx, int mode, const double* threshold, int32_t* ndeg, double* degvec, int degstride) {
    if (!ctx || ctx->ninst <= 0 || (mode != 0 && mode != 1) || !threshold) return PINT_E_INVALID;
    hipSetDevice(ctx->device);
    if (int rc = flush_cq_now(ctx)) return rc;  // k_eig rewrites the step outputs
    int maxK = 0;
    for (auto& I : ctx->inst) maxK = std::max(maxK, mode == 0 ? ctx->psrs[I.psr].spec.ncol : I.K);
    if (degstride < maxK) { ctx->err = "degstride < columns"; return PINT_E_INVALID; }
    const long wstride = 2L * maxK * maxK;
    if ((size_t)(wstride * ctx->ninst) > ctx->eig_cap) {
        dfree((void*&)ctx->d_eigw);
        HIPCHK(cmalloc((void**)&ctx->d_eigw, sizeof(double) * wstride * ctx->ninst));
        ctx->eig_cap = wstride * ctx->ninst;
        dfree((void*&)ctx->d_ndeg);
        dfree((void*&)ctx->d_degv);
        HIPCHK(cmalloc((void**)&ctx->d_ndeg, sizeof(int) * ctx->ninst));
        HIPCHK(cmalloc((void**)&ctx->d_degv, sizeof(double) * ctx->ninst * PINT_EIG_MAXDEG * (size_t)maxK));
        ctx->degv_cap = maxK;
    }
    if (ctx->degv_cap < maxK) { ctx->err = "eig scratch too small"; return PINT_E_INVALID; }
    const size_t lds = sizeof(double) * (4 * (size_t)maxK + maxK + 2);
    if (ctx->sigma_pending) HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_sigma, 0));
    HIPCHK(h2d(ctx->d_lam, threshold, sizeof(double) * ctx->ninst, ctx->stream, false));
    ctx->cov_pending = false;  // k_eig writes every instance's covariance
    hipLaunchKernelGGL(k_eig, dim3(ctx->ninst), dim3(EIG_T), lds, ctx->stream, ctx->d_psrs, ctx->d_inst, ctx->d_G,
                       ctx->d_colsq, ctx->nsplit, mode, ctx->m_compact, ctx->d_Sd, ctx->d_DD, ctx->d_DCS, ctx->d_lam,
                       ctx->d_eigw, wstride, ctx->d_dpars, ctx->d_errs, ctx->d_cov, ctx->d_chi2lin, ctx->d_ndeg,
                       ctx->d_degv, ctx->degv_cap);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ctx->ev_solved, ctx->stream));
    HIPCHK(d2h(ndeg, ctx->d_ndeg, sizeof(int) * ctx->ninst, ctx->stream));
    std::vector<double> tmp((size_t)ctx->ninst * PINT_EIG_MAXDEG * ctx->degv_cap);
    HIPCHK(d2h(tmp.data(), ctx->d_degv, sizeof(double) * tmp.size(), ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    for (int i = 0; i < ctx->ninst; i++)
        for (int d = 0; d < PINT_EIG_MAXDEG; d++)
            for (int k = 0; k < maxK; k++)
                degvec[((long)i * PINT_EIG_MAXDEG + d) * degstride + k] =
                    tmp[((size_t)i * PINT_EIG_MAXDEG + d) * ctx->degv_cap + k];
    return PINT_OK;
}

int pint_read_step(pint_ctx* ctx, double* dpars, double* errs, double* cov, double* chi2lin) {
    if (!ctx || ctx->ninst <= 0) return PINT_E_INVALID;
    hipSetDevice(ctx->device);
    if (ctx->lazy && !ctx->capturing) {
        // lazy: k_cov_dmx and the copies go on the copy stream at the step's end (flush_cq),
        // overlapped with the next step's kernels; the caller's buffers (pinned:
        // pint_host_alloc) are valid after pint_check() / pint_check_step().  The slot's
        // output buffers and the launch state are taken now.
        const bool cov_run = (cov || errs) && ctx->cov_pending;
        static const int cov_env = getenv("PINT_COV_WG") ? atoi(getenv("PINT_COV_WG")) : 0;
        const int cov_wg = cov_env > 0 ? cov_env : COV_WG;
        const int ninst = ctx->ninst, mode = ctx->cov_mode;
        const size_t lds = ctx->cov_lds;
        const long tc = ctx->tot_c, tcv = ctx->tot_cv;
        double *d_dp = ctx->d_dpars, *d_er = ctx->d_errs, *d_cv = ctx->d_cov, *d_cl = ctx->d_chi2lin;
        const double* d_xw = ctx->d_xw;
        const PsrDev* psrs = ctx->d_psrs;
        const InstDev* insts = ctx->d_inst;
        ctx->cq.push_back([=]() -> int {
            hipStream_t st = ctx->cstream;
            HostLap lap{"read_step op"};
            if (cov_run) {
                hipLaunchKernelGGL(k_cov_dmx<16>, dim3(ninst, cov ? cov_wg : 1), dim3(1024), lds, st, psrs, insts, d_xw,
                                   mode, cov ? d_cv : nullptr, d_er);
                HIPCHK(hipGetLastError());
                lap("k_cov_dmx launch");
            }
            if (int rc = export_seg(ctx, dpars, d_dp, tc)) return rc;
            if (int rc = export_seg(ctx, errs, d_er, tc)) return rc;
            if (int rc = export_seg(ctx, cov, d_cv, tcv)) return rc;
            if (int rc = export_seg(ctx, chi2lin, d_cl, ninst)) return rc;
            lap("segments");
            return PINT_OK;
        });
        if (cov_run) ctx->cov_pending = cov == nullptr;  // errors only: a later read of the covariance re-runs it
        return PINT_OK;
    }
    // synchronous, or inside a graph capture: on the copy stream after ev_solved (capture: the
    // cross-stream edge of the graph), or on the kernel stream
    hipStream_t st = ctx->lazy ? ctx->cstream : ctx->stream;
    if (ctx->lazy) HIPCHK(hipStreamWaitEvent(ctx->cstream, ctx->ev_solved, 0));
    if ((cov || errs) && ctx->cov_pending) {  // the DMX-eliminated solve's W, DMX errors, covariance
        // (round 4: capping it at ~half the CUs, beside the next pipelined step's evaluation,
        // looked 7 % faster in one A/B sweep and not at all in a second -- the 68-pulsar step is
        // bimodal run to run on one box, 0.38 or 0.41 ms; PINT_COV_WG sets a fixed count)
        static const int cov_env = getenv("PINT_COV_WG") ? atoi(getenv("PINT_COV_WG")) : 0;
        const int cov_wg = cov_env > 0 ? cov_env : COV_WG;
        hipLaunchKernelGGL(k_cov_dmx<16>, dim3(ctx->ninst, cov ? cov_wg : 1), dim3(1024), ctx->cov_lds, st,
                           ctx->d_psrs, ctx->d_inst, ctx->d_xw, ctx->cov_mode, cov ? ctx->d_cov : nullptr,
                           ctx->d_errs);
        HIPCHK(hipGetLastError());
        ctx->cov_pending = cov == nullptr;  // errors only: a later read of the covariance re-runs it
    }
    if (dpars) HIPCHK(d2h(dpars, ctx->d_dpars, sizeof(double) * ctx->tot_c, st));
    if (errs) HIPCHK(d2h(errs, ctx->d_errs, sizeof(double) * ctx->tot_c, st));
    if (cov) HIPCHK(d2h(cov, ctx->d_cov, sizeof(double) * ctx->tot_cv, st));
    if (chi2lin) HIPCHK(d2h(chi2lin, ctx->d_chi2lin, sizeof(double) * ctx->ninst, st));
    if (ctx->lazy) {
        HIPCHK(hipEventRecord(ctx->ev_copied, ctx->cstream));
        ctx->copy_pend[ctx->slot] = true;
        return PINT_OK;
    }
    HIPCHK(hipStreamSynchronize(st));
    return PINT_OK;
}

void* pint_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 8, hipHostMallocDefault) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_pinned_mu);
    g_pinned[reinterpret_cast<uintptr_t>(p)] = bytes ? bytes : 8;
    return p;
}

void pint_host_free(void* p) {
    if (!p) return;
    {
        std::lock_guard<std::mutex> lk(g_pinned_mu);
        g_pinned.erase(reinterpret_cast<uintptr_t>(p));
    }
    hipHostFree(p);
}

int pint_apply_step(pint_ctx* ctx, const double* lambda_) {
    if (!ctx || ctx->ninst <= 0 || !lambda_) return PINT_E_INVALID;
    if (flush_restore(ctx)) return PINT_E_HIP;
    if (ctx->sigma_pending) HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_sigma, 0));  // k_sigma reads F0
    HIPCHK(h2d(ctx->d_lam, lambda_, sizeof(double) * ctx->ninst, ctx->stream, false));
    launch_apply(ctx, ctx->d_lam, 0.0);
    HIPCHK(hipGetLastError());
    ctx->ic_valid = true;
    if (!ctx->lazy) HIPCHK(hipStreamSynchronize(ctx->stream));
    return PINT_OK;
}

// The same step with one lambda for every instance (GLSFitter / WLSFitter take the full
// step, fitter.py:2254-2263): a kernel argument, no host->device copy.
int pint_apply_step_uniform(pint_ctx* ctx, double lambda_) {
    if (!ctx || ctx->ninst <= 0) return PINT_E_INVALID;
    if (flush_restore(ctx)) return PINT_E_HIP;
    if (ctx->sigma_pending) HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_sigma, 0));  // k_sigma reads F0
    launch_apply(ctx, nullptr, lambda_);
    HIPCHK(hipGetLastError());
    ctx->ic_valid = true;
    if (!ctx->lazy) HIPCHK(hipStreamSynchronize(ctx->stream));
    return PINT_OK;
}

// A fit step followed by tables += lambda * step (pint_fit_step + pint_apply_step_uniform):
// when every instance takes the DMX-eliminated solve on the generated-Fourier path, the
// apply and the new table's per-instance constants are formed at the end of the solve
// kernel (solve_apply_tail) instead of in a k_apply launch.  The step's outputs (pint_read_step,
// pint_noise_resids) read the step, not the tables, so they may follow.
int pint_fit_step_apply(pint_ctx* ctx, int mode, double lambda_) {
    if (!ctx || ctx->ninst <= 0) return PINT_E_INVALID;
    ctx->apply_req = true;
    ctx->apply_lam = lambda_;
    ctx->apply_done = false;
    const int rc = pint_fit_step(ctx, mode);
    ctx->apply_req = false;
    if (rc != PINT_OK) return rc;
    if (ctx->apply_done) {
        ctx->apply_done = false;
        ctx->ic_valid = true;
        return PINT_OK;
    }
    return pint_apply_step_uniform(ctx, lambda_);
}

// Parameter tables resident on the device: pint_save_tables snapshots the current tables,
// pint_restore_tables puts the snapshot back (a device copy on the stream), e.g. to start
// every fit of a benchmark loop from the same initial models without a host->device upload.
int pint_save_tables(pint_ctx* ctx) {
    if (!ctx || ctx->ninst <= 0) return PINT_E_INVALID;
    if (flush_restore(ctx)) return PINT_E_HIP;
    hipSetDevice(ctx->device);
    if (ctx->tot_table > ctx->tables0_cap) {
        dfree((void*&)ctx->d_tables0);
        HIPCHK(cmalloc((void**)&ctx->d_tables0, sizeof(double) * ctx->tot_table));
        ctx->tables0_cap = ctx->tot_table;
    }
    HIPCHK(hipMemcpyAsync(ctx->d_tables0, ctx->d_tables, sizeof(double) * ctx->tot_table, hipMemcpyDeviceToDevice,
                          ctx->stream));
    // the snapshot's per-instance constants, so a restore needs no k_prep (pint_eval)
    if (!ctx->d_ic0) HIPCHK(cmalloc((void**)&ctx->d_ic0, sizeof(InstConst) * ctx->ninst));
    launch_prep(ctx, ctx->d_tables0, nullptr, ctx->d_ic0);
    HIPCHK(hipGetLastError());
    ctx->ic0_valid = true;
    if (!ctx->lazy) HIPCHK(hipStreamSynchronize(ctx->stream));
    return PINT_OK;
}

int pint_restore_tables(pint_ctx* ctx) {
    if (!ctx || ctx->ninst <= 0 || !ctx->d_tables0 || ctx->tables0_cap < ctx->tot_table) {
        if (ctx) ctx->err = "pint_restore_tables: no snapshot of this batch (pint_save_tables)";
        return PINT_E_INVALID;
    }
    ctx->ic_valid = false;
    ctx->tables_fresh = false;
    if (ctx->sigma_pending) HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_sigma, 0));  // k_sigma reads F0
    // deferred: the next pint_eval's k_prep copies the snapshot back as it forms the
    // per-instance constants (one launch less); every other reader of the tables flushes it
    ctx->restore_pending = true;
    return PINT_OK;
}

static int flush_restore(pint_ctx* ctx) {
    if (!ctx->restore_pending) return PINT_OK;
    ctx->restore_pending = false;
    HIPCHK(hipMemcpyAsync(ctx->d_tables, ctx->d_tables0, sizeof(double) * ctx->tot_table, hipMemcpyDeviceToDevice,
                          ctx->stream));
    return PINT_OK;
}

// Woodbury GLS chi2 of the current residuals; requires a previous pint_fit_step(mode=1)
// (Sigma factor) and the red-noise columns of the last design matrix.
int pint_chi2_gls(pint_ctx* ctx, double* chi2) {
    flush_r2(ctx);
    if (flush_chi2(ctx)) return PINT_E_HIP;
    int R = 0;
    for (int pi : ctx->upsr) R = 2 * ctx->psrs[pi].spec.nred > R ? 2 * ctx->psrs[pi].spec.nred : R;
    int stride = R + 2;
    int nsw = ctx->nsplit;  // same N-split as the Gram (fills the CUs)
    if (ctx->wtile_valid) {  // the residual pass formed the dots (k_resid2 tiles -> k_rsum)
        nsw = 1;
        stride = ctx->wstride;
    }
    size_t need = (size_t)ctx->ninst * nsw * stride;
    if (need > ctx->wpart_cap) {
        if (ctx->capturing) { ctx->err = "pint_chi2_gls: first call inside a graph capture"; return PINT_E_INVALID; }
        dfree((void*&)ctx->d_wpart);
        HIPCHK(cmalloc((void**)&ctx->d_wpart, sizeof(double) * need));
        ctx->wpart_cap = need;
    }
    record(ctx, 10);
    if (ctx->sigma_pending) HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_sigma, 0));
    if (!ctx->wtile_valid) {
        hipLaunchKernelGGL(k_wdot, dim3(nsw, ctx->ninst), dim3(256), 0, ctx->stream, ctx->d_psrs, ctx->d_inst, ctx->d_M,
                           ctx->d_rt, nsw, stride, ctx->m_compact, ctx->d_wpart);
        HIPCHK(hipGetLastError());
    }
    hipLaunchKernelGGL(k_wsolve, dim3(ctx->ninst), dim3(256), sizeof(double) * ((R + 1) + (R + 1) * (R + 2) / 2),
                       ctx->stream, ctx->d_psrs,
                       ctx->d_inst, ctx->d_rt, ctx->d_sigL, ctx->d_esum, ctx->d_eD, ctx->d_eW, ctx->d_wpart, nsw,
                       stride, ctx->d_ecs, ctx->d_chi2g, ctx->d_lognorm,
                       ctx->wtile_valid ? (const double*)ctx->d_wtile : nullptr, (const double*)ctx->d_rpart,
                       ctx->d_chi2, ctx->m_compact);
    HIPCHK(hipGetLastError());
    if (ctx->wtile_valid) ctx->chi2_pending = false;  // k_wsolve stored the residuals' chi2
    record(ctx, 11);
    if (ctx->lazy && !ctx->capturing) {
        // the copy is deferred to pint_step_end (the copy stream, after the step's end event:
        // no event of its own on the kernel stream) or pint_check; valid after either
        ctx->chi2_dst = chi2;
        return PINT_OK;
    }
    HIPCHK(d2h(chi2, ctx->d_chi2g, sizeof(double) * ctx->ninst, ctx->stream));
    if (!ctx->lazy) HIPCHK(hipStreamSynchronize(ctx->stream));
    return PINT_OK;
}

// WLS chi2 of the current residuals, per instance (k_chi2w); the chi2 that pint_read_resids
// reports comes from the residual pass itself, this one from whatever d_rt holds now.
int pint_chi2_wls(pint_ctx* ctx, double* chi2) {
    if (!ctx || ctx->ninst <= 0 || !chi2) return PINT_E_INVALID;
    flush_r2(ctx);
    if (flush_chi2(ctx)) return PINT_E_HIP;
    hipSetDevice(ctx->device);
    hipLaunchKernelGGL(k_chi2w, dim3(ctx->ninst), dim3(256), 0, ctx->stream, ctx->d_psrs, ctx->d_inst, ctx->d_rt,
                       ctx->d_chi2g);
    HIPCHK(hipGetLastError());
    HIPCHK(d2h(chi2, ctx->d_chi2g, sizeof(double) * ctx->ninst, ctx->stream));
    if (!ctx->lazy) HIPCHK(hipStreamSynchronize(ctx->stream));
    return PINT_OK;
}

// Lazy mode: launches return without synchronising; pint_check() syncs, reads the device
// status word and the event timings.
int pint_set_lazy(pint_ctx* ctx, int lazy) {
    ctx->lazy = lazy;
    return PINT_OK;
}

int pint_set_option(pint_ctx* ctx, int key, int value) {
    if (!ctx) return PINT_E_INVALID;
    if (key == PINT_OPT_BLOCKED_SOLVE) { ctx->blocked_solve = value ? 1 : 0; return PINT_OK; }
    if (key == PINT_OPT_VGRAM) { ctx->vgram = value ? 1 : 0; return PINT_OK; }
    if (key == PINT_OPT_VBIN) { ctx->vbin = value ? 1 : 0; return PINT_OK; }
    if (key == PINT_OPT_WBFIT) { ctx->wbfit = value ? 1 : 0; return PINT_OK; }
    if (key == PINT_OPT_COV_DEFER) {
        if (value < 0 || value > 2) return PINT_E_INVALID;
        ctx->cov_defer = value;
        return PINT_OK;
    }
    if (key == PINT_OPT_REFINE) { ctx->refine = value ? 1 : 0; return PINT_OK; }
    if (key == PINT_OPT_SCHUR) { ctx->schur = value ? 1 : 0; return PINT_OK; }
    if (key == PINT_OPT_SMALL) { ctx->small = value ? 1 : 0; return PINT_OK; }
    if (key == PINT_OPT_LA_CHOL) { ctx->la_chol = value ? 1 : 0; return PINT_OK; }
    if (key == PINT_OPT_SOLVE_W8) { ctx->solve_w8 = value ? 1 : 0; return PINT_OK; }
    if (key == PINT_OPT_EFUSE) { ctx->efuse = value ? 1 : 0; return PINT_OK; }
    if (key == PINT_OPT_LANE_SOLVE) { ctx->lane_solve = value ? 1 : 0; return PINT_OK; }
    if (key == PINT_OPT_SPIN_EVAL) { ctx->spin_eval = value ? 1 : 0; return PINT_OK; }
    if (key == PINT_OPT_TIMING_EVERY) {
        if (value < 1) return PINT_E_INVALID;
        ctx->timing_every = value;
        ctx->gram_calls = 0;
        return PINT_OK;
    }
    if (key == 99) { ctx->gvdbg = value; return PINT_OK; }
    if (key == PINT_OPT_TIMING_MASK) {
        ctx->timing_mask = value & 0xff;
        for (int sl = 0; sl < pint_ctx::NSLOT; sl++)
            for (int k = 0; k < pint_ctx::NEV; k++) ctx->rec_slot[sl][k] = false;
        for (int k = 0; k < pint_ctx::NMS; k++) ctx->ms[k] = 0.0f;
        return PINT_OK;
    }
    ctx->err = "unknown option";
    return PINT_E_INVALID;
}

// Stream capture of a launch sequence into a HIP graph (lazy mode): everything the calls
// between pint_capture_begin and pint_capture_end enqueue -- kernels, copies to/from the
// caller's pinned buffers, the side-stream kernels and copies -- becomes one graph that
// pint_graph_launch replays with a single launch.  Device buffers and host pointers are
// frozen at capture: replays re-run the same batch on whatever the buffers hold.
static void join_side_streams(pint_ctx* ctx) {
    if (ctx->sigma_pending) hipStreamWaitEvent(ctx->stream, ctx->ev_sigma, 0);
    if (any_copy_pend(ctx)) hipStreamWaitEvent(ctx->stream, ctx->ev_copied, 0);
    ctx->sigma_pending = false;
    clear_copy_pend(ctx);
}

int pint_capture_begin(pint_ctx* ctx) {
    if (!ctx || ctx->ninst <= 0 || ctx->capturing) return PINT_E_INVALID;
    if (!ctx->lazy) { ctx->err = "graph capture needs lazy mode"; return PINT_E_INVALID; }
    hipSetDevice(ctx->device);
    if (int rc = flush_cq_now(ctx)) return rc;
    HIPCHK(hipStreamSynchronize(ctx->cstream));
    HIPCHK(hipStreamSynchronize(ctx->sstream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->sigma_pending = false;
    clear_copy_pend(ctx);
    HIPCHK(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeRelaxed));
    ctx->capturing = true;
    return PINT_OK;
}

int pint_capture_end(pint_ctx* ctx) {
    if (!ctx || !ctx->capturing) return PINT_E_INVALID;
    join_side_streams(ctx);
    ctx->capturing = false;
    hipGraph_t g = nullptr;
    HIPCHK(hipStreamEndCapture(ctx->stream, &g));
    const int s = ctx->slot;  // the graph writes this slot's outputs, status word and pinned buffers
    if (ctx->graph_exec_s[s]) hipGraphExecDestroy(ctx->graph_exec_s[s]);
    if (ctx->graph_s[s]) hipGraphDestroy(ctx->graph_s[s]);
    ctx->graph_s[s] = g;
    ctx->graph_exec_s[s] = nullptr;
    HIPCHK(hipGraphInstantiate(&ctx->graph_exec_s[s], g, nullptr, nullptr, 0));
    return PINT_OK;
}

int pint_graph_launch(pint_ctx* ctx) {
    if (!ctx || !ctx->graph_exec_s[ctx->slot]) {
        if (ctx) ctx->err = "pint_graph_launch: no graph captured for this pipeline slot";
        return PINT_E_INVALID;
    }
    hipSetDevice(ctx->device);
    join_side_streams(ctx);
    HIPCHK(hipGraphLaunch(ctx->graph_exec_s[ctx->slot], ctx->stream));
    return PINT_OK;
}

// Likelihood normalisation per instance (Residuals.calc_chi2(lognorm=True)): gls == 1 the
// logdet(C)/2 of the last pint_chi2_gls; gls == 2 a correlated-noise model whose basis has
// no columns (C = N + 1e40 1 1^T: logdet C = logdet N + log 1e40 + log(1e-40 + sum w));
// gls == 0 sum log sigma (residuals.py:638-667).
int pint_lognorm(pint_ctx* ctx, int gls, double* out) {
    if (!ctx || ctx->ninst <= 0 || !out) return PINT_E_INVALID;
    if (gls == 2) {
        for (int k = 0; k < ctx->ninst; k++) {
            const PsrDev& d = ctx->psrs[ctx->inst[k].psr].dev;
            out[k] = ctx->psrs[ctx->inst[k].psr].spec.wb_noones
                         ? d.logsig
                         : 0.5 * (2.0 * d.logsig + std::log(1e40) + std::log(1e-40 + d.sumw));
        }
    } else if (gls) {
        HIPCHK(d2h(out, ctx->d_lognorm, sizeof(double) * ctx->ninst, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
    } else {
        for (int k = 0; k < ctx->ninst; k++) out[k] = ctx->psrs[ctx->inst[k].psr].dev.logsig;
    }
    return PINT_OK;
}

int pint_query(pint_ctx* ctx, int key) {
    if (!ctx) return -PINT_E_INVALID;
    if (key == PINT_QUERY_NVGRAM) return ctx->n_vg;
    if (key == PINT_QUERY_NSPLIT) return ctx->nsplit;
    ctx->err = "unknown query";
    return -PINT_E_INVALID;
}

int pint_check(pint_ctx* ctx) {
    int rc = check_status(ctx);
    update_timings(ctx);
    return rc;
}

// Pipelined steps: pint_step_end closes the work enqueued since the previous step_end (the
// side streams joined, the step's deferred copy-stream work enqueued behind its last kernel,
// the status word copied to its pinned mirror, an end event) and moves the launches that
// follow to the next slot; pint_check_step(s) waits for step s only, so the host enqueues
// steps k+1 .. k+NSLOT-1 while the device still runs step k.  NSLOT steps in flight at most:
// the caller checks step s before ending the step that reuses its slot.
int pint_step_end(pint_ctx* ctx, int* slot) {
    if (!ctx || ctx->capturing || !slot) return PINT_E_INVALID;
    hipSetDevice(ctx->device);
    // the output copies of this step stay on the copy stream, overlapped with the next
    // step's evaluation and Gram: the next solve waits for them (copy_pending), and the
    // step's completion covers them through ev_cdone
    if (ctx->sigma_pending) HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_sigma, 0));
    ctx->sigma_pending = false;
    const int s = ctx->slot;
    // the step's kernels end at ev_done; its status word goes to the host on the copy stream
    // after them (off the kernel stream), and ev_cdone covers it and the step's output copies
    HostLap lap{"step_end"};
    HIPCHK(hipEventRecord(ctx->ev_done[s], ctx->stream));
    lap("record ev_done");
    // the step's deferred copy-stream work behind its last kernel, its host-bound outputs --
    // with the chi2 of pint_chi2_gls and the slot's status word -- in one k_export
    if (ctx->chi2_dst) {
        if (int rc = export_seg(ctx, ctx->chi2_dst, ctx->d_chi2g, ctx->ninst)) return rc;
        ctx->chi2_dst = nullptr;
    }
    bool st_exp = false;
    {
        void* sd = nullptr;
        if (hipHostGetDevicePointer(&sd, ctx->h_status + s, 0) == hipSuccess && sd) {
            ctx->exp_st_src = ctx->d_status_slots + s;
            ctx->exp_st_dst = static_cast<int*>(sd);
            st_exp = true;
        } else {
            (void)hipGetLastError();
        }
    }
    if (int rc = flush_cq(ctx, ctx->ev_done[s])) return rc;
    lap("flush");
    if (!st_exp)  // (no device-visible address of the status mirror: a runtime copy)
        HIPCHK(d2h(ctx->h_status + s, ctx->d_status_slots + s, sizeof(int), ctx->cstream));
    HIPCHK(hipEventRecord(ctx->ev_cdone[s], ctx->cstream));
    lap("record ev_cdone");
    ctx->cdone_rec[s] = true;
    ctx->slot = (s + 1) % pint_ctx::NSLOT;
    ctx->d_status = ctx->d_status_slots + ctx->slot;
    ctx->ev = ctx->ev_slot[ctx->slot];
    ctx->rec = ctx->rec_slot[ctx->slot];
    select_out_slot(ctx, ctx->slot);  // the next step's fit outputs (read them before step_end)
    // (the new slot's event flags still belong to its previous step, which the caller checks
    // next: pint_check_step reads and clears them)
    *slot = s;
    return PINT_OK;
}

// One GLSFitter.fit_toas(maxiter=1) step of every instance (fitter.py:2164-2289), enqueued by
// one call: [the snapshot restored], the evaluation with the fit layout, the GLS step with the
// full step applied (fused into the solve where possible), the step outputs and the noise
// realisations on the copy stream, the post-fit evaluation and Woodbury chi2, then the step
// closed (pint_step_end).  The same launches as the separate calls, without a host round trip
// per call; lazy mode only (the outputs are complete after pint_check_step(*slot)).
int pint_fit_step_enqueue(pint_ctx* ctx, int restore, int mode, double lambda_, double* dpars, double* errs,
                          double* cov, double* chi2lin, double* noise_red, double* noise_ecorr, double* noise_dm,
                          double* chi2, int* slot) {
    if (!ctx || ctx->ninst <= 0 || !slot) return PINT_E_INVALID;
    if (!ctx->lazy || ctx->capturing) { ctx->err = "pint_fit_step_enqueue needs lazy mode (no capture)"; return PINT_E_INVALID; }
    if (mode != 1) { ctx->err = "pint_fit_step_enqueue: GLS steps (mode 1) only"; return PINT_E_INVALID; }
    int rc = PINT_OK;
    // PINT_TRACE_ENQ=1: the host time of each enqueue stage (a stall > 1 ms is printed)
    static const bool tr = getenv("PINT_TRACE_ENQ") && atoi(getenv("PINT_TRACE_ENQ"));
    static long ncall = 0;
    ncall++;
    auto t_prev = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!tr) return;
        const auto t = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(t - t_prev).count();
        if (ms > 1.0) fprintf(stderr, "[pint enqueue %ld] %s took %.3f ms\n", ncall, what, ms);
        t_prev = t;
    };
    if (restore && (rc = pint_restore_tables(ctx))) return rc;
    lap("restore");
    if ((rc = pint_eval(ctx, 2))) return rc;
    lap("eval(M)");
    if ((rc = pint_fit_step_apply(ctx, mode, lambda_))) return rc;
    lap("fit_step_apply");
    if ((dpars || errs || cov || chi2lin) && (rc = pint_read_step(ctx, dpars, errs, cov, chi2lin))) return rc;
    lap("read_step");
    if ((noise_red || noise_ecorr) && (rc = pint_noise_resids(ctx, noise_red, noise_ecorr))) return rc;
    if (noise_dm && (rc = pint_noise_resids_dm(ctx, noise_dm))) return rc;
    lap("noise");
    if ((rc = pint_eval(ctx, 0))) return rc;
    lap("eval");
    if (chi2 && (rc = pint_chi2_gls(ctx, chi2))) return rc;
    lap("chi2_gls");
    rc = pint_step_end(ctx, slot);
    lap("step_end");
    return rc;
}

int pint_check_step(pint_ctx* ctx, int s) {
    if (!ctx || s < 0 || s >= pint_ctx::NSLOT) return PINT_E_INVALID;
    hipSetDevice(ctx->device);
    HIPCHK(hipEventSynchronize(ctx->ev_done[s]));
    if (ctx->cdone_rec[s]) HIPCHK(hipEventSynchronize(ctx->ev_cdone[s]));
    ctx->cdone_rec[s] = false;
    ctx->copy_pend[s] = false;  // its output copies are complete
    const int st = ctx->h_status[s];
    if (st) {
        ctx->h_status[s] = 0;
        HIPCHK(hipMemsetAsync(ctx->d_status_slots + s, 0, sizeof(int), ctx->stream));
    }
    hipEvent_t* ev = ctx->ev;
    bool* rec = ctx->rec;
    ctx->ev = ctx->ev_slot[s];
    ctx->rec = ctx->rec_slot[s];
    update_timings(ctx, true);  // this step's timings (0 where it recorded none)
    for (int k = 0; k < pint_ctx::NEV; k++) ctx->rec[k] = false;
    ctx->ev = ev;
    ctx->rec = rec;
    return decode_status(ctx, st);
}

int pint_last_timing(pint_ctx* ctx, double* ms) {
    update_timings(ctx);
    for (int k = 0; k < pint_ctx::NMS; k++) ms[k] = ctx->ms[k];
    return PINT_OK;
}

// debug/introspection: which 0 = Gram partials (sum over splits done by caller),
// 1 = column sums of squares, 2 = Woodbury Sigma factor, 3 = L^-1 work
int pint_debug_read(pint_ctx* ctx, int which, double* out) {
    HIPCHK(hipStreamSynchronize(ctx->sstream));
    if (which == 5) {  // (experiment) k_gram_v per-workgroup timestamps
        static unsigned long long t[4096 * 5];
        HIPCHK(hipStreamSynchronize(ctx->stream));
        HIPCHK(hipMemcpyFromSymbol(t, HIP_SYMBOL(g_gvts), sizeof(t)));
        for (int i = 0; i < 4096 * 5; i++) out[i] = (double)t[i];
        return 4096;
    }
    if (which == 4) {  // phase timestamps (us) of k_solve_dmx workgroup 0
        unsigned long long ts[32];
        HIPCHK(hipStreamSynchronize(ctx->stream));
        HIPCHK(hipMemcpyFromSymbol(ts, HIP_SYMBOL(g_ts), sizeof(ts)));
        // (signed: a stamp this launch did not write -- zero after a reset (which 6), or stale --
        // comes out negative or beyond the end stamp instead of as an unsigned wrap-around)
        for (int i = 0; i < 32; i++) out[i] = (double)(long long)(ts[i] - ts[0]) * 0.01;
        return 32;
    }
    if (which == 7) {  // the per-workgroup timeline (WgTimer), raw 100 MHz ticks
        static unsigned long long t[WGT_K * WGT_B * 2];
        HIPCHK(hipStreamSynchronize(ctx->stream));
        HIPCHK(hipMemcpyFromSymbol(t, HIP_SYMBOL(g_wgt), sizeof(t)));
        for (int i = 0; i < WGT_K * WGT_B * 2; i++) out[i] = (double)t[i];
        return WGT_K * WGT_B * 2;
    }
    if (which == 9) {  // the evaluation blocks' phase stamps (g_wgp), raw 100 MHz ticks
        static unsigned long long t[WGT_B * 2];
        HIPCHK(hipStreamSynchronize(ctx->stream));
        HIPCHK(hipMemcpyFromSymbol(t, HIP_SYMBOL(g_wgp), sizeof(t)));
        for (int i = 0; i < WGT_B * 2; i++) out[i] = (double)t[i];
        return WGT_B * 2;
    }
    if (which == 8) {  // the timeline on (out[0] != 0) or off, cleared
        static unsigned long long z[WGT_K * WGT_B * 2];
        HIPCHK(hipStreamSynchronize(ctx->stream));
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_wgt), z, sizeof(z)));
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_wgp), z, sizeof(unsigned long long) * WGT_B * 2));
        const int on = out && out[0] != 0.0 ? 1 : 0;
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_wgt_on), &on, sizeof(on)));
        HIPCHK(hipDeviceSynchronize());
        return on;
    }
    if (which == 6) {  // reset the phase timestamps (before a probed launch)
        unsigned long long z[32] = {0};
        HIPCHK(hipStreamSynchronize(ctx->stream));
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_ts), z, sizeof(z)));
        return 32;
    }
    size_t n = which == 0 ? ctx->tot_g : which == 1 ? ctx->tot_c * ctx->nsplit : ctx->tot_s;
    double* src = which == 0 ? ctx->d_G : which == 1 ? ctx->d_colsq : which == 2 ? ctx->d_sigL : ctx->d_work;
    HIPCHK(d2h(out, src, sizeof(double) * n, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return ctx->nsplit;
}

// Per-instance status bits (1 << PINT_E_*) raised by the evaluations since the last call,
// one int per instance of the batch; reading clears them.  The batch status word still
// reports the first error of any instance; this tells the host which instances raised it
// (fitter.py:926-935 InvalidModelParameters is per fit, gridutils.py:89-106 NaN per point).
int pint_inst_status(pint_ctx* ctx, int32_t* out) {
    if (!ctx || ctx->ninst <= 0 || !out) return PINT_E_INVALID;
    hipSetDevice(ctx->device);
    HIPCHK(d2h(out, ctx->d_istatus, sizeof(int) * ctx->ninst, ctx->stream));
    HIPCHK(hipMemsetAsync(ctx->d_istatus, 0, sizeof(int) * ctx->ninst, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PINT_OK;
}

// Noise realisations of the last pint_fit_step(mode=1): red[n_i], ecorr[n_i] per instance
// (either pointer may be NULL).  The kernels run on the main stream right after the solve
// (they read its dpars and ECORR epoch sums) into a device buffer kept by the context.
// Lazy mode (GLSFitter.fit_toas's noise_resids inside a pipelined step): the device->host
// copies go to the copy stream after them, into the caller's pinned buffers, valid after
// pint_check / pint_check_step; the next solve waits for them (copy_pending).
int pint_noise_resids(pint_ctx* ctx, double* red, double* ecorr) {
    if (!ctx || ctx->ninst <= 0) return PINT_E_INVALID;
    hipSetDevice(ctx->device);
    const long need = 3 * std::max<long>(1, ctx->tot_out);  // red, ECORR, DM noise
    if (need > ctx->noise_cap) {
        if (ctx->capturing) { ctx->err = "pint_noise_resids: first call inside a graph capture"; return PINT_E_INVALID; }
        dfree((void*&)ctx->d_noise);
        HIPCHK(cmalloc((void**)&ctx->d_noise, sizeof(double) * need));
        ctx->noise_cap = need;
    }
    double* dr = ctx->d_noise;
    double* de = ctx->d_noise + std::max<long>(1, ctx->tot_out);
    int maxn = 1;
    for (auto& I : ctx->inst) maxn = std::max(maxn, I.n);
    // lazy: the kernels and the copies run on the copy stream at the step's end (flush_cq; in
    // a graph capture after ev_solved): they read dpars and the ECORR epoch sums, which the
    // next fit step overwrites only after waiting for ev_copied
    if (ctx->lazy && !ctx->capturing) {
        const int ninst = ctx->ninst, maxep = ctx->max_nep, cmp = ctx->m_compact;
        const long tot = ctx->tot_out;
        const double* d_dp = ctx->d_dpars;
        const PsrDev* psrs = ctx->d_psrs;
        const InstDev* insts = ctx->d_inst;
        double *d_es = ctx->d_esum, *d_eD = ctx->d_eD, *d_eC = ctx->d_eC, *d_df = ctx->d_dfac;
        ctx->cq.push_back([=]() -> int {
            hipStream_t st = ctx->cstream;
            HostLap lap{"noise op"};
            if (red)
                hipLaunchKernelGGL(k_noise_red, dim3((maxn + 255) / 256, ninst), dim3(256), 0, st, psrs, insts, d_dp, dr, 0,
                                   d_df);
            if (ecorr) {
                HIPCHK(hipMemsetAsync(de, 0, sizeof(double) * tot, st));
                if (maxep > 0)
                    hipLaunchKernelGGL(k_noise_ecorr, dim3(maxep, ninst), dim3(64), 0, st, psrs, insts, d_dp, d_es, d_eD,
                                       de, cmp, d_eC);
            }
            HIPCHK(hipGetLastError());
            lap("kernels");
            if (red)
                if (int rc = export_seg(ctx, red, dr, tot)) return rc;
            if (ecorr)
                if (int rc = export_seg(ctx, ecorr, de, tot)) return rc;
            return PINT_OK;
        });
        return PINT_OK;
    }
    hipStream_t st = ctx->stream;
    if (ctx->lazy) {
        st = ctx->cstream;
        HIPCHK(hipStreamWaitEvent(st, ctx->ev_solved, 0));
    }
    if (red)
        hipLaunchKernelGGL(k_noise_red, dim3((maxn + 255) / 256, ctx->ninst), dim3(256), 0, st, ctx->d_psrs,
                           ctx->d_inst, ctx->d_dpars, dr, 0, ctx->d_dfac);
    if (ecorr) {
        HIPCHK(hipMemsetAsync(de, 0, sizeof(double) * ctx->tot_out, st));
        if (ctx->max_nep > 0)
            hipLaunchKernelGGL(k_noise_ecorr, dim3(ctx->max_nep, ctx->ninst), dim3(64), 0, st, ctx->d_psrs,
                               ctx->d_inst, ctx->d_dpars, ctx->d_esum, ctx->d_eD, de, ctx->m_compact, ctx->d_eC);
    }
    if (hipGetLastError() != hipSuccess) { ctx->err = "pint_noise_resids: launch failed"; return PINT_E_HIP; }
    if (red) HIPCHK(d2h(red, dr, sizeof(double) * ctx->tot_out, st));
    if (ecorr) HIPCHK(d2h(ecorr, de, sizeof(double) * ctx->tot_out, st));
    if (ctx->lazy) {
        HIPCHK(hipEventRecord(ctx->ev_copied, ctx->cstream));
        ctx->copy_pend[ctx->slot] = true;
        return PINT_OK;
    }
    HIPCHK(hipStreamSynchronize(st));
    return PINT_OK;
}

int pint_noise_resids_dm(pint_ctx* ctx, double* dm) {
    if (!ctx || ctx->ninst <= 0 || !dm) return PINT_E_INVALID;
    hipSetDevice(ctx->device);
    const long need = 3 * std::max<long>(1, ctx->tot_out);
    if (need > ctx->noise_cap) {
        if (ctx->capturing) { ctx->err = "pint_noise_resids_dm: first call inside a graph capture"; return PINT_E_INVALID; }
        dfree((void*&)ctx->d_noise);
        HIPCHK(cmalloc((void**)&ctx->d_noise, sizeof(double) * need));
        ctx->noise_cap = need;
    }
    double* d = ctx->d_noise + 2 * std::max<long>(1, ctx->tot_out);
    int maxn = 1;
    for (auto& I : ctx->inst) maxn = std::max(maxn, I.n);
    // lazy: on the copy stream at the step's end, like pint_noise_resids; the next evaluation
    // with M (which rewrites the per-TOA DM-noise scale d_dfac) waits for it
    if (ctx->lazy && !ctx->capturing) {
        const int ninst = ctx->ninst;
        const long tot = ctx->tot_out;
        const double* d_dp = ctx->d_dpars;
        const PsrDev* psrs = ctx->d_psrs;
        const InstDev* insts = ctx->d_inst;
        double* d_df = ctx->d_dfac;
        ctx->cq.push_back([=]() -> int {
            hipStream_t st = ctx->cstream;
            hipLaunchKernelGGL(k_noise_red, dim3((maxn + 255) / 256, ninst), dim3(256), 0, st, psrs, insts, d_dp, d, 1, d_df);
            HIPCHK(hipGetLastError());
            return export_seg(ctx, dm, d, tot);
        });
        ctx->dm_noise_pend = true;
        return PINT_OK;
    }
    hipStream_t st = ctx->stream;
    if (ctx->lazy) {
        st = ctx->cstream;
        HIPCHK(hipStreamWaitEvent(st, ctx->ev_solved, 0));
    }
    hipLaunchKernelGGL(k_noise_red, dim3((maxn + 255) / 256, ctx->ninst), dim3(256), 0, st, ctx->d_psrs,
                       ctx->d_inst, ctx->d_dpars, d, 1, ctx->d_dfac);
    if (hipGetLastError() != hipSuccess) { ctx->err = "pint_noise_resids_dm: launch failed"; return PINT_E_HIP; }
    HIPCHK(d2h(dm, d, sizeof(double) * ctx->tot_out, st));
    if (ctx->lazy) {
        HIPCHK(hipEventRecord(ctx->ev_copied, ctx->cstream));
        ctx->copy_pend[ctx->slot] = true;
        ctx->dm_noise_pend = true;
        return PINT_OK;
    }
    HIPCHK(hipStreamSynchronize(st));
    return PINT_OK;
}

// Parity introspection: the assembled normal matrix of the last pint_fit_step (see
// k_debug_gram); out holds (K_i+1)^2 + K_i doubles per instance, concatenated.
// The normalisation of the last pint_fit_step's design matrix (k_norms): per instance K
// values at the instance's K+1-stride offset (read_step's layout), squared column norms.
int pint_read_norms(pint_ctx* ctx, int mode, double* out) {
    if (!ctx || ctx->ninst <= 0 || !out || (mode != 0 && mode != 1)) return PINT_E_INVALID;
    if (ctx->lazy) { ctx->err = "pint_read_norms is synchronous (lazy mode is on)"; return PINT_E_INVALID; }
    hipSetDevice(ctx->device);
    hipLaunchKernelGGL(k_norms, dim3(ctx->ninst), dim3(64), 0, ctx->stream, ctx->d_psrs, ctx->d_inst, ctx->d_G,
                       ctx->d_colsq, ctx->nsplit, ctx->m_compact, ctx->d_Sd, ctx->d_DD, ctx->d_DCS, mode, ctx->d_norms);
    HIPCHK(hipGetLastError());
    HIPCHK(d2h(out, ctx->d_norms, sizeof(double) * ctx->tot_c, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PINT_OK;
}

int pint_debug_gram(pint_ctx* ctx, int pre_ecorr, double* out) {
    if (!ctx || ctx->ninst <= 0 || !out) return PINT_E_INVALID;
    hipSetDevice(ctx->device);
    std::vector<long> off(ctx->ninst + 1, 0);
    for (int k = 0; k < ctx->ninst; k++) {
        const long W = ctx->inst[k].K + 1;
        off[k + 1] = off[k] + W * W + ctx->inst[k].K;
    }
    double* d = nullptr;
    long* doff = nullptr;
    HIPCHK(hipStreamSynchronize(ctx->sstream));
    HIPCHK(hipMalloc(&d, sizeof(double) * off[ctx->ninst]));
    HIPCHK(hipMalloc(&doff, sizeof(long) * ctx->ninst));
    HIPCHK(h2d(doff, off.data(), sizeof(long) * ctx->ninst, nullptr, true));
    hipLaunchKernelGGL(k_debug_gram, dim3(ctx->ninst), dim3(256), 0, ctx->stream, ctx->d_psrs, ctx->d_inst, ctx->d_G,
                       ctx->d_colsq, ctx->nsplit, ctx->m_compact, ctx->d_Sd, ctx->d_DD, ctx->d_DCS, ctx->d_esum,
                       ctx->d_eD, pre_ecorr && ctx->max_nep > 0, doff, d, ctx->d_eC);
    HIPCHK(hipGetLastError());
    HIPCHK(d2h(out, d, sizeof(double) * off[ctx->ninst], ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    hipFree(d);
    hipFree(doff);
    return PINT_OK;
}

// Parity introspection: replace the time residuals of every instance (n_i each) by the
// caller's, e.g. the reference's own residual arrays, so that pint_fit_step / pint_chi2_gls
// run on them (SURVEY.md 8(a) stage-wise parity).
int pint_debug_set_resids(pint_ctx* ctx, const double* time_resid) {
    if (!ctx || ctx->ninst <= 0 || !time_resid) return PINT_E_INVALID;
    flush_r2(ctx);  // (its rpart partials and phases first; the time residuals are replaced below)
    hipSetDevice(ctx->device);
    HIPCHK(h2d(ctx->d_rt, time_resid, sizeof(double) * ctx->tot_out, ctx->stream, false));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->wtile_valid = false;  // the fused Woodbury dots were those of the replaced residuals
    return PINT_OK;
}

int pint_set_resids(pint_ctx* ctx, const double* time_resid) { return pint_debug_set_resids(ctx, time_resid); }

// Replace the scaled TOA uncertainties (s) of pulsar psr in place: the weights of later
// Gram / Woodbury / likelihood evaluations (a noise-parameter fit's trial EFAC/EQUAD,
// fitter.py:1242-1247); the residuals on the device are left as they are.
int pint_set_sigma(pint_ctx* ctx, int psr, const double* sigma_s) {
    if (!ctx || psr < 0 || psr >= (int)ctx->psrs.size() || !sigma_s) return PINT_E_INVALID;
    hipSetDevice(ctx->device);
    if (int rc_ = commit_uploads(ctx)) return rc_;  // (staged pulsar uploads first)
    ctx->wtile_valid = false;  // new weights: the fused Woodbury dots are stale
    PsrHost& ph = ctx->psrs[psr];
    const int n = ph.n;
    std::vector<double> is(n);
    double ls = 0.0, sw = 0.0;
    for (int i = 0; i < n; i++) {
        if (!(sigma_s[i] > 0.0)) { ctx->err = "TOA uncertainty must be > 0"; return PINT_E_INVALID; }
        is[i] = 1.0 / sigma_s[i];
        ls += std::log(sigma_s[i]);
        sw += is[i] * is[i];
    }
    HIPCHK(hipStreamSynchronize(ctx->sstream));
    HIPCHK(h2d((void*)ph.dev.sigma, sigma_s, sizeof(double) * n, ctx->stream, false));
    HIPCHK(h2d((void*)ph.dev.isig, is.data(), sizeof(double) * n, ctx->stream, false));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (ph.spec.nred > 0 && form_trigw(ctx, ph)) return PINT_E_HIP;  // the F^T W F sums of the new weights
    ph.dev.logsig = ls;
    ph.dev.sumw = sw;
    return refresh_psrs(ctx) ? PINT_E_HIP : PINT_OK;
}

// Replace the noise-basis prior variances of pulsar psr in place: red_phi (2 nred, the
// PLRedNoise weights, s^2) and/or ep_phi (nep ECORR variances, s^2); either may be NULL.
int pint_set_noise_weights(pint_ctx* ctx, int psr, const double* red_phi, const double* ep_phi) {
    if (!ctx || psr < 0 || psr >= (int)ctx->psrs.size()) return PINT_E_INVALID;
    hipSetDevice(ctx->device);
    if (int rc_ = commit_uploads(ctx)) return rc_;  // (staged pulsar uploads first)
    PsrHost& ph = ctx->psrs[psr];
    const int nred = ph.spec.nred, nep = ph.dev.nep;
    if (red_phi)
        for (int k = 0; k < 2 * nred; k++)
            if (!(red_phi[k] > 0.0)) { ctx->err = "red-noise weight must be > 0"; return PINT_E_INVALID; }
    if (ep_phi)
        for (int e = 0; e < nep; e++)
            if (!(ep_phi[e] > 0.0)) { ctx->err = "ECORR weight must be > 0"; return PINT_E_INVALID; }
    HIPCHK(hipStreamSynchronize(ctx->sstream));
    if (red_phi && nred > 0)
        HIPCHK(h2d((void*)ph.dev.red_phi, red_phi, sizeof(double) * 2 * nred, ctx->stream, false));
    if (ep_phi && nep > 0)
        HIPCHK(h2d((void*)ph.dev.ep_phi, ep_phi, sizeof(double) * nep, ctx->stream, false));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PINT_OK;
}

int pint_set_noise_classes(pint_ctx* ctx, int psr, int ncls, const int32_t* cls_ptr, const int32_t* cls_idx,
                           const double* sigma0_us) {
    if (!ctx || psr < 0 || psr >= (int)ctx->psrs.size() || ncls <= 0 || !cls_ptr || !cls_idx || !sigma0_us)
        return PINT_E_INVALID;
    hipSetDevice(ctx->device);
    if (int rc_ = commit_uploads(ctx)) return rc_;  // (staged pulsar uploads first)
    PsrHost& ph = ctx->psrs[psr];
    const int n = ph.n;
    if (cls_ptr[0] != 0 || cls_ptr[ncls] != n) { ctx->err = "noise classes must cover every TOA once"; return PINT_E_INVALID; }
    std::vector<int32_t> tc(n, -1);
    for (int c = 0; c < ncls; c++) {
        if (cls_ptr[c + 1] < cls_ptr[c]) { ctx->err = "bad noise class list"; return PINT_E_INVALID; }
        for (int k = cls_ptr[c]; k < cls_ptr[c + 1]; k++) {
            const int i = cls_idx[k];
            if (i < 0 || i >= n || tc[i] >= 0) { ctx->err = "noise classes must cover every TOA once"; return PINT_E_INVALID; }
            tc[i] = c;
        }
    }
    for (int i = 0; i < n; i++)
        if (!(sigma0_us[i] > 0.0)) { ctx->err = "TOA uncertainty must be > 0"; return PINT_E_INVALID; }
    int rc = 0;
    rc |= upload(ctx, ph, cls_ptr, (size_t)ncls + 1, ph.dev.cls_ptr);
    rc |= upload(ctx, ph, cls_idx, (size_t)n, ph.dev.cls_idx);
    rc |= upload(ctx, ph, tc.data(), (size_t)n, ph.dev.toa_cls);
    rc |= upload(ctx, ph, sigma0_us, (size_t)n, ph.dev.sigma0);
    if (rc) return PINT_E_HIP;
    ph.dev.ncls = ncls;
    return refresh_psrs(ctx) ? PINT_E_HIP : PINT_OK;
}

int pint_noise_lnlike(pint_ctx* ctx, const int32_t* kind, const double* cls_qf, const double* ep_w, double* out3,
                      double* cls_g, double* ep_g) {
    if (!ctx || ctx->ninst <= 0 || !kind || !cls_qf || !out3) return PINT_E_INVALID;
    flush_r2(ctx);
    hipSetDevice(ctx->device);
    const int ni = ctx->ninst;
    std::vector<long> meta(3 * (size_t)ni);
    long nq = 0;
    bool any_ep = false;
    for (int k = 0; k < ni; k++) {
        const PsrDev& d = ctx->psrs[ctx->inst[k].psr].dev;
        if (d.ncls <= 0) { ctx->err = "pint_noise_lnlike: no noise classes (pint_set_noise_classes)"; return PINT_E_INVALID; }
        if (kind[k] < 0 || kind[k] > 2) { ctx->err = "pint_noise_lnlike: bad kind"; return PINT_E_INVALID; }
        if (kind[k] > 0 && d.nep > 0) {
            if (d.ep_overlap) { ctx->err = "pint_noise_lnlike: overlapping ECORR epochs"; return PINT_E_INVALID; }
            any_ep = true;
        }
        meta[3 * k] = nq;
        meta[3 * k + 1] = kind[k];
        meta[3 * k + 2] = 0;
        nq += d.ncls;
    }
    if (any_ep && !ep_w) { ctx->err = "pint_noise_lnlike: ECORR weights required"; return PINT_E_INVALID; }
    const long nep = std::max<long>(1, ctx->tot_ep);
    // scratch: meta (as doubles' storage) | qf 2nq | clsg 2nq | epw nep | epsv 2nep | epg nep | out 3ni
    const size_t need = (size_t)3 * ni + 4 * nq + 4 * nep + 3 * ni;
    if (need > ctx->nz_cap) {
        if (ctx->d_nz) hipFree(ctx->d_nz);
        ctx->d_nz = nullptr;
        ctx->nz_cap = 0;
        HIPCHK(hipMalloc(&ctx->d_nz, sizeof(double) * need));
        ctx->nz_cap = need;
    }
    long* d_meta = (long*)ctx->d_nz;
    double* d_q = ctx->d_nz + 3 * ni;
    double* d_g = d_q + 2 * nq;
    double* d_w = d_g + 2 * nq;
    double* d_sv = d_w + nep;
    double* d_eg = d_sv + 2 * nep;
    double* d_out = d_eg + nep;
    static_assert(sizeof(long) == sizeof(double), "meta packing");
    HIPCHK(h2d(d_meta, meta.data(), sizeof(long) * meta.size(), ctx->stream, false));
    HIPCHK(h2d(d_q, cls_qf, sizeof(double) * 2 * nq, ctx->stream, false));
    if (any_ep) HIPCHK(h2d(d_w, ep_w, sizeof(double) * ctx->tot_ep, ctx->stream, false));
    hipLaunchKernelGGL(k_noise_lnl, dim3(ni), dim3(256), 0, ctx->stream, ctx->d_psrs, ctx->d_inst, ctx->d_rt, d_meta,
                       d_q, d_w, d_sv, d_out, d_g, d_eg);
    HIPCHK(hipGetLastError());
    HIPCHK(d2h(out3, d_out, sizeof(double) * 3 * ni, ctx->stream));
    if (cls_g) HIPCHK(d2h(cls_g, d_g, sizeof(double) * 2 * nq, ctx->stream));
    if (ep_g && ctx->tot_ep > 0)
        HIPCHK(d2h(ep_g, d_eg, sizeof(double) * ctx->tot_ep, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PINT_OK;
}

int pint_sync(pint_ctx* ctx) {
    HIPCHK(hipStreamSynchronize(ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->cstream));
    HIPCHK(hipStreamSynchronize(ctx->sstream));
    return PINT_OK;
}

}  // extern "C"
