/*
 * pint_amd.h — C-ABI of libpint_hip.so, the MI355X (gfx950) implementation of PINT's
 * fit-and-residual hot path.
 *
 * The reference (Jackson-D-Taylor/PINT, pure Python) has no FFI; every entry point below
 * replaces a Python call on the hot path, cited as reference file:line.  Plain pointers
 * and sizes only: caller-owned host buffers, library-owned device buffers, int status
 * codes (0 = ok) and pint_last_error() for a message.  One context per host thread; each
 * context owns one HIP stream on one device.
 *
 * Data model (see DESIGN.md "Data layout in HBM"):
 *   - a *pulsar* is a packed SoA TOA set (N rows + 1 TZR row) plus a ModelSpec
 *     (structure: which components, column map, table offsets);
 *   - an *instance* is one parameter table (doubles, every parameter a double-double
 *     hi/lo pair, in the reference's par-file units) bound to a pulsar.  A batch of
 *     instances (grid points, PTA pulsars, downhill trial states) is evaluated by one
 *     launch sequence.
 */
#ifndef PINT_AMD_H
#define PINT_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes -------------------------------------------------------------- */
#define PINT_OK 0
#define PINT_E_INVALID 1      /* bad argument / shape / unsupported model feature    */
#define PINT_E_HIP 2          /* HIP runtime error                                    */
#define PINT_E_NOT_PD 3       /* normal matrix not positive definite (LinAlgError)    */
#define PINT_E_KEPLER 4       /* Kepler iteration did not converge / ECC outside [0,1)*/
#define PINT_E_PARAM 5        /* invalid model parameter region (InvalidModelParameters)*/
#define PINT_E_SIGMA 6        /* Woodbury Sigma = Phi^-1 + U^T N^-1 U not positive definite */

/* ---- limits -------------------------------------------------------------------- */
#define PINT_MAX_COLS 320     /* design-matrix columns incl. Offset                   */
#define PINT_MAX_F 16
#define PINT_MAX_DMK 10
#define PINT_MAX_FD 10
#define PINT_MAX_JUMP 64

/* ---- per-TOA packed input (reference TOAs.table columns
 *      toa.py:2320 tdbld, :2385-2439 posvels, freq, error, mjd_float, pulse_number) ---- */
typedef struct {
    int32_t n;                      /* TOAs, excluding the TZR row                      */
    const double *tdb_hi, *tdb_lo;  /* n+1: exact double-double split of longdouble tdbld (days) */
    const double *freq_mhz;         /* n+1                                              */
    const double *sigma_s;          /* n: scaled TOA uncertainty (s), noise_model.py:159 */
    const double *pos_km;           /* (n+1)*3 ssb_obs_pos (row-major xyz)              */
    const double *vel_kms;          /* (n+1)*3 ssb_obs_vel                              */
    const double *sun_km;           /* (n+1)*3 obs_sun_pos                              */
    const double *pulse_number;     /* n (NaN-free when track_mode=pulse numbers)       */
    const double *delta_pn;         /* n+1 delta_pulse_number                           */
    const uint32_t *flags;          /* n+1 bit0: barycentric obs, bit1: all ssb_obs_pos != 0 */
    const uint64_t *jump_mask;      /* n+1 bit k: JUMP k selects this TOA               */
    const int32_t *dmx_a, *dmx_b;   /* n+1 DMX bin indices (-1 none; two allow overlap) */
    const double *planet_km;        /* (n+1)*15 obs_<planet>_pos for jupiter, saturn, venus,
                                       uranus, neptune (toa.py:2403-2433); read only when
                                       spec.shapiro == 2, may be NULL otherwise             */
    const int32_t *dmx_x;           /* DMX bins beyond a TOA's first two (any number may overlap,
                                       dispersion_model.py:659-678): n+2 offsets into this array,
                                       then the bin indices; NULL when no TOA has more than two */
} pint_toas_t;

/* The same per-TOA input as the TOA table's own columns (n rows each, no TZR row) plus the TZR
 * TOA's values and the DMX ranges: the library forms the n+1-row pint_toas_t itself (the TZR
 * row appended, flags, DMX bins) -- the host packing of engine.pack_toas in native code. */
typedef struct {
    int32_t n;
    const double *tdb_hi, *tdb_lo;  /* n                                                  */
    const double *freq_mhz;         /* n                                                  */
    const double *pos_km;           /* n*3 ssb_obs_pos; vel_kms, sun_km likewise          */
    const double *vel_kms;
    const double *sun_km;
    const double *delta_pn;         /* n, or NULL (zeros)                                 */
    const double *mjd;              /* n float MJDs: the DMX ranges select on them (toa_select.py:101) */
    const uint8_t *is_bary;         /* n: barycentric observatory                         */
    const double *sigma_us;         /* n: scaled TOA uncertainty (us), noise_model.py:159  */
    const double *pulse_number;     /* n, or NULL (zeros)                                 */
    const uint64_t *jump_mask;      /* n+1, or NULL (no JUMPs)                            */
    const double *planet_km;        /* (n+1)*15 as in pint_toas_t, or NULL               */
    double tzr[15];                 /* the TZR TOA: tdb_hi, tdb_lo, freq_mhz, pos[3], vel[3], sun[3],
                                       delta_pn, mjd, is_bary (0/1)                      */
    int32_t ndmx;                   /* DMX ranges in parameter order (DMXR1_k, DMXR2_k)   */
    const double *dmx_r1, *dmx_r2;
} pint_toa_cols_t;

/* Form the pint_toas_t of `cols` into caller buffers (host only, no device): out->n and every
 * n+1 (n for sigma_s, pulse_number) array pointer must be set; dmx_x receives the overflow CSR
 * of TOAs in three or more bins when dmx_x_cap holds it.  Returns that CSR's length (0: none,
 * out->dmx_x set to NULL; larger than dmx_x_cap: nothing written to dmx_x, call again), or a
 * negative status.  Bit-identical to engine.pack_toas. */
int64_t pint_pack_toas(const pint_toa_cols_t *cols, pint_toas_t *out, int32_t *dmx_x, int64_t dmx_x_cap);

/* ---- model structure ------------------------------------------------------------ */
/* column kinds for the design matrix (timing_model.py:2073 designmatrix)              */
enum {
    PINT_COL_OFFSET = 0, PINT_COL_F = 1, PINT_COL_LON = 2, PINT_COL_LAT = 3,
    PINT_COL_PMLON = 4, PINT_COL_PMLAT = 5, PINT_COL_PX = 6, PINT_COL_DM = 7,
    PINT_COL_DMX = 8, PINT_COL_FD = 9, PINT_COL_JUMP = 10, PINT_COL_BIN = 11,
    PINT_COL_ZERO = 12      /* a parameter without a delay (DMJUMP, dispersion_model.py:797) */
};
/* binary parameter ids (stand_alone_psr_binaries/binary_generic.py, ELL1_model.py, DD_model.py,
 * ELL1H_model.py (H3, H4, STIGMA), DDK_model.py (KIN, KOM)) */
enum {
    PINT_B_PB = 0, PINT_B_PBDOT, PINT_B_XPBDOT, PINT_B_A1, PINT_B_A1DOT, PINT_B_ECC,
    PINT_B_EDOT, PINT_B_T0, PINT_B_OM, PINT_B_OMDOT, PINT_B_M2, PINT_B_SINI, PINT_B_GAMMA,
    PINT_B_DR, PINT_B_DTH, PINT_B_A0, PINT_B_B0, PINT_B_TASC, PINT_B_EPS1, PINT_B_EPS2,
    PINT_B_EPS1DOT, PINT_B_EPS2DOT, PINT_B_H3, PINT_B_H4, PINT_B_STIGMA, PINT_B_KIN, PINT_B_KOM,
    PINT_B_NPAR
};
/* binary models (spec.binary) */
enum { PINT_BIN_NONE = 0, PINT_BIN_ELL1 = 1, PINT_BIN_DD = 2, PINT_BIN_ELL1H = 3, PINT_BIN_BT = 4, PINT_BIN_DDK = 5,
       PINT_NBIN = 6 };

typedef struct {
    int32_t nf;             /* spin terms F0..F{nf-1}                                   */
    int32_t astrometry;     /* 0 none, 1 equatorial (RAJ/DECJ), 2 ecliptic (ELONG/ELAT) */
    int32_t shapiro;        /* SolarSystemShapiro: 0 absent, 1 the Sun, 2 the Sun and the
                               PLANET_SHAPIRO planets (solar_system_shapiro.py:105-117)    */
    int32_t ndm;            /* DispersionDM taylor terms (0 = component absent)         */
    int32_t ndmx;           /* DMX bins                                                 */
    int32_t binary;         /* PINT_BIN_*: 0 none, 1 ELL1, 2 DD, 3 ELL1H, 4 BT, 5 DDK   */
    int32_t nfd;            /* FD terms                                                 */
    int32_t njump;          /* phase JUMPs                                              */
    int32_t track_pn;       /* 1: use_pulse_numbers, 0: nearest  (residuals.py:133-149) */
    int32_t subtract_mean;  /* residuals.py:124                                         */
    int32_t weighted_mean;
    int32_t ncol;           /* design-matrix columns incl. Offset                      */
    int32_t nred;           /* PLRedNoise modes (2*nred Fourier columns), 0 = none     */
    int32_t tstride;        /* doubles per instance parameter table                    */
    /* table offsets (doubles; each parameter is a dd pair at [off], [off+1]); -1 absent */
    int32_t o_F, o_PEPOCH, o_lon, o_lat, o_pmlon, o_pmlat, o_px, o_POSEPOCH;
    int32_t o_DM, o_DMEPOCH, o_DMX, o_FD, o_JUMP, o_bin[PINT_B_NPAR];
    int32_t o_PHOFF;        /* PhaseOffset: table slot of PHOFF (-1 none); the TOAs' phase gets
                               -PHOFF, the TZR TOA's does not (phase_offset.py offset_phase)    */
    int32_t wb_noones;      /* 1: the Woodbury chi2 has no offset column of ones (PHOFF free,
                               residuals.py:583-585); the ECORR-only Sherman-Morrison chi2 of
                               :591-636 is this form with the ECORR basis alone             */
    int32_t ell1h;          /* ELL1H Shapiro form (binary_ell1.py:383-405): 1 H3 alone (Eq. 19,
                               stigma 0), 2 H3 + H4 (Eq. 19, stigma = H4/H3), 3 H3 + STIGMA
                               (exact, Eq. 29); 0 otherwise                                 */
    int32_t nharms;         /* ELL1H: last harmonic of Eq. 19 (NHARMS; max(NHARMS, 7) with H4) */
    int32_t dmn0;           /* first PLDMNoise mode among the nred Fourier modes (= nred: none);
                               modes >= dmn0 are scaled by (1400 MHz / f_bary)^2 per TOA
                               (noise_model.py:443-540 PLDMNoise.get_noise_basis)           */
    int32_t k96;            /* DDK: 1 = Kopeikin (1996) proper-motion terms on a1, omega and i
                               (K96, the reference default; DDK_model.py:157-349), 0 = off */
    int32_t o_DMJUMP;       /* DispersionJump: table slot of the first DMJUMP (-1 none); they
                               offset the modelled DM values only (dispersion_model.py:724-795) */
    int32_t ndmjump;        /* DMJUMPs (<= 64; bit k of the per-TOA DMJUMP mask selects DMJUMP k+1) */
    double obliquity;       /* rad, ecliptic models (pulsar_ecliptic.py OBL[ECL])       */
    double red_f0;          /* red-noise fundamental 1/T (Hz), noise_model.py:847       */
    double red_t0;          /* unused reserve                                           */
    int32_t col_kind[PINT_MAX_COLS];
    int32_t col_index[PINT_MAX_COLS];
    int32_t col_toff[PINT_MAX_COLS];  /* table offset of the column's parameter (-1: Offset) */
} pint_spec_t;

/* ---- context -------------------------------------------------------------------- */
typedef struct pint_ctx pint_ctx;

/* One context per host thread; it owns one HIP stream on `device`. */
pint_ctx *pint_ctx_create(int device);
void pint_ctx_destroy(pint_ctx *ctx);
const char *pint_last_error(pint_ctx *ctx);

/* Instance buffers are drawn from a process-wide cache per device and returned to it by
 * pint_set_instances / pint_ctx_destroy; this hands every idle cached buffer back to the
 * HIP runtime (no reference counterpart: device memory management). */
void pint_release_cache(void);
int pint_device_count(void);
/* Pipeline slots of pint_step_end / pint_check_step, fixed when the library is built
 * (-DPINT_NSLOT, default 4): the host's slot bookkeeping must use this value. */
int pint_nslot(void);

/* Upload one pulsar (packed TOAs + model structure); returns its id >= 0, or -status.
 * Replaces the TOAs.table hand-off of get_model_and_toas (model_builder.py:859) and the
 * param-independent noise bases: red_freq[2*nred] are the PLRedNoise Fourier frequencies
 * as double-double pairs (hi[nred] then lo[nred]: the reference keeps them longdouble)
 * (noise_model.py:847 get_rednoise_freqs), red_phi[2*nred] their weights
 * (noise_model.py:780 get_noise_weights).  The library copies everything it needs. */
int pint_add_pulsar(pint_ctx *ctx, const pint_toas_t *toas, const pint_spec_t *spec,
                    const double *red_freq, const double *red_phi);
/* pint_add_pulsar from the TOA table's columns (pint_pack_toas into the context's scratch). */
int pint_add_pulsar_cols(pint_ctx *ctx, const pint_toa_cols_t *cols, const pint_spec_t *spec,
                         const double *red_freq, const double *red_phi);

/* Bind `ninst` instances (grid points, PTA pulsars, trial states): inst_psr[k] is a
 * pulsar id; `tables` concatenates each instance's parameter table (spec.tstride doubles,
 * dd pairs in par-file units).  Replaces the parameter state of a TimingModel
 * (parameter.py values) for a whole batch. */
int pint_set_instances(pint_ctx *ctx, int ninst, const int32_t *inst_psr, const double *tables);

/* A grid of npts instances of pulsar psr (gridutils.py:166 grid_chisq, :392, :588, :773 -- the
 * reference forms one model copy per point, gridutils.py:72): each point's table is `base`
 * (tstride doubles) with nvar (hi, lo) entries replaced, formed on the device from the base
 * table and the grid axes.  Variable j (table offset var_toff[j]) of point k takes the pair
 * vals_j[((k0 + k) / var_stride[j]) % var_size[j]], vals_j = the var_size[j] (hi, lo) pairs
 * of variable j in `vals` (the variables' pairs concatenated): a meshgrid's axis, or every
 * point's own value (stride 1).  k0: the global index of the first point (a rank's block).
 * Otherwise as pint_set_instances. */
int pint_set_grid(pint_ctx *ctx, int psr, int npts, const double *base, int nvar, const int32_t *var_toff,
                  const int64_t *var_stride, const int64_t *var_size, const double *vals, int64_t k0);
int pint_get_tables(pint_ctx *ctx, double *tables_out);
int pint_set_tables(pint_ctx *ctx, const double *tables);

/* Evaluate delay (timing_model.py:1515), phase (:1548, incl. the TZR phase) and, when
 * want_M, the design matrix (:2073) plus the red-noise basis columns; then residuals
 * (residuals.py:314 calc_phase_resids, :483 calc_time_resids) and the WLS chi2 (:638)
 * for every instance. */
int pint_eval(pint_ctx *ctx, int want_M);  /* want_M: 0 none, 1 full, 2 fit layout */

/* Copy results to caller buffers (any pointer may be NULL).  Residual rows are n_i per
 * instance, eval rows n_i+1 (last = TZR TOA), design matrices n_i x K_i column-major
 * with K_i = ncol + 2*nred.  pint_read_resids in lazy mode only enqueues its copies (pinned
 * buffers, valid after pint_check). */
int pint_read_resids(pint_ctx *ctx, double *time_resid, double *phase_resid, double *chi2_wls);
int pint_read_eval(pint_ctx *ctx, double *phase_hi, double *phase_lo, double *ftaylor, double *delay);
int pint_read_designmatrix(pint_ctx *ctx, double *M);

/* One normal-equations step for every instance on the state of the last pint_eval(1):
 * mode 0 = WLS (fitter.py:1965 WLSFitter / :1282 WLSState.step), mode 1 = GLS
 * (:2104 GLSFitter / :1425 GLSState.step, rank-reduced, full_cov=False).  The GLS mode
 * also factors the Woodbury Sigma used by pint_chi2_gls. */
int pint_fit_step(pint_ctx *ctx, int mode);
/* dpars/errs: (K_i+1) per instance (par units, [0] = Offset; noise coefficients after the
 * ncol timing columns); cov: ncol_i x ncol_i per instance (timing-parameter covariance,
 * fitter.py:2240 parameter_covariance_matrix); chi2_lin: linearised post-step chi2. */
int pint_read_step(pint_ctx *ctx, double *dpars, double *errs, double *cov, double *chi2_lin);

/* tables += lambda[k] * dpars (double-double add): fitter.py:957 take_step_model and
 * :2073-2080 the longdouble parameter update. */
int pint_apply_step(pint_ctx *ctx, const double *lambda_);
/* The same with one lambda for every instance (GLSFitter / WLSFitter take the full step,
 * fitter.py:2254-2263); a kernel argument, no host->device copy. */
int pint_apply_step_uniform(pint_ctx *ctx, double lambda_);
/* pint_fit_step followed by pint_apply_step_uniform(lambda_) (GLSFitter.fit_toas's step and
 * full-step update, fitter.py:2164-2263): when every instance takes the DMX-eliminated solve
 * on the generated-Fourier path the update and the new tables' per-instance constants are
 * formed at the end of the solve kernel, saving the apply launch.  pint_read_step and
 * pint_noise_resids read the step, not the tables, and may follow it. */
int pint_fit_step_apply(pint_ctx *ctx, int mode, double lambda_);

/* Device-resident parameter tables: pint_save_tables snapshots the batch's current tables
 * on the device, pint_restore_tables copies the snapshot back (device->device on the
 * stream), e.g. to start repeated fits from the same initial models without an upload. */
int pint_save_tables(pint_ctx *ctx);
int pint_restore_tables(pint_ctx *ctx);

/* GLS chi2 (Woodbury, residuals.py:567 _calc_gls_chi2 + utils.py:3074 woodbury_dot) of
 * the current residuals, per instance. */
int pint_chi2_gls(pint_ctx *ctx, double *chi2);

/* WLS chi2 (residuals.py:638-667 _calc_wls_chi2: sum (r / sigma_scaled)^2) of the current
 * residuals, per instance -- e.g. of residuals replaced by pint_debug_set_resids (the
 * residual pass reports its own through pint_read_resids). */
int pint_chi2_wls(pint_ctx *ctx, double *chi2);

/* ECORR epochs of pulsar `psr` (replaces EcorrNoise.ecorr_basis_weight_pair,
 * noise_model.py:385-427 + get_ecorr_epochs :808): nep epochs, TOA index lists in CSR form
 * (ep_ptr[nep+1], ep_idx[ep_ptr[nep]]) and the prior variance phi_e = ECORR^2 in s^2.
 * The quantisation block is eliminated by a Schur complement on the device (its normal
 * matrix block is diagonal), so it adds no Gram columns; on the compact layout each epoch
 * then couples to at most one DMX column (else the pulsar takes the full layout).  Call
 * before pint_set_instances. */
int pint_set_ecorr(pint_ctx *ctx, int psr, int nep, const int32_t *ep_ptr, const int32_t *ep_idx,
                   const double *ep_phi);

/* Fit layout of pulsar `psr` (no reference counterpart; for benchmarks/tests):
 * out4 = {compact, Gram columns excl. residual, sparse DMX columns, padded Gram width}.
 * compact = 1 when the DMX columns are kept out of M and the dense Gram (>= 8 free DMX
 * columns, no TOA in two free bins, no TOA in two ECORR epochs, every ECORR epoch's TOAs in at
 * most one free bin -- its elimination then keeps the DMX block diagonal, k_ecorr_dmx):
 * pint_eval(ctx, 2) then writes the compact
 * design matrix, and pint_fit_step forms their Gram rows as bin sums. */
int pint_fit_layout(pint_ctx *ctx, int psr, int32_t *out4);
/* The k_gram_v layout of a pulsar in the current batch: (on the vg path (+2 with the
 * binned DMX x Fourier tile, PINT_OPT_VBIN), DMX slots, LDS width [T | r | slots | F]
 * padded to 16, timing columns of the compact layout). */
int pint_vgram_layout(pint_ctx *ctx, int psr, int32_t *out4);
/* Wideband DM data of pulsar `psr` (n TOAs): the measured DMs pp_dm and their errors pp_dme
 * (the -pp_dm / -pp_dme TOA flags, toa.py:1767-1791), the errors scaled by DMEFAC/DMEQUAD
 * (ScaleDmError.scale_dm_sigma, noise_model.py:291), and each TOA's DMJUMP mask (bit k:
 * DMJUMP k+1 selects it).  All in pc/cm^3.  Replaces WidebandDMResiduals.get_dm_data
 * (residuals.py:1044-1071). */
int pint_set_wideband(pint_ctx *ctx, int psr, const double *pp_dm, const double *pp_dme,
                      const double *dm_sigma, const uint64_t *dmjump_mask);
/* WidebandDMResiduals.calc_resids / calc_chi2 (residuals.py:1000-1031) of every instance
 * whose pulsar has wideband data: pp_dm - total_dm (DispersionDM Taylor series + DMX +
 * DMJUMP, timing_model.py:1593) at the instance's parameters, the mean (weighted by
 * 1/pp_dme^2 unless use_weighted_mean = 0) removed if subtract_mean; chi2 with the scaled
 * errors.  resid_out: the instances' TOA rows concatenated (n per instance, 0 for pulsars
 * without wideband data), chi2_out[ninst] (NaN without wideband data). */
int pint_dm_resids(pint_ctx *ctx, int subtract_mean, int use_weighted_mean, double *resid_out,
                   double *chi2_out);

/* Lazy mode (1): launches return without synchronising or checking the device status;
 * pint_check() synchronises and returns the accumulated status.  In lazy mode
 * pint_set_tables, pint_read_step and pint_chi2_gls only enqueue their copies
 * (pint_read_step on a second stream, overlapped with the kernels that follow): host
 * buffers must stay valid, and outputs are complete, after pint_check().  Use pinned
 * buffers (pint_host_alloc) for the copies to run asynchronously. */
int pint_set_lazy(pint_ctx *ctx, int lazy);
int pint_check(pint_ctx *ctx);

/* Pipelined steps (replaces the per-step pint_check of a lazy-mode loop; no reference
 * counterpart -- the reference's fitters are synchronous).  pint_step_end closes the work
 * enqueued since the previous step_end and returns its slot (0 .. PINT_NSLOT-1) in *slot;
 * launches after it go to the next slot (own status word, timing events, fit-output
 * buffers).  pint_check_step waits for that step only and returns its status, so the host
 * enqueues the next steps while the device runs step k.  At most PINT_NSLOT steps in
 * flight: check slot s before ending the step that reuses it.  Pinned output buffers must
 * be per slot.  In lazy mode pint_read_step / pint_noise_resids(_dm) put their copy-stream
 * work behind the step's last kernel (at pint_step_end or pint_check), not behind the
 * solve. */
#ifndef PINT_NSLOT
#define PINT_NSLOT 4
#endif
int pint_step_end(pint_ctx *ctx, int *slot);
/* One GLSFitter.fit_toas(maxiter=1) step of every instance (fitter.py:2164-2289: the GLS
 * step, full_cov=False noise realisations :2269-2282, the post-fit chi2 it returns) enqueued
 * by a single call, lazy mode only: [pint_restore_tables when restore], pint_eval(2),
 * pint_fit_step_apply(mode = 1, lambda_), pint_read_step(dpars, errs, cov, chi2lin),
 * pint_noise_resids(noise_red, noise_ecorr), pint_noise_resids_dm(noise_dm), pint_eval(0),
 * pint_chi2_gls(chi2), pint_step_end(slot).  NULL outputs are skipped; pinned buffers
 * (pint_host_alloc), complete after pint_check_step(*slot). */
int pint_fit_step_enqueue(pint_ctx *ctx, int restore, int mode, double lambda_, double *dpars, double *errs,
                          double *cov, double *chi2lin, double *noise_red, double *noise_ecorr, double *noise_dm,
                          double *chi2, int *slot);
int pint_check_step(pint_ctx *ctx, int slot);
/* Engine options (no reference counterpart): PINT_OPT_BLOCKED_SOLVE = 1 (default) solves
 * the normal equations with the blocked FP64-MFMA kernel, 0 with the column-by-column
 * LDS kernel (used by the tests to cross-check the two).  PINT_OPT_VGRAM = 1 (default)
 * generates the PLRedNoise Fourier columns inside the Gram and Woodbury kernels of the
 * compact fit layout (never stored in M) and fuses the DMX bin sums into the Gram; 0
 * keeps them in M (the tests cross-check the two).  Takes effect at pint_set_instances. */
#define PINT_OPT_BLOCKED_SOLVE 1
#define PINT_OPT_VGRAM 2
/* PINT_OPT_TIMING_MASK: bit k enables timing slot k of pint_last_timing (default 0xff).
 * Every HIP timing event costs device time (~5 us each), so a timed run enables only the
 * slots it reports. */
#define PINT_OPT_TIMING_MASK 3
/* PINT_OPT_TIMING_EVERY k (default 1): the Gram kernels' timing events (slot 6) ride on
 * every k-th pint_fit_step only; the other steps carry no events.  The slot then reads 0
 * after an unsampled step. */
#define PINT_OPT_TIMING_EVERY 8
/* PINT_OPT_REFINE = 1 (default): a normal-equations solve whose condition estimate
 * max diag(A) * max diag(A^-1) exceeds 1e8 gets one pass of iterative refinement with a
 * double-double residual (the explicit L^-1 of the blocked solves otherwise loses ~cond(L)
 * digits that LAPACK's cho_solve keeps); 0 skips it (grid points: their post-fit chi2 is
 * second order in a step error along the weak directions). */
#define PINT_OPT_REFINE 4
/* PINT_OPT_VBIN = 1 (default): k_gram_v forms the DMX bins' Fourier entries from one binned
 * trig tile per k-step (the accumulator holds an even and an odd bin) instead of the DMX-slot
 * row tiles x Fourier columns; pulsars whose aligned 4-row groups hold more than two bins
 * (or two of one parity) leave the vg path.  Takes effect at pint_set_instances. */
#define PINT_OPT_VBIN 5
/* PINT_OPT_WBFIT = 1: pint_fit_step adds the wideband DM rows (pint_set_wideband) of every
 * compact-layout instance to its normal equations (WidebandTOAFitter.fit_toas,
 * fitter.py:2465-2637: design matrix [M_toa | F; M_dm | 0], residuals [r; pp_dm - DM]);
 * default 0. */
#define PINT_OPT_WBFIT 6
/* PINT_OPT_COV_DEFER (default 1, env PINT_COV_DEFER): the covariance of the DMX-eliminated
 * solve is formed by pint_read_step (k_cov_dmx, several workgroups per instance, on the copy
 * stream) instead of inside the solve: 0 never, 1 for batches of >= 16 instances, 2 always.
 * Same values bit for bit; takes effect at the next pint_fit_step. */
#define PINT_OPT_COV_DEFER 7
/* PINT_OPT_SCHUR = 1 (default): for deferred solves (PINT_OPT_COV_DEFER) the DMX-eliminated
 * solve's build phase -- column norms, S = A_dd, U = A_dx D^-1/2, S -= U U^T, b'_d -- runs as
 * k_schur, one workgroup per (block of S, instance), before the one-workgroup-per-instance
 * solve; 0 keeps it inside the solve.  Same operations in the same order: same bits. */
#define PINT_OPT_SCHUR 9
/* PINT_OPT_SMALL = 1 (default): instances of at most 32 padded columns and 512 rows (a
 * grid's points) take k_gram_s (a wave per instance, applies from the next
 * pint_set_instances) and the one-wave k_solve_blk (four instances per workgroup); 0 keeps
 * them on the 16-wave Gram and the 4-wave solve (the tests cross-check the two). */
#define PINT_OPT_SMALL 10
/* PINT_OPT_LA_CHOL = 1 (default, env PINT_LA_CHOL): the DMX-eliminated solve factors its
 * dense block with look-ahead (the next diagonal block factored beside the current trailing
 * update, L^-1's block rows beside the panels); 0 runs the plain blocked order.  The same
 * operations in the same order per block: the same bits. */
#define PINT_OPT_LA_CHOL 11
/* PINT_OPT_EFUSE = 1 (default, env PINT_EFUSE): batches off the small-instance path evaluate
 * 254 rows per block plus row 0 and the TZR row, and form the phase residuals and their
 * weighted sums there (the residual pass's first half, no k_resid1 launch); applies from the
 * next pint_set_instances. */
#define PINT_OPT_EFUSE 12
/* PINT_OPT_LANE_SOLVE = 1 (default, env PINT_LANE_SOLVE): small-instance batches (the
 * PINT_OPT_SMALL path) whose normal equations have at most 8 columns are solved with one
 * lane per instance (64 instances per wave) instead of one wave per instance. */
#define PINT_OPT_LANE_SOLVE 13
/* PINT_OPT_SPIN_EVAL = 1 (default, env PINT_SPIN_EVAL): a pint_set_grid batch whose points
 * differ in spin frequencies only (isolated model, no red-noise basis) evaluates its rows'
 * delays and astrometric geometry once, on the first point, for the evaluation with the
 * design matrix that precedes the first fit step; each point then runs the spin part only.
 * The same bits as the full evaluation. */
#define PINT_OPT_SPIN_EVAL 14
/* PINT_OPT_SOLVE_W8 = 1 (default, env PINT_SOLVE_W8): the DMX-eliminated solve runs 8 waves
 * per instance (256 VGPRs per lane) when its dense block has at most 8 16-column blocks,
 * else 16.  The same operations per element: the same bits. */
#define PINT_OPT_SOLVE_W8 15
int pint_set_option(pint_ctx *ctx, int key, int value);
/* The SVD path of the fitters for degenerate normal equations (WLSState.step,
 * fitter.py:1282-1359: singular values of the whitened normalised M below threshold * s_max
 * dropped; GLSFitter fitter.py:2196-2230: SVD of mtcm when Cholesky fails), on the Gram of
 * the last pint_fit_step(mode), threshold[i] per instance: eigendecomposition of the normalised normal matrix (Jacobi,
 * on the device).  Replaces the outputs pint_read_step returns.  ndeg[i] = dropped
 * directions of instance i (<= PINT_EIG_MAXDEG); degvec[(i * PINT_EIG_MAXDEG + d) *
 * degstride + k] their components over the instance's fit columns, scaled to max |.| = 1,
 * smallest singular value first (degstride >= the widest instance's column count). */
#define PINT_EIG_MAXDEG 8
int pint_solve_eig(pint_ctx *ctx, int mode, const double *threshold, int32_t *ndeg, double *degvec,
                   int degstride);

/* Likelihood normalisation per instance, Residuals.calc_chi2(lognorm=True)
 * (residuals.py:567-589, :638-667): gls != 0 gives logdet(C)/2 of the last pint_chi2_gls
 * (C = N + U Phi U^T, U = [F, ECORR, 1], utils.py:3074 woodbury_dot), gls == 2 the same
 * for a correlated-noise model whose basis has no columns (U = [1]), gls == 0 gives
 * sum_i log sigma_i (s).  lnlikelihood = -(chi2/2 + lognorm). */
int pint_lognorm(pint_ctx *ctx, int gls, double *out);

/* HIP-graph capture of a launch sequence (lazy mode only).  Everything the calls between
 * pint_capture_begin and pint_capture_end enqueue (kernels, the copies to and from the
 * caller's pinned buffers, the side-stream work) becomes one graph; pint_graph_launch
 * replays it with one launch.  Device buffers and host pointers are fixed at capture, so a
 * replay re-runs the same batch on whatever those buffers hold (e.g. new parameter tables
 * written into the same pinned buffer).  One graph per pipeline slot (pint_step_end): a
 * capture belongs to the slot current at pint_capture_end (its outputs, status word and
 * pinned buffers), and pint_graph_launch replays the current slot's graph, so captured steps
 * pipeline two deep like enqueued ones.  pint_set_instances discards the graphs. */
int pint_capture_begin(pint_ctx *ctx);
int pint_capture_end(pint_ctx *ctx);
int pint_graph_launch(pint_ctx *ctx);
/* Introspection: PINT_QUERY_NVGRAM = 1 returns the number of instances of the current batch
 * on the generated-Fourier path, PINT_QUERY_NSPLIT = 2 the Gram's N-split count (row blocks
 * per instance); negative status on error. */
#define PINT_QUERY_NVGRAM 1
#define PINT_QUERY_NSPLIT 2
int pint_query(pint_ctx *ctx, int key);
/* Page-locked host memory for the output buffers (hipHostMalloc); NULL on failure. */
void *pint_host_alloc(size_t bytes);
void pint_host_free(void *p);
/* Introspection for tests: 0 Gram partials, 1 column sums of squares, 2 Woodbury factor
 * (L^-1, packed lower). */
int pint_debug_read(pint_ctx *ctx, int which, double *out);
/* Stage-wise parity introspection (SURVEY.md 8(a) parity definition 2; no reference
 * counterpart -- these expose the intermediate arrays of fitter.py:2164-2202):
 * pint_debug_gram writes, per instance, the assembled unnormalised normal matrix
 * [M | r]^T N^-1 [M | r] of the last pint_fit_step ((K_i+1)^2, original column order,
 * residual last; ECORR block eliminated, or with pre_ecorr != 0 its Schur term
 * sum_e s_e s_e^T / D_e added back) followed by M's K_i unweighted column sums of
 * squares (utils.py:2879 normalize_designmatrix).  pint_debug_set_resids replaces every
 * instance's time residuals (n_i each) by the caller's, so that pint_fit_step and
 * pint_chi2_gls run on e.g. the reference's own residual arrays. */
int pint_debug_gram(pint_ctx *ctx, int pre_ecorr, double *out);
int pint_debug_set_resids(pint_ctx *ctx, const double *time_resid);

/* The normalisation of the last pint_fit_step's design matrix, the reference fitters' `fac`
 * / `norm` squared (utils.py:2879 normalize_designmatrix; fitter.py:1320-1343 WLS,
 * fitter.py:2164-2176 GLS): per instance K_i values at the same K_i+1 stride as
 * pint_read_step's dpars.  mode 1: the unweighted column sums of squares of [M | F];
 * mode 0: the diagonal of the whitened normal matrix M^T N^-1 M.  Synchronous. */
int pint_read_norms(pint_ctx *ctx, int mode, double *out);

/* Per-instance status bits (1 << PINT_E_*) raised by evaluations since the last call, one
 * int32 per instance; reading clears them.  The batch status returned by pint_eval/
 * pint_check names the first error of any instance; this names the instances, so one
 * invalid grid point or trial state fails alone (fitter.py:926-935 InvalidModelParameters,
 * gridutils.py:89-106 NaN per point). */
int pint_inst_status(pint_ctx *ctx, int32_t *out);

/* Noise realisations of the last pint_fit_step(mode=1), n_i per instance (either pointer
 * may be NULL): red = F a (PLRedNoise basis times its fitted coefficients), ecorr = the
 * ECORR epoch coefficients back-substituted from the eliminated block, per TOA.  Replaces
 * Residuals.noise_resids as GLSFitter.fit_toas (fitter.py:2270-2282) and
 * DownhillGLSFitter.fit_toas (:1582-1605) set it. */
int pint_noise_resids(pint_ctx *ctx, double *red, double *ecorr);
/* The PLDMNoise realisation of the same step (its modes times (1400 MHz / f_bary)^2), n_i per
 * instance: Residuals.noise_resids["pl_DM_noise"] (zeros for pulsars without PLDMNoise).  In
 * lazy mode it is enqueued on the copy stream like pint_noise_resids (dm valid after
 * pint_check / pint_check_step; the next evaluation with M waits for it). */
int pint_noise_resids_dm(pint_ctx *ctx, double *dm);

/* Device time (ms, HIP events on the streams the kernels run on) of the last launches, 8
 * values: [0] eval (no design matrix), [1] resid, [2] ecorr + Gram + partial reduction,
 * [3] solve, [4] eval with design matrix, [5] Woodbury chi2, [6] the Gram kernels alone
 * (k_gram / k_gram_v), [7] the Gram partial reduction (k_greduce). */
int pint_last_timing(pint_ctx *ctx, double *ms8);
int pint_sync(pint_ctx *ctx);

/* ---- noise-parameter fitting ------------------------------------------
 * DownhillFitter._fit_noise (fitter.py:1230-1273) maximises the likelihood over the free
 * EFAC/EQUAD/ECORR/red-noise parameters with the residuals of the current timing model held
 * fixed (fitter.py:1239-1247: one Residuals object, only its model's noise values change).
 *
 * pint_set_resids replaces every instance's time residuals (n_i each, s): the fixed
 * residuals of such a fit (= pint_debug_set_resids).
 * pint_set_sigma replaces pulsar psr's scaled TOA uncertainties (s) in place
 * (ScaleToaError.scale_toa_sigma, noise_model.py:159, at trial EFAC/EQUAD values) and
 * pint_set_noise_weights its noise-basis prior variances (PLRedNoise 2 nred, ECORR nep; s^2;
 * either NULL), for a Woodbury likelihood (pint_fit_step(ctx,1) + pint_chi2_gls +
 * pint_lognorm(ctx,1)) at trial noise parameters of a model with time-correlated noise. */
int pint_set_resids(pint_ctx *ctx, const double *time_resid);
int pint_set_sigma(pint_ctx *ctx, int psr, const double *sigma_s);
int pint_set_noise_weights(pint_ctx *ctx, int psr, const double *red_phi, const double *ep_phi);
/* White-noise classes of pulsar psr: its TOAs grouped by the set of EFAC/EQUAD masks that
 * select them, CSR (cls_ptr[ncls+1], cls_idx[n]; every TOA in exactly one class), with the
 * raw TOA uncertainties sigma0_us[n] (us).  A class's scaled variance is
 * N_i = (sigma0_i^2 + Q^2) F^2, Q^2 = sum of its EQUAD^2, F = product of its EFACs. */
int pint_set_noise_classes(pint_ctx *ctx, int psr, int ncls, const int32_t *cls_ptr, const int32_t *cls_idx,
                           const double *sigma0_us);
/* Log-likelihood of the current (fixed) residuals of every instance at trial noise
 * parameters, one device pass: Residuals.lnlikelihood (residuals.py:713) with
 * kind[k] = 0 diagonal N (_calc_wls_chi2, :638), 1 N + ECORR blocks by Sherman-Morrison
 * (_calc_ecorr_chi2, :591; PHOFF free), 2 as 1 plus the 1e40 offset column of
 * _calc_gls_chi2 (:583-587).  cls_qf: (Q^2 [us^2], F) per class, instances' classes
 * concatenated; ep_w: ECORR variance (s^2) per epoch of the batch (NULL when no instance
 * has kind > 0 and epochs).  out3[3k] = lnL, [3k+1] = chi2, [3k+2] = logdet(C)/2.
 * Gradients (kinds 0 and 1; either pointer may be NULL): cls_g[2c] = sum_{i in c} N_i
 * dlnL/dN_i, cls_g[2c+1] = sum_{i in c} dlnL/dN_i (s^-2), ep_g[e] = dlnL/dw_e (s^-2) --
 * the chain-rule pieces of Residuals.d_lnlikelihood_d_param (residuals.py:718-828):
 * dlnL/dEFAC_p = sum_{c ∋ p} 2 cls_g[2c] / EFAC_p, dlnL/dEQUAD_p = sum_{c ∋ p}
 * 2 EQUAD_p F_c^2 1e-12 cls_g[2c+1], dlnL/dECORR_p = sum_{e of p} 2 ECORR_p 1e-12 ep_g[e]. */
int pint_noise_lnlike(pint_ctx *ctx, const int32_t *kind, const double *cls_qf, const double *ep_w, double *out3,
                      double *cls_g, double *ep_g);

#ifdef __cplusplus
}
#endif
#endif
