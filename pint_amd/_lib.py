"""ctypes binding of libpint_hip.so (the C-ABI declared in include/pint_amd.h).

The HIP library is the only compute path: if it is missing or no GPU is visible, every
compute call raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBPATH = os.environ.get("PINT_LIB") or os.path.join(HERE, "libpint_hip.so")

MAX_COLS = 320
EIG_MAXDEG = 8  # PINT_EIG_MAXDEG
NSLOT = 4  # pipeline slots (pint_step_end / pint_check_step): set from the library's pint_nslot() by lib()
B_NPAR = 27
BIN_NONE, BIN_ELL1, BIN_DD, BIN_ELL1H, BIN_BT, BIN_DDK = range(6)

COL_OFFSET, COL_F, COL_LON, COL_LAT, COL_PMLON, COL_PMLAT, COL_PX, COL_DM, COL_DMX, COL_FD, COL_JUMP, COL_BIN, COL_ZERO = range(13)

PINT_OK, PINT_E_INVALID, PINT_E_HIP, PINT_E_NOT_PD, PINT_E_KEPLER, PINT_E_PARAM, PINT_E_SIGMA = range(7)

dptr = C.POINTER(C.c_double)


class ToasT(C.Structure):
    _fields_ = [("n", C.c_int32), ("tdb_hi", dptr), ("tdb_lo", dptr), ("freq_mhz", dptr), ("sigma_s", dptr),
                ("pos_km", dptr), ("vel_kms", dptr), ("sun_km", dptr), ("pulse_number", dptr), ("delta_pn", dptr),
                ("flags", C.POINTER(C.c_uint32)), ("jump_mask", C.POINTER(C.c_uint64)),
                ("dmx_a", C.POINTER(C.c_int32)), ("dmx_b", C.POINTER(C.c_int32)), ("planet_km", dptr),
                ("dmx_x", C.POINTER(C.c_int32))]


class ToaColsT(C.Structure):
    _fields_ = [("n", C.c_int32), ("tdb_hi", dptr), ("tdb_lo", dptr), ("freq_mhz", dptr), ("pos_km", dptr),
                ("vel_kms", dptr), ("sun_km", dptr), ("delta_pn", dptr), ("mjd", dptr),
                ("is_bary", C.POINTER(C.c_uint8)), ("sigma_us", dptr), ("pulse_number", dptr),
                ("jump_mask", C.POINTER(C.c_uint64)), ("planet_km", dptr), ("tzr", C.c_double * 15),
                ("ndmx", C.c_int32), ("dmx_r1", dptr), ("dmx_r2", dptr)]


class SpecT(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("nf", "astrometry", "shapiro", "ndm", "ndmx", "binary", "nfd", "njump",
                                          "track_pn", "subtract_mean", "weighted_mean", "ncol", "nred", "tstride",
                                          "o_F", "o_PEPOCH", "o_lon", "o_lat", "o_pmlon", "o_pmlat", "o_px",
                                          "o_POSEPOCH", "o_DM", "o_DMEPOCH", "o_DMX", "o_FD", "o_JUMP")] + [
        ("o_bin", C.c_int32 * B_NPAR), ("o_PHOFF", C.c_int32), ("wb_noones", C.c_int32), ("ell1h", C.c_int32), ("nharms", C.c_int32), ("dmn0", C.c_int32), ("k96", C.c_int32), ("o_DMJUMP", C.c_int32), ("ndmjump", C.c_int32), ("obliquity", C.c_double), ("red_f0", C.c_double), ("red_t0", C.c_double),
        ("col_kind", C.c_int32 * MAX_COLS), ("col_index", C.c_int32 * MAX_COLS), ("col_toff", C.c_int32 * MAX_COLS)]


class PintError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[pint_hip status {code}] {msg}")
        self.code = code


_lib = None
HIP_RUNTIME = None  # the libamdhip64 this process uses ("system", or torch's when torch came first)


def _one_hip_runtime():
    """One HIP runtime per process -- the system ROCm's -- whatever is loaded first.

    libpint_hip.so needs libamdhip64.so.7 (RUNPATH /opt/rocm/lib).  The ROCm torch wheel
    ships its own libamdhip64 / libhsa-runtime64 / librocprofiler-register (ROCm 7.0), which
    its libraries reach through NEEDED "libamdhip64.so" (bare name) and RPATH $ORIGIN.  If
    this library loads first, a later `import torch` maps the wheel's runtimes beside the
    system's: two HIP/HSA runtimes in one process, torch sees no device and the RCCL gathers
    (pta.gather_rows, gridutils.gather_blocks) cannot start.  If torch's runtime is the one
    shared, its asynchronous device->host copies blocked the host ~6-7 ms twice per process
    (inside pint_step_end's copy-stream work, measured; the system runtime: none).  So the
    system runtimes are loaded under the bare names the wheel's libraries ask for: their
    NEEDED entries then match the loaded objects by name and torch runs on the system
    runtime too.  (Loaded after torch, the names resolve to torch's runtime instead: still
    one runtime.)  PINT_HIP_RUNTIME=torch loads the wheel's runtime first instead; =none does
    nothing."""
    global HIP_RUNTIME
    mode = os.environ.get("PINT_HIP_RUNTIME", "system")
    if mode == "none":
        return
    if mode == "torch":
        import importlib.util
        try:
            spec = importlib.util.find_spec("torch")
        except (ImportError, ValueError):
            spec = None
        for d in (spec.submodule_search_locations if spec and spec.submodule_search_locations else []):
            p = os.path.join(d, "lib", "libamdhip64.so")
            if os.path.exists(p):
                C.CDLL(p, mode=C.RTLD_GLOBAL)
                HIP_RUNTIME = p
                return
        return
    for name in ("librocprofiler-register.so", "libhsa-runtime64.so", "libamdhip64.so"):
        try:
            C.CDLL(name, mode=C.RTLD_GLOBAL)
        except OSError:
            return  # (not on the search path: libpint_hip.so's own RUNPATH decides)
    HIP_RUNTIME = "system"


def lib():
    """Load libpint_hip.so (build with ``python -c 'import __graft_entry__ as g; g.build()'``)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIBPATH):
        raise RuntimeError(f"HIP extension missing: {LIBPATH} (run __graft_entry__.build())")
    _one_hip_runtime()
    L = C.CDLL(LIBPATH)
    vp = C.c_void_p
    L.pint_ctx_create.restype = vp
    L.pint_ctx_create.argtypes = [C.c_int]
    L.pint_ctx_destroy.argtypes = [vp]
    L.pint_last_error.restype = C.c_char_p
    L.pint_last_error.argtypes = [vp]
    L.pint_release_cache.restype = None
    L.pint_release_cache.argtypes = []
    L.pint_device_count.restype = C.c_int
    L.pint_nslot.restype = C.c_int
    L.pint_nslot.argtypes = []
    global NSLOT
    NSLOT = int(L.pint_nslot())  # the library's compile-time slot count, not an environment guess
    L.pint_add_pulsar.argtypes = [vp, C.POINTER(ToasT), C.POINTER(SpecT), dptr, dptr]
    L.pint_add_pulsar_cols.argtypes = [vp, C.POINTER(ToaColsT), C.POINTER(SpecT), dptr, dptr]
    L.pint_pack_toas.restype = C.c_int64
    L.pint_pack_toas.argtypes = [C.POINTER(ToaColsT), C.POINTER(ToasT), C.POINTER(C.c_int32), C.c_int64]
    L.pint_set_instances.argtypes = [vp, C.c_int, C.POINTER(C.c_int32), dptr]
    L.pint_set_grid.argtypes = [vp, C.c_int, C.c_int, dptr, C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_int64),
                                C.POINTER(C.c_int64), dptr, C.c_int64]
    for fn in ("pint_get_tables", "pint_set_tables", "pint_read_designmatrix", "pint_chi2_gls", "pint_chi2_wls",
               "pint_last_timing"):
        getattr(L, fn).argtypes = [vp, dptr]
    L.pint_eval.argtypes = [vp, C.c_int]
    L.pint_fit_step.argtypes = [vp, C.c_int]
    L.pint_read_resids.argtypes = [vp, dptr, dptr, dptr]
    L.pint_read_eval.argtypes = [vp, dptr, dptr, dptr, dptr]
    L.pint_read_step.argtypes = [vp, dptr, dptr, dptr, dptr]
    L.pint_apply_step.argtypes = [vp, dptr]
    L.pint_apply_step_uniform.argtypes = [vp, C.c_double]
    L.pint_fit_step_apply.argtypes = [vp, C.c_int, C.c_double]
    L.pint_save_tables.argtypes = [vp]
    L.pint_restore_tables.argtypes = [vp]
    L.pint_sync.argtypes = [vp]
    L.pint_debug_read.argtypes = [vp, C.c_int, dptr]
    L.pint_set_lazy.argtypes = [vp, C.c_int]
    L.pint_set_option.argtypes = [vp, C.c_int, C.c_int]
    L.pint_query.argtypes = [vp, C.c_int]
    for fn in ("pint_capture_begin", "pint_capture_end", "pint_graph_launch"):
        getattr(L, fn).argtypes = [vp]
    L.pint_query.restype = C.c_int
    L.pint_fit_layout.argtypes = [vp, C.c_int, C.POINTER(C.c_int32)]
    L.pint_vgram_layout.argtypes = [vp, C.c_int, C.POINTER(C.c_int32)]
    L.pint_lognorm.argtypes = [vp, C.c_int, dptr]
    L.pint_solve_eig.argtypes = [vp, C.c_int, dptr, C.POINTER(C.c_int32), dptr, C.c_int]
    L.pint_host_alloc.restype = vp
    L.pint_host_alloc.argtypes = [C.c_size_t]
    L.pint_host_free.argtypes = [vp]
    L.pint_set_ecorr.argtypes = [vp, C.c_int, C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_int32), dptr]
    L.pint_check.argtypes = [vp]
    L.pint_step_end.argtypes = [vp, C.POINTER(C.c_int)]
    L.pint_fit_step_enqueue.argtypes = [vp, C.c_int, C.c_int, C.c_double] + [dptr] * 8 + [C.POINTER(C.c_int)]
    L.pint_check_step.argtypes = [vp, C.c_int]
    L.pint_inst_status.argtypes = [vp, C.POINTER(C.c_int32)]
    L.pint_noise_resids.argtypes = [vp, dptr, dptr]
    L.pint_noise_resids_dm.argtypes = [vp, dptr]
    L.pint_debug_gram.argtypes = [vp, C.c_int, dptr]
    L.pint_read_norms.argtypes = [vp, C.c_int, dptr]
    L.pint_debug_set_resids.argtypes = [vp, dptr]
    L.pint_set_resids.argtypes = [vp, dptr]
    L.pint_set_sigma.argtypes = [vp, C.c_int, dptr]
    L.pint_set_noise_weights.argtypes = [vp, C.c_int, dptr, dptr]
    L.pint_set_noise_classes.argtypes = [vp, C.c_int, C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_int32), dptr]
    L.pint_noise_lnlike.argtypes = [vp, C.POINTER(C.c_int32), dptr, dptr, dptr, dptr, dptr]
    _lib = L
    L.pint_set_wideband.argtypes = [vp, C.c_int, dptr, dptr, dptr, C.POINTER(C.c_uint64)]
    L.pint_dm_resids.argtypes = [vp, C.c_int, C.c_int, dptr, dptr]
    return L


EXPORTED = ["pint_ctx_create", "pint_ctx_destroy", "pint_last_error", "pint_release_cache", "pint_device_count", "pint_nslot", "pint_add_pulsar",
            "pint_set_instances", "pint_get_tables", "pint_set_tables", "pint_eval", "pint_read_resids",
            "pint_read_eval", "pint_read_designmatrix", "pint_fit_step", "pint_read_step", "pint_apply_step",
            "pint_chi2_gls", "pint_set_ecorr", "pint_last_timing", "pint_sync", "pint_debug_read", "pint_set_lazy", "pint_check",
            "pint_set_option", "pint_host_alloc", "pint_host_free",
            "pint_fit_layout", "pint_query", "pint_capture_begin", "pint_capture_end", "pint_graph_launch",
            "pint_vgram_layout", "pint_lognorm", "pint_solve_eig", "pint_step_end", "pint_check_step",
            "pint_inst_status", "pint_noise_resids", "pint_debug_gram", "pint_debug_set_resids",
            "pint_set_resids", "pint_set_sigma", "pint_set_noise_weights", "pint_set_noise_classes",
            "pint_noise_lnlike", "pint_noise_resids_dm", "pint_set_wideband", "pint_dm_resids", "pint_chi2_wls",
            "pint_apply_step_uniform", "pint_fit_step_apply", "pint_save_tables", "pint_restore_tables", "pint_read_norms",
            "pint_fit_step_enqueue", "pint_set_grid", "pint_add_pulsar_cols", "pint_pack_toas"]


def ptr(a: np.ndarray, ct=C.c_double):
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(ct))
