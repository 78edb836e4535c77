"""ctypes binding of libttk.so (the HIP C ABI, include/ttk.h).

The product path has no CPU fallback: importing this module on a machine without the built
library raises immediately, and every wrapper raises on a non-zero status."""
import ctypes
import os

import torch  # noqa: F401  -- load PyTorch's HIP runtime first so libttk binds to the same one

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TTK_LIB_PATH") or os.path.join(HERE, "libttk.so")  # override: diagnostics builds

if not os.path.exists(LIB_PATH):
    raise ImportError(f"libttk.so not found at {LIB_PATH}: run `python __graft_entry__.py build` "
                      "(hipcc --offload-arch=gfx950); the MI355X path has no CPU fallback")

lib = ctypes.CDLL(LIB_PATH)

c_dp = ctypes.POINTER(ctypes.c_double)
c_i64p = ctypes.POINTER(ctypes.c_int64)
c_ip = ctypes.POINTER(ctypes.c_int)
vp = ctypes.c_void_p
i32 = ctypes.c_int
i64 = ctypes.c_int64
f64 = ctypes.c_double

_SIGS = {
    "ttk_last_error": (ctypes.c_char_p, []),
    "ttk_version": (i32, []),
    "ttk_launch_count": (ctypes.c_longlong, []),
    "ttk_sync_count": (ctypes.c_longlong, []),
    "ttk_gemm_offs": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, f64, f64]),
    "ttk_gemm_offs_grouped": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, f64, f64]),
    "ttk_copy_nd": (i32, [vp, vp, vp, i32, c_i64p, c_i64p, c_i64p, f64, f64]),
    "ttk_mul_nd": (i32, [vp, vp, vp, vp, i32, c_i64p, c_i64p, c_i64p, c_i64p, f64, f64]),
    "ttk_recip": (i32, [vp, vp, vp, i64]),
    "ttk_tt_join": (i32, [vp, vp, vp, vp, i32, i32, i32, i32, i64, i32]),
    "ttk_axpby_nd": (i32, [vp, vp, vp, vp, i32, c_i64p, c_i64p, c_i64p, c_i64p, f64, f64, f64]),
    "ttk_scale_axis_ss": (i32, [vp, vp, vp, i32, c_i64p, c_i64p, c_i64p, i32, vp, i32]),
    "ttk_normalize": (i32, [vp, vp, vp, i32, c_i64p, c_i64p]),
    "ttk_rayleigh_tail_sync": (i32, [vp, vp, vp, i64, c_dp, c_dp]),
    "ttk_rayleigh_tail_dev": (i32, [vp, vp, vp, i64, vp]),
    "ttk_scale_axis": (i32, [vp, vp, vp, i32, c_i64p, c_i64p, c_i64p, i32, c_dp]),
    "ttk_fill": (i32, [vp, vp, i64, f64]),
    "ttk_add_diag": (i32, [vp, vp, i32, i32, f64]),
    "ttk_dot_nd_sync": (i32, [vp, vp, vp, i32, c_i64p, c_i64p, c_i64p, c_dp]),
    "ttk_dot_nd_dev": (i32, [vp, vp, vp, i32, c_i64p, c_i64p, c_i64p, vp]),
    "ttk_sumsq_batched": (i32, [vp, vp, i64, i32, i64, vp]),
    "ttk_sumsq_batched_strided": (i32, [vp, vp, i64, i32, i64, i64, i64, vp]),
    "ttk_read_sync": (i32, [vp, vp, c_dp, i64]),
    "ttk_upload": (i32, [vp, vp, vp, i64]),
    "ttk_svd_work": (i64, [i32, i32]),
    "ttk_svd": (i32, [vp, vp, i32, i32, vp, vp, vp, vp]),
    "ttk_qr_work": (i64, [i32, i32]),
    "ttk_qr": (i32, [vp, vp, i32, i32, vp, vp, vp]),
    "ttk_cholesky_sync": (i32, [vp, vp, i32]),
    "ttk_dense_set_block_min": (i32, [i32]),
    "ttk_trsm_lower": (i32, [vp, vp, i32, vp, i32, i32, i32]),
    "ttk_lu_sync": (i32, [vp, vp, i32, vp, vp, c_dp]),
    "ttk_lu_solve": (i32, [vp, vp, i32, vp, vp, i32, i32]),
    "ttk_syev_work": (i64, [i32]),
    "ttk_syev": (i32, [vp, vp, i32, vp, vp, vp]),
    "ttk_syev_extreme_work": (i64, [i32]),
    "ttk_syev_set_small": (i32, [i32]),
    "ttk_syev_set_fused_max": (i32, [i32]),
    "ttk_debug_counters": (i32, [vp, i32]),
    "ttk_svd_set_timing": (i32, [i32]),
    "ttk_svd_set_big_threshold": (i32, [i32]),
    "ttk_svd_tol": (i32, [vp, vp, i32, i32, vp, vp, vp, vp, f64]),
    "ttk_svd_tol_read": (i32, [vp, vp, i32, i32, vp, vp, vp, vp, f64, c_dp]),
    "ttk_einsum": (i32, [vp, ctypes.c_char_p, vp, vp, f64, f64]),
    "ttk_einsum_stats": (i32, [vp]),
    "ttk_einsum_batch_begin": (i32, [vp]),
    "ttk_einsum_batch_flush": (i32, [vp]),
    "ttk_einsum_batch_end": (i32, [vp]),
    "ttk_einsum_batch_stats": (i32, [vp]),
    "ttk_rank_scan_sync": (i32, [vp, vp, vp, i64, i32, vp]),
    "ttk_ctx_create": (i32, [vp, vp]),
    "ttk_ctx_destroy": (i32, [vp]),
    "ttk_ctx_bind": (i32, [vp]),
    "ttk_ctx_stream": (vp, [vp]),
    "ttk_lgmres": (i32, [vp, i64, vp, vp, i64, i32, i32, f64, i32, i32, vp]),
    "ttk_env_update": (i32, [vp, i32, i32, vp]),
    "ttk_round": (i32, [vp, i32, vp, vp, vp, f64, i32, vp]),
    "ttk_zipup": (i32, [vp, i32, i32, vp, vp, vp, vp, vp, f64, vp, vp]),
    "ttk_dense_schur_solve": (i32, [vp, i64, i64, i64, vp, vp, vp, vp, vp]),
    "ttk_dense_schur_solve_ineq": (i32, [vp, i64, i64, i64, vp, vp, vp, vp]),
    "ttk_fused_set_mfma": (i32, [i32]),
    "ttk_mfma_profile": (i32, [vp, i32]),
    "ttk_dep_timeouts": (i32, [vp, i32]),
    "ttk_einsum_set_fused": (i32, [i32]),
    "ttk_qr_set_big_threshold": (i32, [i32]),
    "ttk_contract_timing": (i32, [i32]),
    "ttk_gemm_hist": (i32, [i32, ctypes.c_char_p]),
    "ttk_linalg_hist": (i32, [i32, ctypes.c_char_p]),
    "ttk_gemm_set_splitk": (i32, [i32]),
    "ttk_contract_stats": (i32, [vp, i32]),
    "ttk_syev_extreme": (i32, [vp, vp, i32, i32, vp, vp, vp]),
    "ttk_copy_many": (i32, [vp, i32, vp, vp, vp]),
    "ttk_lgmres_arnoldi_sync": (i32, [vp, vp, i32, i32, vp, i32, f64, c_dp, c_ip]),
    "ttk_schur_build": (i32, [vp, i32, i64, c_i64p, vp, c_i64p]),
    "ttk_schur_apply": (i32, [vp, i64, vp, vp]),
    "ttk_schur_free": (i32, [vp, i64]),
    "ttk_ctx_set_knob": (i32, [vp, i32, i32, c_ip]),
    "ttk_ctx_get_knob": (i32, [vp, i32, c_ip]),
    "ttk_lgmres_arnoldi_async": (i32, [vp, vp, i32, i32, vp, i32, f64, f64, f64, vp, i32, f64]),
    "ttk_lgmres_chunk": (i32, [vp, i64, vp, i32, i32, i32, vp, i32, f64, f64, f64, vp, f64]),
    "ttk_lgmres_build": (i32, [vp, vp, i32, i32, ctypes.POINTER(vp), i32, i32, vp, vp]),
    "ttk_lgmres_aug": (i32, [vp, vp, i32, i32, vp, i32, f64, vp, vp, vp]),
    "ttk_lgmres_set_mw_threshold": (i32, [i32]),
}

# Entry points that wait for the device (a stream synchronisation or a blocking copy inside): they
# release the GIL while they wait, so another solve thread of the process runs its host code then.
BLOCKING = frozenset(n for n in _SIGS if "sync" in n) | frozenset((
    "ttk_lgmres", "ttk_round", "ttk_zipup", "ttk_svd_tol_read", "ttk_dense_schur_solve", "ttk_dense_schur_solve_ineq",
    "ttk_lgmres_chunk", "ttk_lgmres_build", "ttk_lgmres_aug", "ttk_schur_build", "ttk_schur_free",
    "ttk_ctx_create", "ttk_ctx_destroy", "ttk_upload", "ttk_dep_timeouts", "ttk_debug_counters",
    "ttk_mfma_profile", "ttk_contract_stats", "ttk_gemm_hist", "ttk_linalg_hist"))
# Every other (launch-only, microseconds) entry point keeps the GIL (ctypes.PyDLL calling
# convention; TTK_HOLD_GIL=0 releases it on every call, as plain ctypes does).  A thread that drops
# the GIL for a 3 us launch and takes it straight back makes a second solve thread of the process
# wait for the GIL hand-over on every launch; holding it, the threads switch where one of them
# waits for the device (2 slot threads of one process,
# maxcut_10 s41 + s235: whole job 0.153 -> 0.141 s/IPM-iter, 0.130 with a 0.5 ms switch interval;
# profiles/r04_slot_threads.txt).
_held = ctypes.PyDLL(LIB_PATH) if os.environ.get("TTK_HOLD_GIL", "1") == "1" else None
# the same entry points, every one releasing the GIL: for calls whose host side is itself long
# (e.g. the eigensolver's one launch per Householder reflector at n > 128, dev.syev_extreme)
lib_release = ctypes.CDLL(LIB_PATH) if _held is not None else lib

for _name, (_res, _args) in _SIGS.items():
    if os.environ.get("TTK_LIB_PATH") and not hasattr(lib, _name):
        continue  # diagnostics: an older build loaded for a bit-identity comparison
    _f = getattr(_held if _held is not None and _name not in BLOCKING else lib, _name)
    _f.restype = _res
    _f.argtypes = _args
    if _held is not None and _name not in BLOCKING:
        setattr(lib, _name, _f)
        _g = getattr(lib_release, _name)
        _g.restype = _res
        _g.argtypes = _args

EXPORTED = tuple(_SIGS)

TTK_OK, TTK_ERR_ARG, TTK_ERR_HIP, TTK_ERR_NOT_PD, TTK_ERR_SINGULAR, TTK_ERR_NOT_CONVERGED = range(6)
# per-context numerics knobs (include/ttk.h enum ttk_knob)
(KNOB_FUSED_APPLY, KNOB_FUSED_MFMA, KNOB_SPLITK, KNOB_SPLITK_MINK, KNOB_LGMRES_MW_MIN, KNOB_MFMA_CSPLIT, KNOB_APPLY_DUAL,
 KNOB_RCOND_EXACT, KNOB_SCHUR_ONE, KNOB_ARNOLDI_ONE, KNOB_SCHUR_PREP, KNOB_SPLITK_FUSED, KNOB_TRI_HOIST,
 KNOB_TRI_ONE, KNOB_SVD_SWEEP_ONE, KNOB_TRI_PERSIST, KNOB_SYEV_WAVES8, KNOB_BT_STAGE) = range(18)


class TTKError(RuntimeError):
    pass


class LinAlgError(ValueError):
    """Raised where LAPACK/SciPy would raise scipy.linalg.LinAlgError (potrf/getrf failure)."""


class LinAlgWarning(RuntimeWarning):
    """Raised (as an exception, like the reference's warnings-as-errors, src/tt_ipm.py:16) where
    scipy.linalg.solve would warn about an ill-conditioned matrix."""


def check(status, what=""):
    if status == TTK_OK:
        return
    msg = lib.ttk_last_error().decode(errors="replace")
    if status == TTK_ERR_NOT_PD:
        raise LinAlgError(msg)
    if status == TTK_ERR_SINGULAR:
        raise LinAlgError(msg)
    raise TTKError(f"{what}: status {status}: {msg}")
