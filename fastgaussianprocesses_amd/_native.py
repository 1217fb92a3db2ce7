"""ctypes binding of the C-ABI library libfgp_hip.so (include/fgp_hip.h).

The library is built in-tree by `python -m fastgaussianprocesses_amd.build` (or
__graft_entry__.build()) into fastgaussianprocesses_amd/_lib/.  There is no fallback: if the
library is missing or a call fails, a RuntimeError is raised.
"""
import ctypes
import os
import threading

import torch

_LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
LIB_PATH = os.environ.get("FGP_LIB_PATH") or os.path.join(_LIB_DIR, "libfgp_hip.so")   # override: experiments
ABI_VERSION = 18
MT_MAX_TASKS = 16
MAX_D = 8
PARTS_ARRAY = 0
PARTS_LATTICE = 1

_lock = threading.Lock()
_lib = None

_c_i64 = ctypes.c_int64
_c_int = ctypes.c_int
_c_dbl = ctypes.c_double
_c_vp = ctypes.c_void_p

_c_pi = ctypes.POINTER(ctypes.c_int)
_c_pd = ctypes.POINTER(ctypes.c_double)
_c_pl = ctypes.POINTER(ctypes.c_int64)


class NllDesc(ctypes.Structure):
    """Mirror of fgp_nll_desc (include/fgp_hip.h)."""
    _fields_ = [
        ("family", _c_int), ("log2n", _c_int), ("d", _c_int), ("G", _c_int),
        ("parts", _c_vp), ("parts_stride", _c_i64),
        ("ysq", _c_vp), ("ysq_stride", _c_i64),
        ("raw", _c_vp),
        ("scale_off", _c_int), ("scale_pp", _c_int),
        ("ls_off", _c_int), ("ls_pp", _c_int), ("ls_pd", _c_int),
        ("noise_off", _c_int), ("noise_pp", _c_int),
        ("logdet_weight", _c_dbl),
        ("grad_lam", _c_vp), ("work", _c_vp), ("partials", _c_vp),
        ("parts_gen", _c_int), ("gen_order", _c_int * 8), ("gen_coef", _c_dbl * 8), ("gen_z", _c_i64 * 8),
        ("gen_shift", _c_vp), ("gen_shift_stride", _c_i64),
        ("stamps", _c_vp),
        ("basis", _c_vp), ("basis_stride", _c_i64), ("ysq_chunked", _c_int),
        ("mt_tasks", _c_int), ("mt_basis", _c_vp), ("mt_ytilde", _c_vp), ("mt_kt", _c_vp),
        ("loss_metric", _c_int), ("cv_weight", _c_dbl),
        ("mt_task_rg", _c_int), ("mt_rank", _c_int), ("mt_vexp", _c_int),
    ]


LOSS_MLL, LOSS_GCV, LOSS_CV = 0, 1, 2       # fgp_nll_desc.loss_metric (include/fgp_hip.h, ABI 16)


class FitDesc(ctypes.Structure):
    """Mirror of fgp_fit_desc (include/fgp_hip.h)."""
    _fields_ = [
        ("n_params", _c_int),
        ("raw", _c_vp), ("rprop_prev", _c_vp), ("rprop_step", _c_vp), ("grad_out", _c_vp),
        ("loss_hist", _c_vp), ("raw_hist", _c_vp),
        ("scale_rg", _c_int), ("ls_rg", _c_int), ("noise_rg", _c_int),
        ("mll_const", _c_dbl), ("eta_minus", _c_dbl), ("eta_plus", _c_dbl),
        ("step_min", _c_dbl), ("step_max", _c_dbl),
        ("per_problem", _c_int),
        ("hist_stride", _c_int), ("hist_offset", _c_int),
    ]


class PredDesc(ctypes.Structure):
    """Mirror of fgp_pred_desc (include/fgp_hip.h)."""
    _fields_ = [
        ("family", _c_int), ("d", _c_int), ("tbits", _c_int), ("P", _c_int), ("n", _c_i64),
        ("order", _c_int * 8), ("coef", _c_dbl * 8),
        ("z", _c_vp), ("z_stride", _c_i64), ("hyp", _c_vp), ("hyp_stride", _c_i64),
        ("coeffs", _c_vp), ("coeff_stride", _c_i64), ("wa", _c_vp), ("wa_stride", _c_i64),
        ("points_gen", _c_int), ("gen_z", _c_i64 * 8), ("gen_shift", _c_vp), ("gen_shift_stride", _c_i64),
    ]


class MtLayout(ctypes.Structure):
    """Mirror of fgp_mt_layout (include/fgp_hip.h)."""
    _fields_ = [("T", _c_int), ("n", _c_i64 * 16)]


class MtFitDesc(ctypes.Structure):
    """Mirror of fgp_mt_fit_desc (include/fgp_hip.h, ABI 14; parameter batches and the adaptive nugget ABI 16)."""
    _fields_ = [
        ("family", _c_int), ("d", _c_int), ("B", _c_int),
        ("layout", MtLayout), ("task", _c_int * 16),
        ("T_all", _c_int), ("rank", _c_int), ("dl", _c_int),
        ("spectra", _c_vp), ("spec_off", _c_i64 * 136), ("y", _c_vp), ("raw", _c_vp),
        ("vtask_exp", _c_int),
        ("rg_scale", _c_int), ("rg_ls", _c_int), ("rg_noise", _c_int), ("rg_factor", _c_int), ("rg_vtask", _c_int),
        ("rprop_prev", _c_vp), ("rprop_step", _c_vp), ("grad_out", _c_vp), ("loss_hist", _c_vp), ("raw_hist", _c_vp),
        ("grad_norm", _c_dbl), ("grad_logdet", _c_dbl),
        ("logdet_weight", _c_dbl), ("mll_const", _c_dbl), ("eta_minus", _c_dbl), ("eta_plus", _c_dbl),
        ("step_min", _c_dbl), ("step_max", _c_dbl),
        ("work", _c_vp),
        ("G", _c_int), ("rows", _c_vp), ("nrows", _c_int * 5),
        ("nugget_coef", _c_vp), ("nugget_ref", _c_int),
    ]


_P_NLL = ctypes.POINTER(NllDesc)
_P_MTFIT = ctypes.POINTER(MtFitDesc)
_P_MT = ctypes.POINTER(MtLayout)
_P_FIT = ctypes.POINTER(FitDesc)
_P_PRED = ctypes.POINTER(PredDesc)

# name -> argtypes (all return int status); must match include/fgp_hip.h
_SIGNATURES = {
    "fgp_init": [_c_vp],
    "fgp_wall_clock_khz": [_c_int, _c_pi],
    "fgp_clock_stamp": [_c_vp, _c_vp],
    "fgp_fftbr": [_c_vp, _c_i64, _c_int, _c_vp, _c_i64, _c_int, _c_int, _c_vp],
    "fgp_ifftbr": [_c_vp, _c_i64, _c_vp, _c_int, _c_vp, _c_i64, _c_int, _c_int, _c_vp],
    "fgp_fwht": [_c_vp, _c_i64, _c_vp, _c_i64, _c_int, _c_int, _c_vp],
    "fgp_fftbr_real": [_c_vp, _c_i64, _c_vp, _c_vp, _c_i64, _c_int, _c_vp],
    "fgp_ifftbr_real": [_c_vp, _c_i64, _c_vp, _c_i64, _c_vp, _c_i64, _c_vp, _c_i64, _c_int, _c_vp],
    "fgp_ifftbr_real_rf": [_c_vp, _c_i64, _c_vp, _c_i64, _c_vp, _c_i64, _c_vp, _c_i64, _c_int, _c_vp],
    "fgp_fftbr_c64": [_c_vp, _c_i64, _c_int, _c_vp, _c_i64, _c_int, _c_int, _c_vp],
    "fgp_ifftbr_c64": [_c_vp, _c_i64, _c_vp, _c_int, _c_vp, _c_i64, _c_int, _c_int, _c_vp],
    "fgp_fwht_f32": [_c_vp, _c_i64, _c_vp, _c_i64, _c_int, _c_int, _c_vp],
    "fgp_ifftbr_mul": [_c_int, _c_int, _c_vp, _c_i64, _c_vp, _c_i64, _c_vp, _c_int, _c_vp, _c_i64, _c_int, _c_int,
                       _c_vp],
    "fgp_sum_sq": [_c_vp, _c_i64, _c_int, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp],
    "fgp_lattice_parts": [_c_vp, _c_i64, _c_vp, _c_i64, _c_int, _c_pi, _c_pd, _c_vp, _c_vp],
    "fgp_lattice_points": [_c_pl, _c_vp, _c_i64, _c_i64, _c_int, _c_vp, _c_vp],
    "fgp_lattice_parts_gen": [_c_pl, _c_vp, _c_int, _c_int, _c_int, _c_pd, _c_vp, _c_vp],
    "fgp_net_parts": [_c_vp, _c_i64, _c_vp, _c_i64, _c_int, _c_int, _c_vp, _c_vp, _c_vp],
    "fgp_nll_fwd": [_P_NLL, _c_vp],
    "fgp_nll_bwd": [_P_NLL, _c_vp],
    "fgp_nll_lam": [_P_NLL, _c_vp],
    "fgp_spec_inv_eig": [_P_NLL, _c_vp, _c_vp],
    "fgp_spec_post_var": [_P_NLL, _c_vp, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp],
    "fgp_nll_stage": [_P_NLL, _c_int, _c_vp],
    "fgp_post_var_qf": [_c_int, _c_vp, _c_i64, _c_vp, _c_int, _c_int, _c_int, _c_pi, _c_pd, _c_vp, _c_vp, _c_vp,
                        _c_vp, _c_vp, _c_vp],
    "fgp_fit_step": [_P_NLL, _P_FIT, _c_int, _c_int, _c_vp],
    "fgp_fit_run": [_P_NLL, _P_FIT, _c_int, _c_int, _c_int, _c_vp],
    "fgp_post_mean": [_c_int, _c_vp, _c_i64, _c_vp, _c_i64, _c_int, _c_int, _c_pi, _c_pd, _c_vp, _c_int, _c_vp,
                      _c_i64, _c_int, _c_vp, _c_i64, _c_vp, _c_i64, _c_vp],
    "fgp_kernel_rows": [_c_int, _c_vp, _c_i64, _c_vp, _c_i64, _c_int, _c_int, _c_pi, _c_pd, _c_vp, _c_int, _c_vp,
                        _c_vp],
    "fgp_post_mean_batched": [_P_PRED, _c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp],
    "fgp_post_mean_batched_work": [_P_PRED, _c_i64, _c_pl],
    "fgp_post_var_batched": [_P_PRED, _c_vp, _c_i64, _c_i64, _c_pd, _c_vp, _c_vp, _c_vp, _c_vp],
    "fgp_net_points": [_c_vp, _c_int, _c_vp, _c_i64, _c_i64, _c_int, _c_int, _c_vp, _c_vp, _c_vp],
    "fgp_double_update": [_c_int, _c_vp, _c_i64, _c_vp, _c_i64, _c_i64, _c_int, _c_vp, _c_i64, _c_vp],
    "fgp_mt_parts": [_c_int, _c_vp, _c_i64, _c_i64, _c_vp, _c_i64, _c_i64, _c_int, _c_int, _c_int, _c_vp, _c_vp,
                     _c_vp, _c_int, _c_vp, _c_vp],
    "fgp_mt_factor": [_P_MT, _c_vp, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp],
    "fgp_mt_solve": [_P_MT, _c_vp, _c_i64, _c_vp, _c_i64, _c_i64, _c_vp, _c_vp],
    "fgp_mt_selinv": [_P_MT, _c_vp, _c_i64, _c_vp, _c_vp],
    "fgp_mt_mll_grad": [_P_MT, _c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_i64, _c_vp, _c_vp],
    "fgp_fftbr_real_half": [_c_vp, _c_i64, _c_vp, _c_i64, _c_vp, _c_i64, _c_int, _c_vp],
    "fgp_fftbr_real_half_f32": [_c_vp, _c_i64, _c_vp, _c_i64, _c_vp, _c_i64, _c_int, _c_vp],
    "fgp_sum_sq_half": [_c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp],
    "fgp_fit_persist_ok": [_P_NLL, _c_pi],
    "fgp_fit_persist": [_P_NLL, _P_FIT, _c_int, _c_dbl, _c_int, _c_vp, _c_vp],
    "fgp_mt_fit_nparams": [_P_MTFIT, _c_pi],
    "fgp_mt_fit_work": [_P_MTFIT, _c_pl],
    "fgp_mt_fit_run": [_P_MTFIT, _c_int, _c_int, _c_int, _c_vp],
    "fgp_handoff_check": [_c_int, ctypes.POINTER(ctypes.c_ulonglong)],
    "fgp_set_persist_poll_max": [_c_i64],
    "fgp_persist_giveups": [ctypes.POINTER(ctypes.c_ulonglong), _c_int],
    "fgp_fit_graph_stats": [ctypes.POINTER(ctypes.c_longlong)],
    "fgp_fit_run_graph": [_P_NLL, _P_FIT, _c_int, _c_int, _c_int, _c_i64, _c_vp],
    "fgp_fit_graph_release": [_c_i64],
    "fgp_set_mt_class_kernel": [_c_int],
    "fgp_nll_partials_len": [_P_NLL, _c_pl],
    "fgp_spec_basis": [_c_int, _c_vp, _c_i64, _c_i64, _c_int, _c_int, _c_vp, _c_vp, _c_i64, _c_vp],
    "fgp_spec_basis_work": [_c_int, _c_int, _c_int, _c_pl],
    "fgp_spec_basis_gen": [_c_pl, _c_int, _c_int, _c_int, _c_pd, _c_vp, _c_vp, _c_i64, _c_vp],
    "fgp_inv_eig": [_c_int, _c_vp, _c_vp, _c_i64, _c_vp, _c_i64, _c_i64, _c_int, _c_vp, _c_vp, _c_vp],
}


def int_array(vals):
    return (ctypes.c_int * max(1, len(vals)))(*[int(v) for v in vals])


def int64_array(vals):
    return (ctypes.c_int64 * max(1, len(vals)))(*[int(v) for v in vals])


def double_array(vals):
    return (ctypes.c_double * max(1, len(vals)))(*[float(v) for v in vals])


def _load():
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.isfile(LIB_PATH):
            raise RuntimeError(
                "fastgaussianprocesses_amd: native library %s is missing; build it with "
                "`python -m fastgaussianprocesses_amd.build` (hipcc, gfx950). There is no CPU fallback." % LIB_PATH)
        lib = ctypes.CDLL(LIB_PATH)
        lib.fgp_last_error.restype = ctypes.c_char_p
        lib.fgp_abi_version.restype = ctypes.c_int
        if lib.fgp_abi_version() != ABI_VERSION:
            raise RuntimeError("libfgp_hip.so ABI version %d != expected %d; rebuild"
                               % (lib.fgp_abi_version(), ABI_VERSION))
        for name, argt in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argt
            fn.restype = ctypes.c_int
        _lib = lib
        return lib


def lib():
    return _lib if _lib is not None else _load()


def exported_symbols():
    return ["fgp_abi_version", "fgp_last_error"] + list(_SIGNATURES.keys())


def call(name, *args):
    """Invoke a C-ABI entry point; raise RuntimeError with the library's message on failure."""
    L = lib()
    rc = getattr(L, name)(*args)
    if rc != 0:
        msg = L.fgp_last_error().decode(errors="replace")
        raise RuntimeError("%s failed (%d): %s" % (name, rc, msg))
    return rc


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device):
    """The current HIP stream of `device` (torch's raw-stream query: ~1 us instead of the ~7 us of building a
    torch.cuda.Stream object per call)."""
    if _RAW_STREAM is not None:
        idx = device.index if isinstance(device, torch.device) and device.index is not None else \
            torch.cuda.current_device() if not isinstance(device, int) else device
        return ctypes.c_void_p(_RAW_STREAM(idx))
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def byref_layout(lay):
    return ctypes.byref(lay)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)
