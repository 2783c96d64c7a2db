"""ctypes binding of libmpvae_hip.so (C ABI: include/mpvae_hip.h).

The library is loaded from this directory, after ``import torch`` so that the
HIP runtime torch already loaded is the one the kernels register with (both
share the SONAME libamdhip64.so.7).  There is deliberately no fallback: if the
library is missing or the device is not a GPU, every entry point raises.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the .so load: one HIP runtime per process)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MPVAE_HIP_LIB", os.path.join(HERE, "libmpvae_hip.so"))

ABI_VERSION = 10
F32, F64 = 0, 1
G_TOTAL, G_NLL, G_NLL_X, G_C, G_C_X, G_KL = range(6)

c_float_p = ctypes.POINTER(ctypes.c_float)
vp = ctypes.c_void_p


class MPVError(RuntimeError):
    """An MPV_E* status returned by libmpvae_hip.so."""


class Shape(ctypes.Structure):
    _fields_ = [("S_local", ctypes.c_int64), ("S_total", ctypes.c_int64),
                ("s_offset", ctypes.c_int64), ("B", ctypes.c_int64), ("L", ctypes.c_int64),
                ("z", ctypes.c_int64)]


class Split16(ctypes.Structure):
    """mpv_split16: chunked hi/lo planes (include/mpvae_hip.h)."""
    _fields_ = [("data", vp), ("scale", vp), ("rows_pad", ctypes.c_int64),
                ("ld", ctypes.c_int64)]


GEMM_F16X3, GEMM_F32 = 0, 1


class FwdArgs(ctypes.Structure):
    _fields_ = [("y", vp), ("fe_out", vp), ("fx_out", vp), ("gemm", ctypes.c_int), ("R32", vp),
                ("eps", vp), ("R16", Split16), ("eps16", Split16), ("T", vp), ("rowstat", vp),
                ("bstat", vp), ("colsum", vp), ("workspace", vp),
                ("workspace_bytes", ctypes.c_size_t)]


class FinalArgs(ctypes.Structure):
    _fields_ = [("bstat", vp), ("colsum", vp), ("fe_mu", vp), ("fe_logvar", vp), ("fx_mu", vp),
                ("fx_logvar", vp), ("d", ctypes.c_int64), ("nll_coeff", ctypes.c_float),
                ("c_coeff", ctypes.c_float), ("total", vp), ("nll", vp), ("nll_x", vp),
                ("c", vp), ("c_x", vp), ("kl", vp), ("indiv_prob", vp),
                ("indiv_prob_label", vp), ("seed_advance", vp)]


class BwdArgs(ctypes.Structure):
    _fields_ = [("y", vp), ("fe_out", vp), ("fx_out", vp), ("gemm", ctypes.c_int), ("eps", vp),
                ("eps16", Split16), ("T", vp),
                ("rowstat", vp), ("bstat", vp), ("gscal", vp), ("g_indiv", vp),
                ("g_indiv_label", vp), ("nll_coeff", ctypes.c_float),
                ("c_coeff", ctypes.c_float), ("live", ctypes.c_int), ("dfe_dfx", vp),
                ("dR32", vp), ("workspace", vp), ("workspace_bytes", ctypes.c_size_t),
                ("dR64", vp), ("kl", vp)]


class KlBwdArgs(ctypes.Structure):
    _fields_ = [("fe_mu", vp), ("fe_logvar", vp), ("fx_mu", vp), ("fx_logvar", vp),
                ("B", ctypes.c_int64), ("d", ctypes.c_int64), ("gscal", vp), ("g_fe_mu", vp),
                ("g_fe_logvar", vp), ("g_fx_mu", vp), ("g_fx_logvar", vp), ("live", ctypes.c_int)]


class ReparamArgs(ctypes.Structure):
    _fields_ = [("mu_e", vp), ("logvar_e", vp), ("eps_e", vp), ("z_e", vp), ("n_e", ctypes.c_int64),
                ("mu_x", vp), ("logvar_x", vp), ("eps_x", vp), ("z_x", vp), ("n_x", ctypes.c_int64),
                ("mu_e_out", vp), ("logvar_e_out", vp), ("mu_x_out", vp), ("logvar_x_out", vp)]


class ReparamBwdArgs(ctypes.Structure):
    _fields_ = [("gz_e", vp), ("logvar_e", vp), ("eps_e", vp), ("gmu_e", vp), ("glogvar_e", vp),
                ("n_e", ctypes.c_int64), ("gz_x", vp), ("logvar_x", vp), ("eps_x", vp),
                ("gmu_x", vp), ("glogvar_x", vp), ("n_x", ctypes.c_int64),
                ("gmu_add_e", vp), ("glogvar_add_e", vp), ("gmu_add_x", vp),
                ("glogvar_add_x", vp)]


class LabelTable(ctypes.Structure):
    """mpv_label_table: packed 0/1 label patterns -> distance (fairness.hip)."""
    _fields_ = [("keys", vp), ("vals", vp), ("used", vp), ("nslots", ctypes.c_int64),
                ("W", ctypes.c_int64)]


FAIR_L1, FAIR_L2 = 1, 2


class LinearArgs(ctypes.Structure):
    """mpv_linear_args: one fp32 matrix-core GEMM with a fused epilogue (linear.hip)."""
    _fields_ = [("M", ctypes.c_int64), ("N", ctypes.c_int64), ("R", ctypes.c_int64),
                ("a", vp), ("a_si", ctypes.c_int64), ("a_sr", ctypes.c_int64), ("a_mask", vp),
                ("a_scale", ctypes.c_float), ("b", vp), ("b_sj", ctypes.c_int64),
                ("b_sr", ctypes.c_int64), ("ones_col", ctypes.c_int64), ("bias", vp),
                ("alpha", ctypes.c_float), ("relu", ctypes.c_int), ("out", vp),
                ("out_si", ctypes.c_int64), ("out_col", vp), ("a2", vp),
                ("a2_si", ctypes.c_int64), ("b2", vp), ("R1", ctypes.c_int64)]


ADAM_MAX_TENSORS = 32


class AdamTensor(ctypes.Structure):
    _fields_ = [("param", vp), ("grad", vp), ("exp_avg", vp), ("exp_avg_sq", vp), ("step", vp),
                ("numel", ctypes.c_int64), ("is_f64", ctypes.c_int)]


class AdamArgs(ctypes.Structure):
    """mpv_adam_args: one Adam update over up to 32 tensors (adam.hip)."""
    _fields_ = [("n", ctypes.c_int), ("t", AdamTensor * ADAM_MAX_TENSORS),
                ("lr", ctypes.c_double), ("beta1", ctypes.c_double), ("beta2", ctypes.c_double),
                ("weight_decay", ctypes.c_double), ("eps", ctypes.c_double),
                ("found_inf", vp), ("lr_dev", vp)]


ADAM_FINISH_MAX = 256


class AdamFinishArgs(ctypes.Structure):
    """mpv_adam_finish_args: step counts, update counter and StepLR (adam.hip)."""
    _fields_ = [("n_steps", ctypes.c_int), ("steps", vp * ADAM_FINISH_MAX), ("found_inf", vp),
                ("updates", vp), ("n_lr", ctypes.c_int), ("lr", vp), ("last_epoch", vp),
                ("step_size", ctypes.c_double), ("gamma", ctypes.c_double)]


class FairArgs(ctypes.Structure):
    _fields_ = [("label_z", vp), ("feat_z", vp), ("w", vp), ("order", vp), ("goff", vp),
                ("gid", vp), ("B", ctypes.c_int64), ("L", ctypes.c_int64), ("T", ctypes.c_int64),
                ("G", ctypes.c_int64), ("norm", ctypes.c_int), ("fair_coeff", ctypes.c_double),
                ("out", vp)]


# name -> (restype, argtypes); exactly the symbols of include/mpvae_hip.h
SIGNATURES = {
    "mpv_abi_version": (ctypes.c_int, []),
    "mpv_last_error": (ctypes.c_char_p, []),
    "mpv_noise_philox": (ctypes.c_int, [vp, ctypes.POINTER(Shape), ctypes.c_uint64,
                                        ctypes.c_uint64, vp]),
    "mpv_philox_raw": (ctypes.c_int, [vp, ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint64, vp]),
    "mpv_convert": (ctypes.c_int, [vp, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int64, vp]),
    "mpv_split_workspace_bytes": (ctypes.c_size_t, []),
    "mpv_noise_plane_cols": (ctypes.c_int64, [ctypes.POINTER(Shape)]),
    "mpv_split_f16": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                                     ctypes.POINTER(Split16), vp, vp]),
    "mpv_noise_philox_f16": (ctypes.c_int, [ctypes.POINTER(Shape), ctypes.c_uint64,
                                            ctypes.c_uint64, ctypes.POINTER(Split16), vp]),
    "mpv_noise_philox_dev": (ctypes.c_int, [vp, ctypes.POINTER(Shape), vp, ctypes.c_uint64, vp]),
    "mpv_noise_philox_f16_dev": (ctypes.c_int, [ctypes.POINTER(Shape), vp, ctypes.c_uint64,
                                                ctypes.POINTER(Split16), vp]),
    "mpv_noise_philox_f16_split": (ctypes.c_int, [ctypes.POINTER(Shape), ctypes.c_uint64, vp,
                                                  ctypes.c_uint64, ctypes.POINTER(Split16), vp,
                                                  ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                                                  ctypes.POINTER(Split16), vp]),
    "mpv_fwd_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(Shape)]),
    "mpv_probit_fwd": (ctypes.c_int, [ctypes.POINTER(Shape), ctypes.POINTER(FwdArgs), vp]),
    "mpv_bstat_combine": (ctypes.c_int, [vp, ctypes.c_int64, ctypes.c_int64, vp, vp]),
    "mpv_probit_finalize": (ctypes.c_int, [ctypes.POINTER(Shape), ctypes.POINTER(FinalArgs), vp]),
    "mpv_probit_finalize_shards": (ctypes.c_int, [ctypes.POINTER(Shape), vp, ctypes.c_int64, vp,
                                                  ctypes.POINTER(FinalArgs), vp]),
    "mpv_bwd_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(Shape), ctypes.c_int]),
    "mpv_probit_bwd": (ctypes.c_int, [ctypes.POINTER(Shape), ctypes.POINTER(BwdArgs), vp]),
    "mpv_kl_bwd": (ctypes.c_int, [ctypes.POINTER(KlBwdArgs), vp]),
    "mpv_reparam_fwd": (ctypes.c_int, [ctypes.POINTER(ReparamArgs), vp]),
    "mpv_reparam_bwd": (ctypes.c_int, [ctypes.POINTER(ReparamBwdArgs), vp]),
    "mpv_linear_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64, ctypes.c_int64,
                                                     ctypes.c_int64]),
    "mpv_linear": (ctypes.c_int, [ctypes.POINTER(LinearArgs), vp, ctypes.c_size_t, vp]),
    "mpv_linear_batch_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(LinearArgs), ctypes.c_int]),
    "mpv_linear_batch": (ctypes.c_int, [ctypes.POINTER(LinearArgs), ctypes.c_int, vp,
                                        ctypes.c_size_t, vp]),
    "mpv_adam_step": (ctypes.c_int, [ctypes.POINTER(AdamArgs), vp]),
    "mpv_adam_finish": (ctypes.c_int, [ctypes.POINTER(AdamFinishArgs), vp]),
    "mpv_timing_enable": (ctypes.c_int, [ctypes.c_int]),
    "mpv_timing_reset": (ctypes.c_int, []),
    "mpv_timing_query": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64),
                                        ctypes.POINTER(ctypes.c_double)]),
    "mpv_label_weights": (ctypes.c_int, [vp, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.POINTER(LabelTable), vp, vp, vp]),
    "mpv_fair_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64, ctypes.c_int64,
                                                   ctypes.c_int64]),
    "mpv_fair_fwd": (ctypes.c_int, [ctypes.POINTER(FairArgs), vp, ctypes.c_size_t, vp]),
    "mpv_fair_bwd": (ctypes.c_int, [ctypes.POINTER(FairArgs), vp, vp, vp, vp, ctypes.c_size_t,
                                    vp]),
    "mpv_metrics_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64, ctypes.c_int64]),
    "mpv_train_metrics": (ctypes.c_int, [vp, vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_float,
                                         vp, vp, ctypes.c_size_t, vp]),
}

_lib = None


def load_library(path=None):
    """Load (once) and type the C ABI.  Raises if the library is absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise MPVError(f"libmpvae_hip.so not found at {p}: run `make -C mpvae-1_amd` "
                       "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    if lib.mpv_abi_version() != ABI_VERSION:
        raise MPVError(f"ABI mismatch: library {lib.mpv_abi_version()} != {ABI_VERSION}")
    if path is None:
        _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        msg = load_library().mpv_last_error().decode(errors="replace")
        raise MPVError(f"{what} failed (status {rc}): {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_of(device):
    """The current HIP stream of `device` (the capturing stream inside
    torch.cuda.graph).  The raw-handle query costs ~0.3 us where building a
    torch.cuda.Stream object costs ~6 (several per compute_loss call)."""
    d = device if isinstance(device, torch.device) else torch.device(device)
    idx = d.index if d.index is not None else torch.cuda.current_device()
    if _raw_stream is None:  # a torch without the private query: the public object
        return ctypes.c_void_p(torch.cuda.current_stream(idx).cuda_stream)
    return ctypes.c_void_p(_raw_stream(idx))


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def require_gpu(*tensors):
    """The product path runs only on the GPU; CPU tensors are an error, not a fallback."""
    for t in tensors:
        if t is not None and t.device.type != "cuda":
            raise RuntimeError("mpvae-1_amd runs the probit-ELBO hot path on the GPU only "
                               f"(got a {t.device} tensor); move inputs to a ROCm device")
    load_library()


KERNELS = ["noise_philox", "split", "probit_fwd", "fwd_combine", "finalize", "bwd_coef", "bwd_elem",
           "dR_gemm", "sum_slabs", "convert", "bstat_combine", "reparam_fwd", "reparam_bwd",
           "kl_bwd", "label_weights", "fair_fwd", "fair_bwd", "metrics", "linear", "adam",
           "adam_finish"]


def kernel_times():
    """{kernel: (launches, total_ms)} recorded since the last mpv_timing_reset()."""
    lib = load_library()
    out = {}
    for k in KERNELS:
        n, ms = ctypes.c_int64(), ctypes.c_double()
        check(lib.mpv_timing_query(k.encode(), ctypes.byref(n), ctypes.byref(ms)), "timing_query")
        if n.value:
            out[k] = (n.value, ms.value)
    return out
