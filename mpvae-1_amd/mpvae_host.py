"""The probit-ELBO hot path for CPU tensors: libmpvae_host.so (include/mpvae_host.h).

The reference runs its small configuration on the CPU (BASELINE configs[0],
script/run_train_mirflickr.sh; fairsoft_trial.py:157-158 picks the CPU when
CUDA is absent).  ``compute_loss`` dispatches on the tensors' device: CPU
tensors run here, in host C++ with OpenMP (the same algorithm as the HIP
kernels: factorised ranking loss, exact log-sum-exp, analytic backward; E in
fp32 in the reference's op order, fp64 after).  This is a backend for CPU
tensors, not a fallback: CUDA tensors always run the HIP library and raise
when it is missing.

``HostShardBackend`` has the per-shard interface of
``mpvae_ops.HipShardBackend`` (forward_local / combine_bstats / finalize /
backward_local / kl_backward), so ``ProbitELBO`` and the sample-sharded exchange
(mpvae_dist.py, gloo on CPU) drive it unchanged.
"""
import ctypes
import os

import torch

import mpvae_hip as H

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MPVAE_HOST_LIB", os.path.join(HERE, "libmpvae_host.so"))
ABI_VERSION = 1
vp = ctypes.c_void_p
F32, F64 = torch.float32, torch.float64


class FwdArgs(ctypes.Structure):
    _fields_ = [("y", vp), ("fe_out", vp), ("fx_out", vp), ("R", vp), ("R_dtype", ctypes.c_int),
                ("eps", vp), ("T", vp), ("rowstat", vp), ("bstat", vp), ("colsum", vp)]


class FinalArgs(ctypes.Structure):
    _fields_ = [("bstat", vp), ("colsum", vp), ("fe_mu", vp), ("fe_logvar", vp), ("fx_mu", vp),
                ("fx_logvar", vp), ("d", ctypes.c_int64), ("nll_coeff", ctypes.c_float),
                ("c_coeff", ctypes.c_float), ("out6", vp), ("indiv_prob", vp),
                ("indiv_prob_label", vp)]


class BwdArgs(ctypes.Structure):
    _fields_ = [("y", vp), ("fe_out", vp), ("fx_out", vp), ("eps", vp), ("T", vp),
                ("rowstat", vp), ("bstat", vp), ("gscal", vp), ("live", ctypes.c_int),
                ("g_indiv", vp), ("g_indiv_label", vp), ("nll_coeff", ctypes.c_float),
                ("c_coeff", ctypes.c_float), ("dfe_dfx", vp), ("dR", vp)]


_SIGS = {
    "mpvh_abi_version": (ctypes.c_int, []),
    "mpvh_last_error": (ctypes.c_char_p, []),
    "mpvh_set_threads": (ctypes.c_int, [ctypes.c_int]),
    "mpvh_probit_fwd": (ctypes.c_int, [ctypes.POINTER(H.Shape), ctypes.POINTER(FwdArgs)]),
    "mpvh_bstat_combine": (ctypes.c_int, [vp, ctypes.c_int64, ctypes.c_int64, vp]),
    "mpvh_probit_finalize": (ctypes.c_int, [ctypes.POINTER(H.Shape), ctypes.POINTER(FinalArgs)]),
    "mpvh_probit_bwd": (ctypes.c_int, [ctypes.POINTER(H.Shape), ctypes.POINTER(BwdArgs)]),
    "mpvh_kl_bwd": (ctypes.c_int, [vp, vp, vp, vp, ctypes.c_int64, ctypes.c_int64, vp, ctypes.c_int,
                                   vp, vp, vp, vp]),
}
EXPORTS = sorted(_SIGS)

_lib = None


def load_library():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise H.MPVError(f"libmpvae_host.so not found at {LIB_PATH}: run `make -C mpvae-1_amd`")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        if lib.mpvh_abi_version() != ABI_VERSION:
            raise H.MPVError(f"host ABI mismatch: library {lib.mpvh_abi_version()} != {ABI_VERSION}")
        _lib = lib
    return _lib


def _check(rc, what):
    if rc != 0:
        raise H.MPVError(f"{what} failed ({rc}): {load_library().mpvh_last_error().decode()}")


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _c(t, dtype):
    if t.dtype != dtype:
        raise TypeError(f"expected {dtype}, got {t.dtype}")
    return t.detach().contiguous()


class HostShardBackend:
    """Per-shard arithmetic on the CPU through libmpvae_host.so (the interface of
    mpvae_ops.HipShardBackend; statistics in fp64)."""

    reads_live_slots = True   # gscal may hold just the live TOTAL slot

    def shape(self, S_local, S_total, s_offset, B, L, z):
        return H.Shape(S_local, S_total, s_offset, B, L, z)

    def make_noise(self, shape, device, seed, offset):
        raise ValueError("args.mpvae_noise = 'philox' draws on the GPU; CPU tensors take the "
                         "reference's torch_cpu draw or an explicit noise tensor")

    def prepare_noise(self, eps, shape):
        return _c(eps, F32)

    def prepare_R(self, R):
        if R.dtype not in (F32, F64):
            raise TypeError(f"r_sqrt_sigma must be float32 or float64 (got {R.dtype})")
        return R.detach().contiguous()

    def from_f32(self, x32, dtype):
        return x32 if dtype == F32 else x32.to(dtype)

    def forward_local(self, shape, y, fe_out, fx_out, Rop, eps, keep_T, stat_slots=None):
        S, B, L = shape.S_local, shape.B, shape.L
        T = torch.empty((S, B, L), dtype=F32) if keep_T else None
        rowstat = torch.empty((6, B, S), dtype=F64)
        packed = None
        if stat_slots is None:
            bstat = torch.empty((6, B), dtype=F64)
            colsum = torch.empty((2, B, L), dtype=F64)
        else:  # [colsum | world slots of bstat]: one all_reduce sums and gathers
            world, slot = stat_slots
            n = 2 * B * L
            packed = torch.zeros((n + world * 6 * B,), dtype=F64)
            colsum = packed[:n].view(2, B, L)
            bstat = packed[n + slot * 6 * B:n + (slot + 1) * 6 * B].view(6, B)
        y, fe_out, fx_out = (_c(t, F32) for t in (y, fe_out, fx_out))
        a = FwdArgs(_p(y), _p(fe_out), _p(fx_out), _p(Rop), H.F64 if Rop.dtype == F64 else H.F32,
                    _p(eps), _p(T), _p(rowstat), _p(bstat), _p(colsum))
        _check(load_library().mpvh_probit_fwd(shape, a), "mpvh_probit_fwd")
        return dict(rowstat=rowstat, bstat=bstat, colsum=colsum, T=T, packed=packed)

    def combine_bstats(self, gathered):
        g = gathered.to(F64).contiguous()
        out = torch.empty(g.shape[1:], dtype=F64)
        _check(load_library().mpvh_bstat_combine(_p(g), g.shape[0], g.shape[2], _p(out)),
               "mpvh_bstat_combine")
        return out

    def finalize(self, shape, bstat, colsum, fe_mu, fe_logvar, fx_mu, fx_logvar, nll_coeff,
                 c_coeff, seed_advance=None):
        if seed_advance is not None:
            raise ValueError("args.mpvae_seed_advance is a device-key option (philox on the GPU)")
        B, L = shape.B, shape.L
        out6 = torch.empty((6,), dtype=F32)
        indiv = torch.empty((B, L), dtype=F32)
        indiv_label = torch.empty((B, L), dtype=F32)
        mus = [_c(t, F32) for t in (fe_mu, fe_logvar, fx_mu, fx_logvar)]
        bstat, colsum = bstat.to(F64).contiguous(), colsum.to(F64).contiguous()
        a = FinalArgs(_p(bstat), _p(colsum), *[_p(t) for t in mus], fe_mu.shape[1], nll_coeff,
                      c_coeff, _p(out6), _p(indiv), _p(indiv_label))
        _check(load_library().mpvh_probit_finalize(shape, a), "mpvh_probit_finalize")
        return (*[out6[i] for i in range(6)], indiv, indiv_label)

    def backward_local(self, shape, saved, gscal, live, g_I, g_IL, nll_coeff, c_coeff, want_dR,
                       dR_dtype=F32, kl=False):
        """HipShardBackend.backward_local's contract: (flat fp32 [d fe_out | d fx_out
        | d r_sqrt_sigma], its (2, B, L) view, dR in dR_dtype[, the 4 KL grads])."""
        B, L, z = shape.B, shape.L, shape.z
        d2 = torch.empty((2, B, L), dtype=F64)
        dR64 = torch.empty((L, z), dtype=F64) if want_dR else None
        # every tensor the call reads is bound to a name here (alive through the call)
        gscal = _c(gscal.reshape(-1).to(F32), F32)
        rowstat = saved["rowstat"].to(F64).contiguous()
        bstat = saved["bstat"].to(F64).contiguous()
        g_I = None if g_I is None else _c(g_I, F32)
        g_IL = None if g_IL is None else _c(g_IL, F32)
        a = BwdArgs(_p(saved["y"]), _p(saved["fe_out"]), _p(saved["fx_out"]), _p(saved["eps"]),
                    _p(saved["T"]), _p(rowstat), _p(bstat), _p(gscal), int(live), _p(g_I),
                    _p(g_IL), nll_coeff, c_coeff, _p(d2), _p(dR64))
        _check(load_library().mpvh_probit_bwd(shape, a), "mpvh_probit_bwd")
        n = 2 * B * L
        local64 = dR_dtype == F64 and want_dR
        flat = torch.empty((n + (L * z if want_dR and not local64 else 0),), dtype=F32)
        flat[:n] = d2.reshape(-1)
        dR = None
        if want_dR:
            if local64:
                dR = dR64
            else:
                flat[n:] = dR64.reshape(-1)
                dR = flat[n:].view(L, z)
        out = (flat, flat[:n].view(2, B, L), dR)
        if kl:
            out = (*out, self.kl_backward(saved["fe_mu"], saved["fe_logvar"], saved["fx_mu"],
                                          saved["fx_logvar"], gscal, live))
        return out

    def kl_backward(self, fe_mu, fe_logvar, fx_mu, fx_logvar, gscal, live=0x3F):
        mus = [_c(t, F32) for t in (fe_mu, fe_logvar, fx_mu, fx_logvar)]
        B, d = fe_mu.shape
        outs = [torch.empty((B, d), dtype=F32) for _ in range(4)]  # g_fe_mu, g_fe_logvar, ...
        g = _c(gscal.reshape(-1).to(F32), F32)
        _check(load_library().mpvh_kl_bwd(*[_p(t) for t in mus], B, d, _p(g), int(live),
                                          _p(outs[0]), _p(outs[1]), _p(outs[2]), _p(outs[3])),
               "mpvh_kl_bwd")
        return outs
