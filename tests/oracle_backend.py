"""A CPU shard backend built on the oracle -- TEST ONLY.

It implements the same per-shard interface as the product's
``mpvae_ops.HipShardBackend`` (forward_local / combine_bstats / finalize /
backward_local / kl_backward) with oracle.probit_elbo, so the product's
autograd Function and its cross-rank exchange (mpvae_dist.SampleShardExchange)
can be exercised on CPU with the gloo backend.  The kernels themselves are
checked on the GPU (test_gpu_parity.py).
"""
import types

import numpy as np
import torch

from oracle import probit_elbo as pe


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))


class OracleShardBackend:
    def shape(self, S_local, S_total, s_offset, B, L, z):
        return types.SimpleNamespace(S_local=S_local, S_total=S_total, s_offset=s_offset, B=B,
                                     L=L, z=z)

    def make_noise(self, shape, device, seed, offset):
        from oracle import philox
        if isinstance(seed, torch.Tensor):  # a device-memory key (mpv_noise_philox*_dev)
            seed = int(seed.reshape(-1)[0]) & (2 ** 64 - 1)
        return _t(philox.normal_noise(shape.S_local, shape.B, shape.z, seed, offset,
                                      shape.s_offset))

    def prepare_R(self, R):
        return R.detach().float().contiguous()

    def prepare_noise(self, eps, shape):
        return eps

    def from_f32(self, x32, dtype):
        return x32.to(dtype)

    def forward_local(self, shape, y, fe_out, fx_out, R32, eps, keep_T, stat_slots=None):
        f = pe.shard_forward(y.numpy(), fe_out.detach().numpy(), fx_out.detach().numpy(),
                             R32.numpy(), eps.numpy())
        out = dict(rowstat=_t(f["rowstat"]), bstat=_t(f["bstat"]), colsum=_t(f["colsum"]),
                   T=f if keep_T else None, packed=None)
        if stat_slots is not None:  # the product's packed layout (HipShardBackend)
            world, slot = stat_slots
            n, m = out["colsum"].numel(), out["bstat"].numel()
            packed = torch.zeros(n + world * m, dtype=torch.float32)
            packed[:n] = out["colsum"].reshape(-1)
            packed[n + slot * m:n + (slot + 1) * m] = out["bstat"].reshape(-1)
            out.update(packed=packed, colsum=packed[:n].view(out["colsum"].shape),
                       bstat=packed[n + slot * m:n + (slot + 1) * m].view(out["bstat"].shape))
        return out

    def combine_bstats(self, gathered):
        return _t(pe.combine_bstats(list(gathered.double().numpy())))

    def finalize(self, shape, bstat, colsum, fe_mu, fe_logvar, fx_mu, fx_logvar, nll_coeff,
                 c_coeff):
        kl = pe.kl_term(*(t.detach().numpy() for t in (fe_mu, fe_logvar, fx_mu, fx_logvar)))
        o = pe.finalize(bstat.double().numpy(), colsum.double().numpy(), shape.S_total, kl,
                        nll_coeff, c_coeff)
        scal = [torch.tensor(float(o[k]), dtype=torch.float32)
                for k in ["total", "nll", "nll_x", "c", "c_x", "kl"]]
        return (*scal, _t(o["indiv_prob"]), _t(o["indiv_prob_label"]))

    def _g(self, gscal, live, nll_coeff, c_coeff):
        gs = gscal.double().numpy()
        livef = lambda *slots: any(live & (1 << s) for s in slots)
        g = dict(nll=gs[1] + nll_coeff * gs[0], nll_x=gs[2] + nll_coeff * gs[0],
                 c=(gs[3] + c_coeff * gs[0]) if livef(0, 3) else None,
                 c_x=(gs[4] + c_coeff * gs[0]) if livef(0, 4) else None)
        return g

    def backward_local(self, shape, saved, gscal, live, g_I, g_IL, nll_coeff, c_coeff, want_dR,
                       dR_dtype=torch.float32, kl=False):
        """HipShardBackend.backward_local's contract: dR in dR_dtype (a
        separate tensor when fp64), the KL gradients appended when kl."""
        out = self._backward_local(shape, saved, gscal, live, g_I, g_IL, nll_coeff, c_coeff,
                                   want_dR)
        if want_dR and dR_dtype == torch.float64:
            flat, dfe_dfx, dR = out
            n = 2 * shape.B * shape.L
            out = (flat[:n].clone(), dfe_dfx, dR.to(torch.float64))
        if kl:
            out = (*out, self.kl_backward(saved["fe_mu"], saved["fe_logvar"], saved["fx_mu"],
                                          saved["fx_logvar"], gscal))
        return out

    def _backward_local(self, shape, saved, gscal, live, g_I, g_IL, nll_coeff, c_coeff, want_dR):
        g = self._g(gscal, live, nll_coeff, c_coeff)
        y = saved["y"].numpy()
        coef = pe.row_coefficients(saved["rowstat"].double().numpy(),
                                   saved["bstat"].double().numpy(), y, shape.S_total, g)
        dfe, dfx, dR = pe.shard_backward(saved["T"], y, saved["fe_out"].detach().numpy(),
                                         saved["fx_out"].detach().numpy(), saved["eps"].numpy(),
                                         coef, shape.S_total,
                                         None if g_I is None else g_I.numpy(),
                                         None if g_IL is None else g_IL.numpy())
        flat = np.concatenate([dfe.ravel(), dfx.ravel()] + ([dR.ravel()] if want_dR else []))
        flat = _t(flat)
        n = 2 * shape.B * shape.L
        return (flat, flat[:n].view(2, shape.B, shape.L),
                flat[n:].view(shape.L, shape.z) if want_dR else None)

    def kl_backward(self, fe_mu, fe_logvar, fx_mu, fx_logvar, gscal):
        gs = gscal.double().numpy()
        g = pe.kl_backward(*(t.detach().numpy() for t in (fe_mu, fe_logvar, fx_mu, fx_logvar)),
                           gs[5] + 1.1 * gs[0])
        return [_t(g[k]) for k in ["fe_mu", "fe_logvar", "fx_mu", "fx_logvar"]]
