"""Drop-in replacement of reference ``mpvae.py`` (lliutianc/MPVAE-1) on MI355X.

Same public names, signatures, parameter names, shapes and dtypes:

  VAE(args)                       nn.Module, reference mpvae.py:10-100
  compute_loss(input_label, fe_out, fe_mu, fe_logvar, fx_out, fx_mu, fx_logvar,
               r_sqrt_sigma, args) -> (total, nll, nll_x, c, c_x, kl,
                                       indiv_prob, indiv_prob_label)
                                  reference mpvae.py:145-210

Put ``mpvae-1_amd/`` on ``sys.path`` and ``from mpvae import VAE, compute_loss``
works unchanged in the reference's training loop (fairsoft_train.py:57-146).
The arithmetic runs in hand-written gfx950 kernels (libmpvae_hip.so),
the encoder/decoder Linear layers included (``nn.Linear`` modules hold the
parameters; their GEMMs run in mpv_linear, see ``mpvae_linear``).

Build-only knobs read from ``args`` (defaults reproduce the reference):
  mpvae_noise  "torch_cpu" (default): draw the probit noise from torch's CPU
               default generator exactly as mpvae.py:162 does (same values,
               same RNG consumption), then copy it to the device;
               "philox": generate it on the device with the counter-based
               Philox4x32-10 kernel (perf mode; a different, equally
               distributed N(0,1) stream -- DESIGN.md);
               a (n_sample, B, z_dim) float32 tensor: use it as the noise.
  mpvae_seed   philox seed (default: drawn from torch's CPU generator, so
               runs are reproducible under torch.manual_seed).
  mpvae_gemm   "f16x3" (default): noise GEMMs on the f16 matrix cores with
               3xf16 split operands (~fp32 accuracy);
               "f32": exact fp32 matrix-core GEMMs.
  mpvae_shard  True: shard the n_sample axis over the default
               torch.distributed group (mpvae_dist.py); default False.
  mpvae_linear "hip" (default): the encoder / decoder Linear layers (with
               their ReLU and scale_coeff) on the fp32 matrix cores
               (mpvae_linear.py, csrc/linear.hip); "torch": nn.Linear
               (hipBLASLt / rocBLAS), for A/B.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

import mpvae_hip
import mpvae_dist
import mpvae_linear
from mpvae_ops import ElboConfig, FusedReparam, ProbitELBO, SingleReparam

__all__ = ["VAE", "compute_loss"]

# the encoders' dropout backward folded into mpv_linear (same values; False:
# nn.Dropout's own backward kernel, for A/B)
FOLD_DROPOUT = True
# mu / logvar returned through FusedReparam (their KL gradient added in its
# backward launch; same values; False: autograd adds them, for A/B)
REPARAM_PASSTHROUGH = True

# (attribute, in_features, out_features) in the reference's construction order
# (mpvae.py:14-32).  The order fixes the torch init draws and the state_dict
# key order, so seeded runs and existing .pkl checkpoints carry over.
def _layer_table(F_, d, L):
    return [
        ("fx1", F_, 256), ("fx2", 256, 512), ("fx3", 512, 256),
        ("fx_mu", 256, d), ("fx_logvar", 256, d),
        ("fd_x1", F_ + d, 256), ("fd_x2", 256, 512), ("feat_mp_mu", 512, L),
        ("fe1", F_ + L, 512), ("fe2", 512, 256),
        ("fe_mu", 256, d), ("fe_logvar", 256, d),
    ]


def _init_r_sqrt_sigma(args):
    """r_sqrt_sigma (L, z): mpvae.py:40-48.  'random' -> fp64 frozen,
    'zero' -> fp32 zeros frozen, otherwise fp64 trainable; uniform draws come
    from numpy's global RNG like the reference."""
    L, z = args.label_dim, args.z_dim
    bound = np.sqrt(6.0 / (L + z))
    if args.residue_sigma == "zero":
        return nn.Parameter(torch.zeros((L, z)), requires_grad=False)
    draw = torch.from_numpy(np.random.uniform(-bound, bound, (L, z)))
    return nn.Parameter(draw, requires_grad=args.residue_sigma != "random")


class VAE(nn.Module):
    """MPVAE: label encoder q(z|x,y), feature encoder p(z|x), shared decoder."""

    def __init__(self, args):
        super().__init__()
        for name, n_in, n_out in _layer_table(args.feature_dim, args.latent_dim, args.label_dim):
            setattr(self, name, nn.Linear(n_in, n_out))
        # the label branch decodes through the feature branch's first two layers
        self.fd1 = self.fd_x1
        self.fd2 = self.fd_x2
        self.label_mp_mu = nn.Linear(512, args.label_dim)
        assert self.fd1 is self.fd_x1 and self.fd2 is self.fd_x2
        self.dropout = nn.Dropout(p=args.keep_prob)   # keep_prob is the DROP rate (mpvae.py:38)
        self.scale_coeff = args.scale_coeff
        self.linear_backend = getattr(args, "mpvae_linear", "hip")
        if self.linear_backend not in ("hip", "torch"):
            raise ValueError(f"mpvae_linear must be 'hip' or 'torch', got {self.linear_backend!r}")
        self.register_parameter("r_sqrt_sigma", _init_r_sqrt_sigma(args))
        # eps ~ N(0,1) like torch.randn_like (mpvae.py:68,73); replaceable for tests
        self.reparam_noise = torch.randn_like

    # -- one Linear layer: act(alpha * layer(x)), act = ReLU if `relu`
    def _hip(self, x):
        """mpv_linear / the fused reparameterisation on CUDA tensors; CPU tensors
        run the reference's own torch ops (mpvae.py:51-84)."""
        return self.linear_backend == "hip" and x.is_cuda

    def _lin(self, layer, x, relu=False, alpha=1.0):
        if self._hip(x):
            return mpvae_linear.linear(x, layer, relu, alpha)
        y = layer(x)
        if relu:
            return F.relu(y)
        return y * alpha if alpha != 1.0 else y

    # -- encoders (mpvae.py:51-64)
    def _mlp(self, x, layers):
        drop = self.dropout
        fold = (FOLD_DROPOUT and self._hip(x) and type(drop) is nn.Dropout
                and drop.training
                and drop.p > 0.0 and not drop.inplace)
        for lin in layers:
            if fold:  # torch's dropout kernel, its backward folded into mpv_linear
                x = mpvae_linear.linear(x, lin, True, 1.0, drop.p)
            else:
                x = drop(self._lin(lin, x, relu=True))
        return x

    def _heads(self, h, mu, logvar):
        if self._hip(h):  # both heads in one launch
            return mpvae_linear.heads(h, mu, logvar, self.scale_coeff)
        return (self._lin(mu, h, alpha=self.scale_coeff),
                self._lin(logvar, h, alpha=self.scale_coeff))

    def label_encode(self, x):
        return self._heads(self._mlp(x, (self.fe1, self.fe2)), self.fe_mu, self.fe_logvar)

    def feat_encode(self, x):
        return self._heads(self._mlp(x, (self.fx1, self.fx2, self.fx3)), self.fx_mu,
                           self.fx_logvar)

    # -- reparameterisation (mpvae.py:66-74), one encoder at a time
    def _reparam(self, mu, logvar):
        eps = self.reparam_noise(logvar)
        if mu.is_cuda:
            return SingleReparam.apply(mu, logvar, eps)
        return mu + eps * torch.exp(0.5 * logvar)  # mpvae.py:67-69 on the CPU

    def label_reparameterize(self, mu, logvar):
        return self._reparam(mu, logvar)

    def feat_reparameterize(self, mu, logvar):
        return self._reparam(mu, logvar)

    # -- decoders (mpvae.py:76-84); fd1/fd2 are fd_x1/fd_x2
    def _decode(self, z, head):
        h = self._lin(self.fd_x2, self._lin(self.fd_x1, z, relu=True), relu=True)
        return self._lin(head, h)

    def label_decode(self, z):
        return self._decode(z, self.label_mp_mu)

    def feat_decode(self, z):
        return self._decode(z, self.feat_mp_mu)

    def label_forward(self, x, feat):
        mu, logvar = self.label_encode(torch.cat((feat, x), 1))
        z = self.label_reparameterize(mu, logvar)
        return self.label_decode(torch.cat((feat, z), 1)), mu, logvar

    def feat_forward(self, x):
        mu, logvar = self.feat_encode(x)
        z = self.feat_reparameterize(mu, logvar)
        return self.feat_decode(torch.cat((x, z), 1)), mu, logvar

    def forward(self, label, feature):
        """(label_out, label_mu, label_logvar, feat_out, feat_mu, feat_logvar).

        Both encoders are evaluated first and reparameterised by ONE fused
        launch.  RNG draws keep the reference order: label-encoder dropouts,
        label eps, feature-encoder dropouts, feature eps (mpvae.py:86-100).
        On mpv_linear the two decoders, which share fd_x1 / fd_x2, run as one
        pass over both inputs stacked (no dropout there: same values)."""
        mu_e, lv_e = self.label_encode(torch.cat((feature, label), 1))
        eps_e = self.reparam_noise(lv_e)
        mu_x, lv_x = self.feat_encode(feature)
        eps_x = self.reparam_noise(lv_x)
        if not feature.is_cuda:  # the reference's ops on the CPU (mpvae.py:67-74, 76-84)
            z_e = mu_e + eps_e * torch.exp(0.5 * lv_e)
            z_x = mu_x + eps_x * torch.exp(0.5 * lv_x)
            return (self.label_decode(torch.cat((feature, z_e), 1)), mu_e, lv_e,
                    self.feat_decode(torch.cat((feature, z_x), 1)), mu_x, lv_x)
        # mu / logvar come back through the fused op: compute_loss's KL gradient
        # for them is then added inside its backward launch
        r = FusedReparam.apply(mu_e, lv_e, eps_e, mu_x, lv_x, eps_x)
        z_e, z_x = r[:2]
        if REPARAM_PASSTHROUGH:
            mu_e, lv_e, mu_x, lv_x = r[2:]
        if self.linear_backend == "hip":
            # both decoders share fd_x1 / fd_x2 (mpvae.py:31-32): run them
            # once on the two inputs stacked, then the two heads on their rows
            B = feature.shape[0]
            zz = torch.cat((torch.cat((feature, feature), 0), torch.cat((z_e, z_x), 0)), 1)
            h = self._lin(self.fd_x2, self._lin(self.fd_x1, zz, relu=True), relu=True)
            label_out, feat_out = mpvae_linear.row_heads(h, self.label_mp_mu, self.feat_mp_mu, B)
        else:
            label_out = self.label_decode(torch.cat((feature, z_e), 1))
            feat_out = self.feat_decode(torch.cat((feature, z_x), 1))
        return label_out, mu_e, lv_e, feat_out, mu_x, lv_x


# Reference-exact CPU noise under sample sharding: every rank draws all
# n_sample * B * z normals on its host (torch's CPU generator cannot skip ahead)
# and keeps its 1/world slice.  Above WARN elements per step that is flagged;
# above MAX (16 GiB of fp32 per rank per step, e.g. C5's 1.7e10 = 68.7 GB) it
# is refused: args.mpvae_noise = "philox" draws each rank's own slice on the
# device from a key shared across ranks (the single-device stream at any world).
SHARDED_CPU_NOISE_WARN = 1 << 26
SHARDED_CPU_NOISE_MAX = 1 << 32


def _guard_sharded_cpu_noise(n, world):
    if n > SHARDED_CPU_NOISE_MAX:
        raise ValueError(
            f"args.mpvae_noise='torch_cpu' with args.mpvae_shard draws the whole "
            f"{n:.3g}-element noise tensor ({4 * n / 2 ** 30:.1f} GiB) on every one of the "
            f"{world} ranks' hosts each step and uses 1/{world} of it; above "
            f"{SHARDED_CPU_NOISE_MAX:.3g} elements that is refused -- use "
            "args.mpvae_noise='philox' (per-rank device noise, the same stream at any world "
            "size) or pass the noise tensor explicitly")
    if n > SHARDED_CPU_NOISE_WARN:
        import warnings
        warnings.warn(f"args.mpvae_noise='torch_cpu' with args.mpvae_shard: each of the {world} "
                      f"ranks draws all {n:.3g} normals on its host per step to keep the "
                      "reference's CPU stream, and uses 1/world of them; "
                      "args.mpvae_noise='philox' scales", stacklevel=4)


def _noise_source(args, n_sample, B, z, shard, device):
    """(noise tensor or None, ElboConfig kwargs) for compute_loss."""
    mode = getattr(args, "mpvae_noise", "torch_cpu")
    s0, s1 = shard.s_offset, shard.s_offset + shard.S_local
    if isinstance(mode, torch.Tensor):
        if tuple(mode.shape) != (n_sample, B, z):
            raise ValueError(f"args.mpvae_noise must be {(n_sample, B, z)}, got {tuple(mode.shape)}")
        return mode[s0:s1].to(device=device, dtype=torch.float32), dict(noise="explicit")
    if mode == "torch_cpu":
        # mpvae.py:162 -- same generator, same draw, same shape; then H2D.
        # Sharded, every rank must draw the WHOLE tensor to keep the
        # single-device stream and then uses 1/world of it
        if shard.exchange is not None:
            _guard_sharded_cpu_noise(n_sample * B * z, shard.exchange.world)
        noise = torch.normal(0, 1, size=(n_sample, B, z))
        return noise[s0:s1].to(device), dict(noise="explicit")
    if mode == "philox":
        # args.mpvae_seed: an int, or a one-element int64 tensor on the device
        # whose value the noise kernel reads at run time (no host sync; a step
        # captured in a HIP graph draws fresh noise when the tensor advances).
        # args.mpvae_seed_advance (with a device tensor): the finalize launch
        # advances it by 1 once this step's noise has read it, so the next call
        # (or graph replay) draws fresh noise with no launch of its own
        seed = getattr(args, "mpvae_seed", None)
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        advance = seed if (getattr(args, "mpvae_seed_advance", False)
                           and isinstance(seed, torch.Tensor)) else None
        if getattr(args, "mpvae_seed_advance", False) and advance is None:
            raise ValueError("args.mpvae_seed_advance needs args.mpvae_seed to be a one-element "
                             "int64 device tensor")
        if shard.exchange is not None:
            # one noise stream for the whole job: rank 0's seed (mpvae_dist.py).
            # An int key travels as a device tensor written by a fill kernel (no
            # host copy): the noise kernel reads it at run time, so agreeing on
            # it costs no host sync (the broadcast + .item() of an int did, every
            # step: 0.19 ms of the 512-sample share's step)
            if not isinstance(seed, torch.Tensor):
                u = int(seed) & (2 ** 64 - 1)
                seed = torch.full((1,), u - 2 ** 64 if u >= 2 ** 63 else u, dtype=torch.int64,
                                  device=device)
            seed = shard.exchange.agree_seed(seed, device)
        return None, dict(noise="philox", seed=seed, offset=0, seed_advance=advance)
    raise ValueError(f"unknown args.mpvae_noise {mode!r} (torch_cpu | philox | tensor)")


def _empty_batch(fe_out, fe_mu, fe_logvar, fx_out, fx_mu, fx_logvar, R, args):
    """compute_loss of a batch of 0 rows, as the reference evaluates it: its
    means over the batch are NaN (mpvae.py:147, 190, 199-200) and indiv_prob*
    are (0, L) (:203-204); autograd reaches the same leaves, with empty
    gradients and a zero one for r_sqrt_sigma (an optimizer steps on it as on
    the reference's).  There is nothing to compute, so no kernel runs."""
    nan = torch.full((), float("nan"), dtype=torch.float32, device=fe_out.device)
    zr = (R.sum() * 0).float()
    ze, zx = fe_out.sum() * 0 + zr, fx_out.sum() * 0 + zr
    nll, nll_x, c, c_x = nan + ze, nan + zx, nan + ze, nan + zx
    kl = nan + (fe_mu.sum() + fe_logvar.sum() + fx_mu.sum() + fx_logvar.sum()) * 0
    total = (nll + nll_x) * args.nll_coeff + (c + c_x) * args.c_coeff + kl * 1.1
    return (total, nll, nll_x, c, c_x, kl, fx_out.float() * 0 + zr, fe_out.float() * 0 + zr)


def _backend_for(tensors):
    """None (the HIP library on the GPU) for CUDA tensors -- raising when it is
    missing -- or the host C++ backend (mpvae_host.py) for CPU tensors, as the
    reference runs its small configurations on the CPU (fairsoft_trial.py:
    157-158).  Dispatch by device, never a fallback: CUDA tensors do not reach
    the host backend."""
    kinds = {t.device.type for t in tensors if t is not None}
    if kinds == {"cpu"}:
        import mpvae_host
        return mpvae_host.HostShardBackend()
    mpvae_hip.require_gpu(*tensors)
    if len({t.device for t in tensors if t is not None}) > 1:
        raise RuntimeError("compute_loss inputs must all live on one device")
    return None


def compute_loss(input_label, fe_out, fe_mu, fe_logvar, fx_out, fx_mu, fx_logvar,
                 r_sqrt_sigma, args):
    """Multivariate-probit ELBO of reference mpvae.py:145-210 (8-tuple)."""
    host_be = _backend_for((input_label, fe_out, fe_mu, fe_logvar, fx_out, fx_mu, fx_logvar,
                            r_sqrt_sigma))
    n_sample = args.n_train_sample if args.mode == "train" else args.n_test_sample
    B, z = fe_out.shape[0], args.z_dim
    if r_sqrt_sigma.dim() != 2 or r_sqrt_sigma.shape[1] != z:
        raise ValueError(f"r_sqrt_sigma must be (label_dim, z_dim={z}), "
                         f"got {tuple(r_sqrt_sigma.shape)}")
    if n_sample <= 0:
        # the reference's max over an empty sample axis (mpvae.py:188)
        raise IndexError(f"n_sample = {n_sample}: the Monte-Carlo sample axis is empty")
    if B == 0:
        return _empty_batch(fe_out, fe_mu, fe_logvar, fx_out, fx_mu, fx_logvar, r_sqrt_sigma,
                            args)
    shard = mpvae_dist.shard_for(args, n_sample)
    noise, kw = _noise_source(args, n_sample, B, z, shard, fe_out.device)
    cfg = ElboConfig(n_sample, shard.S_local, shard.s_offset, args.nll_coeff, args.c_coeff,
                     exchange=shard.exchange, gemm=getattr(args, "mpvae_gemm", "f16x3"),
                     backend=host_be, **kw)
    return ProbitELBO.apply(input_label.float(), fe_out, fe_mu, fe_logvar, fx_out, fx_mu,
                            fx_logvar, r_sqrt_sigma, noise, cfg)
