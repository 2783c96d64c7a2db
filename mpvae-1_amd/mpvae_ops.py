"""Autograd Functions over the HIP kernels of libmpvae_hip.so.

``ProbitELBO`` is the whole of reference ``compute_loss`` (mpvae.py:145-210) as
one custom Function: its forward launches noise (optional) -> fused GEMM +
probit decode + row statistics -> combine -> finalize, and its backward the
analytic gradient kernels.  Sharding of the
Monte-Carlo axis across ranks plugs in through ``exchange`` (mpvae_dist.py);
the per-shard arithmetic through ``backend`` (``HipShardBackend`` here -- the
only backend the product ever uses).

``FusedReparam`` is the reparameterisation of both encoders in one launch
(mpvae.py:66-74).
"""
import ctypes

import torch

import mpvae_hip as H


def _f32(t, name):
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32 (got {t.dtype})")
    return t.contiguous()


def _pad(n, m):
    return (n + m - 1) // m * m


class Planes:
    """3xf16 split operand (include/mpvae_hip.h mpv_split16) of `cols` padded
    columns: value = (hi + lo) / scale, stored chunked -- every 32-column chunk
    of a row is 32 hi halves then 32 lo halves (row length ld = 2 * cols)."""

    def __init__(self, rows_pad, cols, device):
        if cols % 32:
            raise ValueError(f"split planes need a multiple of 32 columns (got {cols})")
        self.rows_pad, self.cols, self.ld = int(rows_pad), int(cols), 2 * int(cols)
        self.data = torch.empty((self.rows_pad, self.ld), dtype=torch.int16, device=device)
        self.scale = torch.empty((1,), dtype=torch.float32, device=device)

    def c(self):
        return H.Split16(self.data.data_ptr(), self.scale.data_ptr(), self.rows_pad, self.ld)

    def halves(self):
        """(hi, lo) as (rows_pad, cols) fp16 views' fp32 values."""
        v = self.data.view(torch.float16).float().view(self.rows_pad, self.cols // 32, 2, 32)
        return v[:, :, 0, :].reshape(self.rows_pad, self.cols), \
            v[:, :, 1, :].reshape(self.rows_pad, self.cols)

    def value(self):
        """fp32 value of the planes (tests / diagnostics)."""
        hi, lo = self.halves()
        return (hi + lo) / self.scale


GEMMS = {"f16x3": H.GEMM_F16X3, "f32": H.GEMM_F32}


def eps_cols(shape):
    """Noise plane columns: z padded to whole dR tiles (mpv_noise_plane_cols)."""
    n = H.load_library().mpv_noise_plane_cols(shape)
    if n <= 0:
        raise H.MPVError("mpv_noise_plane_cols: bad shape")
    return int(n)


class HipShardBackend:
    """Per-shard arithmetic on the GPU through the C ABI.

    gemm="f16x3" (default): the two noise GEMMs run on the f16 matrix cores
    with 3xf16 split operands (~fp32 accuracy); gemm="f32": exact fp32 MFMA.

    poison=True (tests and tools/repeat_probe.py only): every output and
    workspace buffer of forward_local / backward_local is filled with NaN bytes
    (0xFF) before the launch, so a write the kernels skip or lose shows up as a
    NaN instead of hiding behind the identical bytes the caching allocator
    hands back from an earlier launch."""

    # the kernels read only the live upstream-gradient slots (ABI 10)
    reads_live_slots = True

    def __init__(self, gemm="f16x3", poison=False):
        if gemm not in GEMMS:
            raise ValueError(f"gemm must be one of {sorted(GEMMS)} (got {gemm!r})")
        self.gemm = GEMMS[gemm]
        self.poison = bool(poison)

    def _buf(self, shape, device, dtype):
        t = torch.empty(shape, device=device, dtype=dtype)
        if self.poison:
            t.view(torch.uint8).fill_(0xFF)  # all-ones words: NaN in fp32 and fp64
        return t

    def shape(self, S_local, S_total, s_offset, B, L, z):
        return H.Shape(S_local, S_total, s_offset, B, L, z)

    @staticmethod
    def _check_seed(seed, device):
        if isinstance(seed, torch.Tensor) and (seed.dtype != torch.int64 or seed.numel() != 1 or
                                               seed.device != torch.device(device)):
            raise ValueError("a device Philox seed must be a one-element int64 tensor on "
                             f"{device} (got {seed.dtype}, {seed.numel()} elements, {seed.device})")

    def make_noise(self, shape, device, seed, offset):
        """Philox noise for this shard.  seed: an int (the key, passed by value)
        or a one-element int64 device tensor holding it (read by the kernel at
        run time: graph-capturable, no host sync)."""
        lib, st = H.load_library(), H.stream_of(device)
        dev_key = isinstance(seed, torch.Tensor)
        self._check_seed(seed, device)
        if self.gemm == H.GEMM_F16X3:
            eps = Planes(shape.S_local * shape.B, eps_cols(shape), device)
            if dev_key:
                H.check(lib.mpv_noise_philox_f16_dev(shape, H.ptr(seed), offset, eps.c(), st),
                        "mpv_noise_philox_f16_dev")
            else:
                H.check(lib.mpv_noise_philox_f16(shape, seed, offset, eps.c(), st),
                        "mpv_noise_philox_f16")
            return eps
        eps = torch.empty((shape.S_local, shape.B, shape.z), device=device, dtype=torch.float32)
        if dev_key:
            H.check(lib.mpv_noise_philox_dev(H.ptr(eps), shape, H.ptr(seed), offset, st),
                    "mpv_noise_philox_dev")
        else:
            H.check(lib.mpv_noise_philox(H.ptr(eps), shape, seed, offset, st), "mpv_noise_philox")
        return eps

    # r_sqrt_sigma of at most this many elements is split inside the noise
    # launch (mpv_noise_philox_f16_split; the split_small path)
    SPLIT_WITH_NOISE = 16384

    def make_noise_and_R(self, shape, device, seed, offset, R):
        """(make_noise(...), prepare_R(R)) -- in ONE launch when the noise is
        3xf16 Philox and R is small (L, z <= 128: C2, C3), else two."""
        L, z = R.shape
        if (self.gemm != H.GEMM_F16X3 or L * z > self.SPLIT_WITH_NOISE
                or R.dtype not in (torch.float32, torch.float64)):
            return self.make_noise(shape, device, seed, offset), self.prepare_R(R)
        lib, st = H.load_library(), H.stream_of(device)
        dev_key = isinstance(seed, torch.Tensor)
        self._check_seed(seed, device)
        eps = Planes(shape.S_local * shape.B, eps_cols(shape), device)
        Rc = R.detach().contiguous()
        Rop = Planes(_pad(L, 256), _pad(z, 128), R.device)
        H.check(lib.mpv_noise_philox_f16_split(
            shape, 0 if dev_key else int(seed) & (2 ** 64 - 1), H.ptr(seed) if dev_key else None,
            offset, eps.c(), H.ptr(Rc), H.F64 if Rc.dtype == torch.float64 else H.F32, L, z,
            Rop.c(), st), "mpv_noise_philox_f16_split")
        return eps, Rop

    def _split(self, x, rows, cols, planes):
        lib = H.load_library()
        ws = torch.empty((lib.mpv_split_workspace_bytes(),), device=x.device, dtype=torch.uint8)
        dt = H.F64 if x.dtype == torch.float64 else H.F32
        H.check(lib.mpv_split_f16(H.ptr(x), dt, rows, cols, planes.c(), H.ptr(ws),
                                  H.stream_of(x.device)), "mpv_split_f16")
        return planes

    def prepare_noise(self, eps, shape):
        """Explicit (S_local,B,z) fp32 noise -> the GEMM operand."""
        if self.gemm == H.GEMM_F32:
            return eps
        rows = shape.S_local * shape.B
        # plane rows are b-major (row b*S + s): split the (B, S, z) transpose
        eps_bs = eps.transpose(0, 1).contiguous()
        return self._split(eps_bs, rows, shape.z, Planes(rows, eps_cols(shape), eps.device))

    def prepare_R(self, R):
        """r_sqrt_sigma (L,z) fp64/fp32 -> the GEMM operand (R.T.float(), mpvae.py:165)."""
        if R.dtype not in (torch.float32, torch.float64):
            raise TypeError(f"r_sqrt_sigma must be float32 or float64 (got {R.dtype})")
        if self.gemm == H.GEMM_F32:
            return self.to_f32(R)
        L, z = R.shape
        return self._split(R.detach().contiguous(), L, z,
                           Planes(_pad(L, 256), _pad(z, 128), R.device))

    def to_f32(self, R):
        if R.dtype == torch.float32:
            return R.contiguous()
        if R.dtype != torch.float64:
            raise TypeError(f"r_sqrt_sigma must be float32 or float64 (got {R.dtype})")
        R = R.contiguous()
        out = torch.empty(R.shape, device=R.device, dtype=torch.float32)
        H.check(H.load_library().mpv_convert(H.ptr(R), H.F64, H.ptr(out), H.F32, R.numel(),
                                             H.stream_of(R.device)), "mpv_convert")
        return out

    def from_f32(self, x32, dtype):
        if dtype == torch.float32:
            return x32
        out = torch.empty(x32.shape, device=x32.device, dtype=dtype)
        H.check(H.load_library().mpv_convert(H.ptr(x32), H.F32, H.ptr(out), H.F64, x32.numel(),
                                             H.stream_of(x32.device)), "mpv_convert")
        return out

    def forward_local(self, shape, y, fe_out, fx_out, Rop, eps, keep_T, stat_slots=None):
        """stat_slots = (world, slot): colsum and bstat are written into one
        packed buffer [colsum (2 B L) | world slots of bstat (6 B)], this
        shard's bstat into its slot and the other slots zero, so that ONE
        all_reduce(SUM) of it both sums colsum and gathers bstat (x + 0 is
        exact); returned as "packed" (SampleShardExchange.combine)."""
        lib = H.load_library()
        dev = y.device
        S, B, L = shape.S_local, shape.B, shape.L
        # rows padded to 4 floats (ABI v5: 16-B aligned rows for the element pass)
        f32 = torch.float32
        T = self._buf((B, S, (L + 3) // 4 * 4), dev, f32) if keep_T else None
        rowstat = self._buf((6, B, S), dev, f32)
        packed = None
        if stat_slots is None:
            bstat = self._buf((6, B), dev, f32)
            colsum = self._buf((2, B, L), dev, f32)
        else:
            world, slot = stat_slots
            n = 2 * B * L
            packed = self._buf((n + world * 6 * B,), dev, f32)
            packed[n:].zero_()
            colsum = packed[:n].view(2, B, L)
            bstat = packed[n + slot * 6 * B:n + (slot + 1) * 6 * B].view(6, B)
        nbytes = lib.mpv_fwd_workspace_bytes(shape)
        ws = self._buf((max(nbytes, 1),), dev, torch.uint8)
        if self.gemm == H.GEMM_F16X3:
            ops = (None, None, Rop.c(), eps.c())
        else:
            ops = (H.ptr(Rop), H.ptr(eps), H.Split16(), H.Split16())
        args = H.FwdArgs(H.ptr(y), H.ptr(fe_out), H.ptr(fx_out), self.gemm, *ops, H.ptr(T),
                         H.ptr(rowstat), H.ptr(bstat), H.ptr(colsum), H.ptr(ws), nbytes)
        H.check(lib.mpv_probit_fwd(shape, args, H.stream_of(dev)), "mpv_probit_fwd")
        return dict(rowstat=rowstat, bstat=bstat, colsum=colsum, T=T, packed=packed)

    def _final_args(self, shape, bstat, colsum, fe_mu, fe_logvar, fx_mu, fx_logvar, nll_coeff,
                    c_coeff, seed_advance=None):
        dev = fe_mu.device
        B, L = shape.B, shape.L
        scal = [torch.empty((), device=dev, dtype=torch.float32) for _ in range(6)]
        indiv = torch.empty((B, L), device=dev, dtype=torch.float32)
        indiv_label = torch.empty((B, L), device=dev, dtype=torch.float32)
        args = H.FinalArgs(H.ptr(bstat), H.ptr(colsum), H.ptr(fe_mu), H.ptr(fe_logvar),
                           H.ptr(fx_mu), H.ptr(fx_logvar), fe_mu.shape[1], nll_coeff, c_coeff,
                           *[H.ptr(s) for s in scal], H.ptr(indiv), H.ptr(indiv_label),
                           H.ptr(seed_advance))
        return args, (*scal, indiv, indiv_label)

    def finalize_slots(self, shape, slots, colsum, fe_mu, fe_logvar, fx_mu, fx_logvar, nll_coeff,
                       c_coeff, seed_advance=None):
        """combine_bstats + finalize in one launch (mpv_probit_finalize_shards):
        slots is the all-reduced (world, 6, B) buffer of the shards' bstat.
        Returns (the combined (6, B) bstat, the 8 outputs)."""
        B = shape.B
        bstat = torch.empty((6, B), device=colsum.device, dtype=torch.float32)
        fin, outs = self._final_args(shape, None, colsum, fe_mu, fe_logvar, fx_mu, fx_logvar,
                                     nll_coeff, c_coeff, seed_advance)
        slots = slots.contiguous()
        H.check(H.load_library().mpv_probit_finalize_shards(shape, H.ptr(slots), slots.shape[0],
                                                             H.ptr(bstat), fin,
                                                             H.stream_of(colsum.device)),
                "mpv_probit_finalize_shards")
        return bstat, outs

    def combine_bstats(self, gathered):
        R, _, B = gathered.shape
        out = torch.empty((6, B), device=gathered.device, dtype=torch.float32)
        H.check(H.load_library().mpv_bstat_combine(H.ptr(gathered.contiguous()), R, B, H.ptr(out),
                                                   H.stream_of(gathered.device)),
                "mpv_bstat_combine")
        return out

    def finalize(self, shape, bstat, colsum, fe_mu, fe_logvar, fx_mu, fx_logvar, nll_coeff,
                 c_coeff, seed_advance=None):
        """The 8 outputs; seed_advance: a device Philox key (int64 tensor) this
        step's noise has read, advanced by 1 in the same launch."""
        args, outs = self._final_args(shape, bstat, colsum, fe_mu, fe_logvar, fx_mu, fx_logvar,
                                      nll_coeff, c_coeff, seed_advance)
        H.check(H.load_library().mpv_probit_finalize(shape, args, H.stream_of(bstat.device)),
                "mpv_probit_finalize")
        return outs

    def backward_local(self, shape, saved, gscal, live, g_I, g_IL, nll_coeff, c_coeff, want_dR,
                       dR_dtype=torch.float32, kl=False):
        """d fe_out, d fx_out and (want_dR) d r_sqrt_sigma of this shard.
        dR_dtype float64: dR written in fp64 directly (no cross-shard sum may
        follow: it is then not part of the packed fp32 buffer).  kl: the KL
        backward runs in the same call (saved fe_mu ... fx_logvar)."""
        lib = H.load_library()
        dev = gscal.device
        B, L, z = shape.B, shape.L, shape.z
        n_fe = 2 * B * L
        dR64 = None
        if want_dR and dR_dtype == torch.float64:
            dR64 = self._buf((L, z), dev, torch.float64)
        with_32 = want_dR and dR64 is None
        flat = self._buf((n_fe + (L * z if with_32 else 0),), dev, torch.float32)
        dfe_dfx = flat[:n_fe].view(2, B, L)
        dR = flat[n_fe:].view(L, z) if with_32 else dR64
        nbytes = lib.mpv_bwd_workspace_bytes(shape, self.gemm)
        ws = self._buf((max(nbytes, 1),), dev, torch.uint8)
        eps = saved["eps"]
        eps_ops = (None, eps.c()) if self.gemm == H.GEMM_F16X3 else (H.ptr(eps), H.Split16())
        kl_outs, kl_ref = None, None
        if kl:
            kl_args, kl_outs = self._kl_args(saved["fe_mu"], saved["fe_logvar"], saved["fx_mu"],
                                             saved["fx_logvar"], gscal, live)
            kl_ref = ctypes.byref(kl_args)
        args = H.BwdArgs(H.ptr(saved["y"]), H.ptr(saved["fe_out"]), H.ptr(saved["fx_out"]),
                         self.gemm, *eps_ops, H.ptr(saved["T"]), H.ptr(saved["rowstat"]),
                         H.ptr(saved["bstat"]), H.ptr(gscal), H.ptr(g_I), H.ptr(g_IL),
                         nll_coeff, c_coeff, live, H.ptr(dfe_dfx),
                         H.ptr(dR if with_32 else None), H.ptr(ws), nbytes, H.ptr(dR64),
                         ctypes.cast(kl_ref, ctypes.c_void_p) if kl_ref is not None else None)
        H.check(lib.mpv_probit_bwd(shape, args, H.stream_of(dev)), "mpv_probit_bwd")
        if kl:
            return flat, dfe_dfx, dR, kl_outs
        return flat, dfe_dfx, dR

    @staticmethod
    def _kl_args(fe_mu, fe_logvar, fx_mu, fx_logvar, gscal, live=0x3F):
        B, d = fe_mu.shape
        outs = [torch.empty_like(fe_mu) for _ in range(4)]
        args = H.KlBwdArgs(H.ptr(fe_mu), H.ptr(fe_logvar), H.ptr(fx_mu), H.ptr(fx_logvar), B, d,
                           H.ptr(gscal), *[H.ptr(o) for o in outs], live)
        return args, outs  # outs: g_fe_mu, g_fe_logvar, g_fx_mu, g_fx_logvar

    def kl_backward(self, fe_mu, fe_logvar, fx_mu, fx_logvar, gscal, live=0x3F):
        args, outs = self._kl_args(fe_mu, fe_logvar, fx_mu, fx_logvar, gscal, live)
        H.check(H.load_library().mpv_kl_bwd(args, H.stream_of(fe_mu.device)), "mpv_kl_bwd")
        return outs


class LocalExchange:
    """Single shard: global statistics are the local ones."""
    world = 1

    def verify_replicas(self, tensors):
        pass

    def stat_slots(self):
        return None

    def combine(self, loc, backend):
        return loc["bstat"], loc["colsum"]

    def reduce_grads(self, flat):
        return flat


class ElboConfig:
    """Non-tensor arguments of ProbitELBO."""

    def __init__(self, S_total, S_local, s_offset, nll_coeff, c_coeff, noise="explicit",
                 seed=0, offset=0, backend=None, exchange=None, gemm="f16x3", seed_advance=None):
        self.S_total, self.S_local, self.s_offset = int(S_total), int(S_local), int(s_offset)
        self.nll_coeff, self.c_coeff = float(nll_coeff), float(c_coeff)
        # seed: an int, or a one-element int64 device tensor (HipShardBackend.make_noise)
        self.noise, self.offset = noise, int(offset)
        self.seed = seed if isinstance(seed, torch.Tensor) else int(seed)
        self.backend = backend if backend is not None else HipShardBackend(gemm)
        # a device int64 key tensor the finalize launch advances by 1 once the
        # noise has read it (args.mpvae_seed_advance), or None
        self.seed_advance = seed_advance
        self.exchange = exchange if exchange is not None else LocalExchange()


class ProbitELBO(torch.autograd.Function):
    """(total, nll, nll_x, c, c_x, kl, indiv_prob, indiv_prob_label) of mpvae.py:145-210."""

    @staticmethod
    def forward(ctx, y, fe_out, fe_mu, fe_logvar, fx_out, fx_mu, fx_logvar, R, eps, cfg):
        be = cfg.backend
        y, fe_out, fx_out = _f32(y, "input_label"), _f32(fe_out, "fe_out"), _f32(fx_out, "fx_out")
        fe_mu, fe_logvar = _f32(fe_mu, "fe_mu"), _f32(fe_logvar, "fe_logvar")
        fx_mu, fx_logvar = _f32(fx_mu, "fx_mu"), _f32(fx_logvar, "fx_logvar")
        B, L = y.shape
        if fe_out.shape != (B, L) or fx_out.shape != (B, L):
            raise ValueError(f"fe_out/fx_out must be {(B, L)}, got {tuple(fe_out.shape)}, "
                             f"{tuple(fx_out.shape)}")
        if R.dim() != 2 or R.shape[0] != L:
            raise ValueError(f"r_sqrt_sigma must be (label_dim={L}, z_dim), got {tuple(R.shape)}")
        z = R.shape[1]
        cfg.exchange.verify_replicas((y, fe_out, fx_out, R))
        shape = be.shape(cfg.S_local, cfg.S_total, cfg.s_offset, B, L, z)
        if cfg.noise == "philox" and hasattr(be, "make_noise_and_R"):
            # small r_sqrt_sigma: its split rides on the noise launch
            eps, Rop = be.make_noise_and_R(shape, y.device, cfg.seed, cfg.offset, R)
        else:
            if cfg.noise == "philox":
                eps = be.make_noise(shape, y.device, cfg.seed, cfg.offset)
            else:
                eps = _f32(eps, "noise")
                if tuple(eps.shape) != (cfg.S_local, B, z):
                    raise ValueError(f"noise must be {(cfg.S_local, B, z)}, "
                                     f"got {tuple(eps.shape)}")
                eps = be.prepare_noise(eps, shape)
            Rop = be.prepare_R(R)
        need = ctx.needs_input_grad
        keep_T = need[1] or need[4] or need[7]
        fin = (fe_mu, fe_logvar, fx_mu, fx_logvar, cfg.nll_coeff, cfg.c_coeff)
        adv = {} if cfg.seed_advance is None else {"seed_advance": cfg.seed_advance}
        loc = be.forward_local(shape, y, fe_out, fx_out, Rop, eps, keep_T,
                               stat_slots=cfg.exchange.stat_slots())
        gathered = (cfg.exchange.gather_slots(loc)
                    if hasattr(be, "finalize_slots") and hasattr(cfg.exchange, "gather_slots")
                    else None)
        if gathered is not None:
            # sharded: the exact cross-shard combine inside the finalize launch
            bstat, outs = be.finalize_slots(shape, gathered[0], gathered[1], *fin, **adv)
        else:
            bstat, colsum = cfg.exchange.combine(loc, be)
            outs = be.finalize(shape, bstat, colsum, *fin, **adv)
        ctx.set_materialize_grads(False)
        ctx.cfg, ctx.shape, ctx.r_dtype, ctx.keep_T = cfg, shape, R.dtype, keep_T
        ctx.consumed = False
        if any(need[:8]):
            ctx.saved = dict(y=y, fe_out=fe_out, fx_out=fx_out, eps=eps, T=loc["T"],
                             rowstat=loc["rowstat"], bstat=bstat, fe_mu=fe_mu,
                             fe_logvar=fe_logvar, fx_mu=fx_mu, fx_logvar=fx_logvar)
        return outs

    @staticmethod
    def backward(ctx, g_total, g_nll, g_nll_x, g_c, g_c_x, g_kl, g_I, g_IL):
        if ctx.consumed:
            raise RuntimeError("ProbitELBO backward reuses its forward buffers in place; "
                               "backward through the same compute_loss twice is not supported")
        ctx.consumed = True
        cfg, shape, be, sv = ctx.cfg, ctx.shape, ctx.cfg.backend, ctx.saved
        need = ctx.needs_input_grad
        gs = [g_total, g_nll, g_nll_x, g_c, g_c_x, g_kl]
        live = sum(1 << i for i, g in enumerate(gs) if g is not None)
        dev = sv["y"].device
        if getattr(be, "reads_live_slots", False) and live == 1:
            # total_loss.backward() alone: the kernels read only the live slot,
            # so the upstream gradient's own storage is gscal (no zeros + stack:
            # two launches fewer per step)
            gscal = gs[0].reshape((1,)).to(torch.float32).contiguous()
        else:
            zero = torch.zeros((), device=dev, dtype=torch.float32)
            gscal = torch.stack([zero if g is None else g.reshape(()).to(torch.float32)
                                 for g in gs])
        g_I = None if g_I is None else g_I.to(torch.float32).contiguous()
        g_IL = None if g_IL is None else g_IL.to(torch.float32).contiguous()
        grads = [None] * 10
        want_kl = need[2] or need[3] or need[5] or need[6]
        gk = None
        if ctx.keep_T and (need[1] or need[4] or need[7]):
            # one shard: dR straight in R's dtype and the KL backward in the
            # same call (two launches fewer); sharded: the packed fp32 buffer
            # is summed over the ranks first
            local = getattr(cfg.exchange, "world", 1) == 1 and isinstance(cfg.exchange,
                                                                         LocalExchange)
            dR_dtype = ctx.r_dtype if local else torch.float32
            res = be.backward_local(shape, sv, gscal, live, g_I, g_IL, cfg.nll_coeff,
                                    cfg.c_coeff, need[7], dR_dtype=dR_dtype, kl=want_kl)
            flat, dfe_dfx, dR = res[:3]
            if want_kl:
                gk = res[3]
            cfg.exchange.reduce_grads(flat)
            if need[1]:
                grads[1] = dfe_dfx[0]
            if need[4]:
                grads[4] = dfe_dfx[1]
            if need[7]:
                grads[7] = dR if dR.dtype == ctx.r_dtype else be.from_f32(dR, ctx.r_dtype)
        if want_kl:
            if gk is None:
                gk = be.kl_backward(sv["fe_mu"], sv["fe_logvar"], sv["fx_mu"], sv["fx_logvar"],
                                    gscal, **({"live": live} if getattr(be, "reads_live_slots",
                                                                       False) else {}))
            grads[2], grads[3], grads[5], grads[6] = gk
        ctx.saved = None
        return tuple(grads)


class FusedReparam(torch.autograd.Function):
    """z = mu + eps*exp(0.5*logvar) for the label and the feature encoder in one
    launch (mpvae.py:66-74).  eps is an input (drawn by the caller with
    torch.randn_like, so the RNG stream matches the reference's draw order).

    mu and logvar are also returned, as fresh copies the kernel writes in the
    same pass (ordinary tensors: a caller may modify them in place, as it may
    the reference's): the VAE returns those to the caller, so the gradient
    compute_loss's KL sends them arrives here and is added inside
    mpv_reparam_bwd -- the one add autograd would otherwise launch per tensor
    when two consumers of an encoder head meet."""

    @staticmethod
    def forward(ctx, mu_e, lv_e, eps_e, mu_x, lv_x, eps_x):
        H.require_gpu(mu_e, mu_x)
        mu_e, lv_e, eps_e = (_f32(t, "reparam input") for t in (mu_e, lv_e, eps_e))
        mu_x, lv_x, eps_x = (_f32(t, "reparam input") for t in (mu_x, lv_x, eps_x))
        z_e, z_x = torch.empty_like(mu_e), torch.empty_like(mu_x)
        outs = [torch.empty_like(t) for t in (mu_e, lv_e, mu_x, lv_x)]
        a = H.ReparamArgs(H.ptr(mu_e), H.ptr(lv_e), H.ptr(eps_e), H.ptr(z_e), mu_e.numel(),
                          H.ptr(mu_x), H.ptr(lv_x), H.ptr(eps_x), H.ptr(z_x), mu_x.numel(),
                          *[H.ptr(o) for o in outs])
        H.check(H.load_library().mpv_reparam_fwd(a, H.stream_of(mu_e.device)), "mpv_reparam_fwd")
        ctx.save_for_backward(lv_e, eps_e, lv_x, eps_x)
        ctx.set_materialize_grads(False)
        return (z_e, z_x, *outs)

    @staticmethod
    def backward(ctx, gz_e, gz_x, gmu_e_in, glv_e_in, gmu_x_in, glv_x_in):
        lv_e, eps_e, lv_x, eps_x = ctx.saved_tensors
        gmu_e, glv_e = torch.empty_like(lv_e), torch.empty_like(lv_e)
        gmu_x, glv_x = torch.empty_like(lv_x), torch.empty_like(lv_x)
        c = lambda g: None if g is None else _f32(g, "reparam gradient")
        gz_e, gz_x = c(gz_e), c(gz_x)
        gmu_e_in, glv_e_in, gmu_x_in, glv_x_in = (c(g) for g in (gmu_e_in, glv_e_in, gmu_x_in,
                                                                  glv_x_in))
        a = H.ReparamBwdArgs(H.ptr(gz_e), H.ptr(lv_e), H.ptr(eps_e), H.ptr(gmu_e), H.ptr(glv_e),
                             lv_e.numel(), H.ptr(gz_x), H.ptr(lv_x), H.ptr(eps_x), H.ptr(gmu_x),
                             H.ptr(glv_x), lv_x.numel(), H.ptr(gmu_e_in), H.ptr(glv_e_in),
                             H.ptr(gmu_x_in), H.ptr(glv_x_in))
        H.check(H.load_library().mpv_reparam_bwd(a, H.stream_of(lv_e.device)), "mpv_reparam_bwd")
        return gmu_e, glv_e, None, gmu_x, glv_x, None


class SingleReparam(torch.autograd.Function):
    """One encoder's reparameterisation (label_reparameterize / feat_reparameterize)."""

    @staticmethod
    def forward(ctx, mu, lv, eps):
        H.require_gpu(mu)
        mu, lv, eps = (_f32(t, "reparam input") for t in (mu, lv, eps))
        z = torch.empty_like(mu)
        a = H.ReparamArgs(H.ptr(mu), H.ptr(lv), H.ptr(eps), H.ptr(z), mu.numel(),
                          None, None, None, None, 0, None, None, None, None)
        H.check(H.load_library().mpv_reparam_fwd(a, H.stream_of(mu.device)), "mpv_reparam_fwd")
        ctx.save_for_backward(lv, eps)
        return z

    @staticmethod
    def backward(ctx, gz):
        lv, eps = ctx.saved_tensors
        gmu, glv = torch.empty_like(lv), torch.empty_like(lv)
        a = H.ReparamBwdArgs(H.ptr(gz.contiguous()), H.ptr(lv), H.ptr(eps), H.ptr(gmu),
                             H.ptr(glv), lv.numel(), None, None, None, None, None, 0)
        H.check(H.load_library().mpv_reparam_bwd(a, H.stream_of(lv.device)), "mpv_reparam_bwd")
        return gmu, glv, None
