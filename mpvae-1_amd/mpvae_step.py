"""The per-step host syncs of the reference training loop, batched (SURVEY.md
section 8(f) rank 3).

After ``total_loss.backward()`` the reference loop (fairsoft_train.py:140-162)
synchronises with the device once per parameter in ``has_finite_grad``
(fairsoft_utils.py:28-41: ``torch.isnan(g).any() or torch.isinf(g).any()`` is a
host bool per tensor) and once per logged scalar (eight ``.item()`` calls,
fairsoft_train.py:154-162).  Each sync drains the stream.  Here:

* ``has_finite_grad(model)`` -- the same answer from one fused multi-tensor
  reduction and one sync: max |g| of every gradient (``torch._foreach_norm``
  with ord = inf, which propagates NaN and cannot overflow), all finite;
* ``step_scalars(**tensors)`` -- every 0-d tensor the loop logs, fetched by ONE
  device-to-host copy, as Python floats (what ``.item()`` returns).

Both are torch glue around the loop, not kernels of the hot path: they run on
whatever device the tensors live on.
"""
import copy
import ctypes
import functools

import torch


def has_finite_grad(model):
    """fairsoft_utils.py:28-41 with one host sync: True iff every existing
    gradient of ``model`` (a module, or a tensor with .grad) is finite."""
    if isinstance(model, torch.Tensor):
        grads = [model.grad]
    else:
        grads = [p.grad for p in model.parameters() if p.grad is not None]
    grads = [g for g in grads if g is not None]
    if not grads:
        return True
    peaks = torch._foreach_norm(grads, float("inf"))
    by_dtype = {}
    for pk in peaks:  # one stack per dtype (fp32 MLP grads, fp64 r_sqrt_sigma grad)
        by_dtype.setdefault(pk.dtype, []).append(pk)
    ok = [torch.isfinite(torch.stack(v)).all() for v in by_dtype.values()]
    return bool((torch.stack(ok).all() if len(ok) > 1 else ok[0]).item())


def step_scalars(**tensors):
    """{name: float} for 0-d tensors (loss components, device metrics) with one
    device-to-host copy instead of one ``.item()`` each (fairsoft_train.py:
    154-162).  Non-tensor values pass through unchanged."""
    names = [k for k, v in tensors.items() if isinstance(v, torch.Tensor)]
    out = {k: v for k, v in tensors.items() if not isinstance(v, torch.Tensor)}
    if names:
        vals = torch.stack([tensors[k].detach().reshape(()).to(torch.float64) for k in names])
        for k, v in zip(names, vals.cpu().tolist()):
            out[k] = v
    return out


def _native_adam(opt):
    """True when ``opt`` is a plain fused torch.optim.Adam that mpv_adam_step
    reproduces (L2 weight decay, float lr, no amsgrad / maximize /
    decoupled weight decay, CUDA parameters)."""
    if type(opt) is not torch.optim.Adam:
        return False
    for g in opt.param_groups:
        if (not g.get("fused") or g.get("amsgrad") or g.get("maximize")
                or g.get("differentiable") or g.get("decoupled_weight_decay", False)
                or isinstance(g["lr"], torch.Tensor) or isinstance(g["betas"][0], torch.Tensor)):
            return False
        if any(p.device.type != "cuda" or p.dtype not in (torch.float32, torch.float64)
               for p in g["params"]):
            return False
    return True


def adam_step(opt, found_inf, updates=None, sched=None):
    """optimizer.step() of a fused torch.optim.Adam in one mpv_adam_step launch
    per parameter group (csrc/adam.hip) instead of torch's multi-tensor kernel,
    which runs the VAE's 1.5 M parameters on ~25 workgroups (DESIGN.md
    section 11), then one mpv_adam_finish launch.  Same state (``step``,
    ``exp_avg``, ``exp_avg_sq`` in ``opt.state``), same step-count protocol as
    torch's capturable fused path (+1 for the update, -found_inf after), same
    per-element arithmetic; nothing is written when ``found_inf`` is 1.
    ``updates`` (an int64 device scalar, or None) counts the applied updates
    and ``sched`` (a DeviceStepLR, or None) takes the scheduler step the
    reference takes after an applied update (fairsoft_train.py:142-146), both
    in the finish launch."""
    import mpvae_hip as H
    lib = H.load_library()
    all_steps = []
    for gi, g in enumerate(opt.param_groups):
        params = [p for p in g["params"] if p.grad is not None]
        if not params:
            continue
        for p in params:
            st = opt.state[p]
            if len(st) == 0:  # torch's _init_group for fused Adam
                st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        all_steps += [opt.state[p]["step"] for p in params]
        beta1, beta2 = g["betas"]
        lr_dev = None if sched is None else sched.lr[gi:gi + 1]
        for c in range(0, len(params), H.ADAM_MAX_TENSORS):
            a = H.AdamArgs(n=0, lr=float(g["lr"]), beta1=float(beta1), beta2=float(beta2),
                           weight_decay=float(g["weight_decay"]), eps=float(g["eps"]),
                           found_inf=H.ptr(found_inf), lr_dev=H.ptr(lr_dev))
            for p in params[c:c + H.ADAM_MAX_TENSORS]:
                st = opt.state[p]
                ts = (p, p.grad, st["exp_avg"], st["exp_avg_sq"])
                if not all(t.is_contiguous() and t.dtype == p.dtype for t in ts):
                    raise ValueError("mpv_adam_step needs contiguous parameters, gradients "
                                     "and state of the parameter's dtype")
                a.t[a.n] = H.AdamTensor(param=p.data_ptr(), grad=p.grad.data_ptr(),
                                        exp_avg=st["exp_avg"].data_ptr(),
                                        exp_avg_sq=st["exp_avg_sq"].data_ptr(),
                                        step=st["step"].data_ptr(), numel=p.numel(),
                                        is_f64=int(p.dtype == torch.float64))
                a.n += 1
            H.check(lib.mpv_adam_step(ctypes.byref(a), H.stream_of(params[0].device)),
                    "mpv_adam_step")
    if not all_steps and updates is None and sched is None:
        return
    dev = (all_steps[0] if all_steps else updates if updates is not None else sched.lr).device
    for c in range(0, max(1, len(all_steps)), H.ADAM_FINISH_MAX):
        chunk = all_steps[c:c + H.ADAM_FINISH_MAX]
        f = H.AdamFinishArgs(n_steps=len(chunk), found_inf=H.ptr(found_inf))
        for i, st in enumerate(chunk):
            f.steps[i] = st.data_ptr()
        if c == 0:  # the counter and the scheduler step once per optimizer step
            f.updates = H.ptr(updates)
            if sched is not None:
                f.n_lr, f.lr, f.last_epoch = sched.lr.numel(), H.ptr(sched.lr), \
                    H.ptr(sched.last_epoch)
                f.step_size, f.gamma = sched.step_size, sched.gamma
        H.check(lib.mpv_adam_finish(ctypes.byref(f), H.stream_of(dev)), "mpv_adam_finish")


class DeviceStepLR:
    """The state of a torch.optim.lr_scheduler.StepLR (fairsoft_jaccard.py:67-68)
    held on the device, so TrainStep can take the reference's scheduler step
    (after an applied update only, fairsoft_train.py:142-145) with no host
    sync and inside a captured graph.  ``lr`` holds one float64 learning rate
    per param group, ``last_epoch`` the scheduler's epoch counter; both follow
    torch's StepLR bit for bit (the chainable ``lr * gamma`` in double when
    last_epoch is a non-zero multiple of step_size).  The optimizer's
    ``param_groups[i]["lr"]`` and the scheduler's ``last_epoch`` /
    ``get_last_lr()`` would go stale while TrainStep owns them; so (ADVICE
    r04):
      * ``opt.state_dict()`` and ``sched.state_dict()`` sync first (an
        optimizer state-dict pre-hook; the scheduler's method wrapped), so a
        checkpoint holds the current lr and epoch;
      * the scheduler's own ``step()`` raises while TrainStep owns it (the
        reference loop's host ``scheduler.step()`` would step it twice) until
        ``release()`` hands it back, synced;
      * a host edit of ``param_groups[i]["lr"]`` is adopted by the device
        state before the next step (``adopt_host_lr``, called by TrainStep: a
        host-side comparison, no device sync), with a warning.
    ``sync()`` (one host sync) writes the device state back on demand, e.g.
    before logging."""

    def __init__(self, sched, opt):
        if type(sched) is not torch.optim.lr_scheduler.StepLR:
            raise ValueError("TrainStep runs torch.optim.lr_scheduler.StepLR (the reference's "
                             f"scheduler) on the device; got {type(sched).__name__}")
        if sched.optimizer is not opt:
            raise ValueError("the scheduler must wrap TrainStep's optimizer")
        dev = next(p.device for g in opt.param_groups for p in g["params"])
        self.sched, self.opt = sched, opt
        self.lr = torch.tensor([float(g["lr"]) for g in opt.param_groups], dtype=torch.float64,
                               device=dev)
        self.last_epoch = torch.tensor(int(sched.last_epoch), dtype=torch.int64, device=dev)
        self.step_size, self.gamma = float(sched.step_size), float(sched.gamma)
        self._epoch0 = int(sched.last_epoch)
        self._host_lr = [float(g["lr"]) for g in opt.param_groups]  # as last synced / adopted
        self._hook = opt.register_state_dict_pre_hook(lambda _opt: self.sync())
        self._sched_state_dict, self._sched_step = sched.state_dict, sched.step
        self._sched_load = sched.load_state_dict

        def state_dict():
            self.sync()
            return self._sched_state_dict()

        def load_state_dict(state):
            # a resumed scheduler checkpoint: the device epoch and
            # lr follow it, so the decay boundaries are the checkpoint's and
            # the next sync() does not write a stale epoch back
            self._sched_load(state)
            self._adopt(int(sched.last_epoch), [float(g["lr"]) for g in opt.param_groups])

        def step(*a, **k):
            raise RuntimeError("this StepLR is stepped on the device by TrainStep after every "
                               "applied update (fairsoft_train.py:142-145); do not call "
                               "scheduler.step() as well -- TrainStep.release_scheduler() hands "
                               "it back")
        sched.state_dict, sched.step, sched.load_state_dict = state_dict, step, load_state_dict

    def _adopt(self, epoch, lrs):
        """Host values -> the device state, stream-ordered, without a host wait:
        the lrs go through a pinned staging tensor (the caching host allocator
        keeps it alive until the copy has run)."""
        src = torch.tensor(lrs, dtype=torch.float64)
        if self.lr.is_cuda:
            src = src.pin_memory()
        self.lr.copy_(src, non_blocking=True)
        if epoch is not None:
            self.last_epoch.fill_(epoch)
            self._epoch0 = epoch
        self._host_lr = list(lrs)

    def sync(self):
        """Copy the device lr / last_epoch into the optimizer and the scheduler."""
        lrs = self.lr.tolist()
        epoch = int(self.last_epoch)
        for g, v in zip(self.opt.param_groups, lrs):
            g["lr"] = v
        self.sched.last_epoch = epoch
        self.sched._last_lr = list(lrs)
        self.sched._step_count += epoch - self._epoch0
        self._epoch0 = epoch
        self._host_lr = list(lrs)
        return lrs

    def adopt_host_lr(self):
        """A param group's lr changed on the host since the last sync: the
        device lr takes it (a host-side compare; the copy is stream-ordered from
        a pinned staging tensor, so the host does not wait for the device)."""
        now = [float(g["lr"]) for g in self.opt.param_groups]
        if now != self._host_lr:
            import warnings
            warnings.warn("optimizer param_groups lr edited on the host while TrainStep owns "
                          "the StepLR: the device lr adopts the new value", stacklevel=3)
            self._adopt(None, now)

    def release(self):
        """Sync, then hand the scheduler and optimizer back to host control."""
        lrs = self.sync()
        self._hook.remove()
        self.sched.state_dict, self.sched.step = self._sched_state_dict, self._sched_step
        self.sched.load_state_dict = self._sched_load
        return lrs


class TrainStep:
    """The loop body of fairsoft_train.py:47-146 (penalty-free) as one call:
    ``model(label, feat)`` -> ``compute_loss`` -> ``backward`` ->
    ``clip_grad_norm_(10)`` -> finite-gradient gate -> optimizer step.

    The gate runs on the device: the optimizer must be a fused Adam
    (``torch.optim.Adam(..., fused=True)``), which takes ``found_inf`` and skips
    the update on the device, step counters included -- the reference's
    ``if has_finite_grad(model): optimizer.step()`` without the host sync.
    ``updates`` counts the applied steps (the reference's succses_updates) on
    the device.  ``scheduler``: the reference's StepLR (fairsoft_jaccard.py:
    67-68), stepped on the device after every applied update
    (fairsoft_train.py:142-145; DeviceStepLR, ``sync_scheduler()`` writes its
    state back to the host objects).  With ``args.mpvae_noise = "philox"`` and
    a device-tensor ``args.mpvae_seed`` nothing in the step waits for the
    host, so ``capture()`` records it in one HIP graph (input batches are
    copied into the static ``label`` / ``feat`` buffers before each
    ``replay()``)."""

    def __init__(self, model, optimizer, args, max_grad_norm=10.0, advance_seed=True,
                 native_adam=True, scheduler=None):
        if not optimizer.defaults.get("fused"):
            raise ValueError("TrainStep gates the update on the device: use a fused optimizer "
                             "(torch.optim.Adam(..., fused=True))")
        self.model, self.opt, self.args = model, optimizer, args
        self.max_grad_norm = max_grad_norm
        self.advance_seed = advance_seed
        # a plain fused Adam steps in mpv_adam_step (adam_step); others in torch
        self.native_adam = bool(native_adam) and _native_adam(optimizer)
        self.params = [p for p in model.parameters() if p.requires_grad]
        dev = self.params[0].device
        self.updates = torch.zeros((), dtype=torch.int64, device=dev)
        self.found_inf = torch.zeros((), dtype=torch.float32, device=dev)
        self._one = torch.ones((), dtype=torch.float32, device=dev)
        self.sched = None
        if scheduler is not None:
            if not self.native_adam:
                raise ValueError("a device StepLR needs the native Adam step (a plain fused "
                                 "torch.optim.Adam with a float lr)")
            self.sched = DeviceStepLR(scheduler, optimizer)
        self.graph = None
        self.label = self.feat = self.out = None

    def _clip(self):
        """torch.nn.utils.clip_grad_norm_(params, max_grad_norm) (fairsoft_train.py:141)
        with the same total norm and coefficient (computed in the promoted
        dtype: fp64, as r_sqrt_sigma's gradient is fp64), but the coefficient
        cast to each gradient dtype before the multi-tensor multiply: torch's
        own version multiplies fp32 gradients by an fp64 0-d tensor, which
        leaves the multi-tensor fast path for one type-promoting multiply and
        one copy per tensor (52 launches at the VAE's 26 fp32 gradients).  A
        clipped fp32 gradient may differ from torch's by one ulp; an unclipped
        one (coefficient 1) is untouched either way."""
        by_dtype = {}
        for p in self.params:
            if p.grad is not None:
                by_dtype.setdefault(p.grad.dtype, []).append(p.grad)
        if not by_dtype:
            return
        # torch stacks the per-tensor norms of every dtype into one promoted
        # (fp64) vector, which casts each fp32 norm in a launch of its own (26
        # at the VAE); here each dtype's norms are stacked and cast once: the
        # same vector, in the same order
        wide = functools.reduce(torch.promote_types, by_dtype)
        parts = [torch.stack(torch._foreach_norm(grads, 2.0)).to(wide)
                 for grads in by_dtype.values()]
        total = torch.linalg.vector_norm(parts[0] if len(parts) == 1 else torch.cat(parts), 2.0)
        coef = torch.clamp(self.max_grad_norm / (total + 1e-6), max=1.0)
        for dt, grads in by_dtype.items():
            torch._foreach_mul_(grads, coef.to(dt))

    def _body(self, label, feat):
        import mpvae
        self.opt.zero_grad(set_to_none=True)
        seed = getattr(self.args, "mpvae_seed", None)
        args = self.args
        if self.advance_seed and isinstance(seed, torch.Tensor):
            # fresh probit noise every step, on the device: compute_loss's
            # finalize launch advances the key after the noise has read it
            # (args.mpvae_seed_advance; no launch of its own)
            args = copy.copy(self.args)
            args.mpvae_seed_advance = True
        out = self.model(label, feat)
        res = mpvae.compute_loss(label, *out, self.model.r_sqrt_sigma, args)
        res[0].backward()
        self._clip()
        # finite gate: the AMP multi-tensor check (one launch per dtype) sets
        # found_inf if any gradient holds a NaN / inf; its unscale by 1.0
        # leaves every value as it is
        self.found_inf.zero_()
        by_dtype = {}
        for p in self.params:
            if p.grad is not None:
                by_dtype.setdefault(p.grad.dtype, []).append(p.grad)
        for grads in by_dtype.values():
            torch._amp_foreach_non_finite_check_and_unscale_(grads, self.found_inf, self._one)
        if self.native_adam:
            # the update, then the step counts, `updates` and the scheduler in
            # one finish launch (counted even when no parameter has a gradient,
            # as the reference's gate passes such a step)
            adam_step(self.opt, self.found_inf, self.updates, self.sched)
        else:
            self.opt.found_inf = self.found_inf
            try:
                self.opt.step()
            finally:
                del self.opt.found_inf
            self.updates.add_(1 - self.found_inf.to(torch.int64))
        return res

    def sync_scheduler(self):
        """The device StepLR's learning rates written back into the optimizer's
        param_groups and the scheduler (one host sync); returns them."""
        return None if self.sched is None else self.sched.sync()

    def release_scheduler(self):
        """Sync and give the StepLR back to host control (its step() works
        again); TrainStep then no longer steps it.  A graph captured before
        holds the device lr / epoch and the scheduler step in its Adam launches
        (ADVICE r05): it is dropped, so later calls run eagerly on the host lr
        until capture() records the step again."""
        if self.sched is None:
            return None
        lrs, self.sched = self.sched.release(), None
        if self.graph is not None:
            self.graph = None
            self.label = self.feat = self.out = None
        return lrs

    def __call__(self, label, feat):
        """One eager step; returns compute_loss's 8 outputs (device tensors)."""
        if self.sched is not None:
            self.sched.adopt_host_lr()
        if self.graph is not None:
            self.label.copy_(label)
            self.feat.copy_(feat)
            self.graph.replay()
            return self.out
        return self._body(label, feat)

    def capture(self, label, feat, warmup=2):
        """Record the step in a HIP graph on static copies of (label, feat);
        later calls copy their batch in and replay.  ``warmup`` eager steps on a
        side stream first (they update the model, as any step does).  The
        optimizer must be built with ``capturable=True`` (its step counter and
        bias corrections then live on the device)."""
        if not all(g.get("capturable") for g in self.opt.param_groups):
            raise ValueError("capture() needs torch.optim.Adam(..., fused=True, capturable=True)")
        self.label, self.feat = label.clone(), feat.clone()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                self._body(self.label, self.feat)
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        self.opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(self.graph):
            self.out = self._body(self.label, self.feat)
        return self.graph
