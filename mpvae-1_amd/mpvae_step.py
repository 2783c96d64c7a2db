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
