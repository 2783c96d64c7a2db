"""The VAE's Linear layers on the fp32 matrix cores (csrc/linear.hip).

``linear(x, layer, relu=False, alpha=1.0)`` computes
``act(alpha * (x @ layer.weight.T + layer.bias))`` -- nn.Linear, the F.relu
after it (reference mpvae.py:53,58-62,78-84) and the ``* scale_coeff`` of the
mu / logvar heads (:54-55,63-64) in one launch pair -- and its backward
(d x, d W, d b, the ReLU mask and the scale folded into the GEMM operand
loads) in one more.  The parameters stay the reference's ``nn.Linear`` modules, so
state_dict, optimiser and initialisation are unchanged.

Why not nn.Linear: at the reference's batch sizes (32-512 rows) hipBLASLt tiles
these GEMMs into a handful of workgroups that walk K ~ 1000 on one CU each
(65-155 us per GEMM at C3, ~45 % of the drop-in training step,
profiles/r03_c3_trainstep.json); mpv_linear splits the reduction until the
launch fills the chip and sums the chunks in a fixed order (deterministic).
"""
import ctypes

import torch

import mpvae_hip as H


def _problem(M, N, R, a, a_si, a_sr, b, b_sj, b_sr, out, out_si, *, a_mask=None, a_scale=1.0,
             ones_col=-1, out_col=None, bias=None, alpha=1.0, relu=False, seg2=None):
    """seg2 = (R1, a2, a2_si, b2): reduction indices >= R1 read a2 / b2."""
    R1, a2, a2_si, b2 = seg2 if seg2 is not None else (0, None, 0, None)
    return H.LinearArgs(M=M, N=N, R=R, a=H.ptr(a), a_si=a_si, a_sr=a_sr, a_mask=H.ptr(a_mask),
                        a_scale=a_scale, b=H.ptr(b), b_sj=b_sj, b_sr=b_sr, ones_col=ones_col,
                        bias=H.ptr(bias), alpha=alpha, relu=int(bool(relu)), out=H.ptr(out),
                        out_si=out_si, out_col=H.ptr(out_col), a2=H.ptr(a2), a2_si=a2_si,
                        b2=H.ptr(b2), R1=R1)


def _launch(device, *problems):
    """One launch (pair) for 1-4 independent problems."""
    lib = H.load_library()
    arr = (H.LinearArgs * len(problems))(*problems)
    nbytes = lib.mpv_linear_batch_workspace_bytes(arr, len(problems))
    ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
    H.check(lib.mpv_linear_batch(arr, len(problems), H.ptr(ws), nbytes, H.stream_of(device)),
            "mpv_linear")


# the two heads' dx as one two-segment GEMM (False: two GEMMs and an add, A/B)
HEADS_DX_ONE_GEMM = True


def _rows(x):
    """x with unit column stride (row stride free), as the kernels address it."""
    return x if x.stride(1) == 1 else x.contiguous()


class HipLinear(torch.autograd.Function):
    """act(alpha * (x W^T + b)), then (drop_p > 0) torch's own dropout.

    With dropout the forward output is ``native_dropout(relu(...), p)`` --
    the kernel nn.Dropout runs, same generator, same masks -- and the
    backward folds the dropout backward into the gradient GEMMs' operand
    load: out = y * keep / (1 - p) is > 0 exactly where the ReLU passes (y > 0)
    AND the element was kept, so masking the upstream gradient by (out > 0)
    and scaling it by 1 / (1 - p) gives torch's masked_scale + threshold_backward
    values bit for bit, without their launches (alpha must be 1)."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu, alpha, drop_p=0.0):
        H.require_gpu(x, weight, bias)
        if x.dtype != torch.float32 or weight.dtype != torch.float32 or (
                bias is not None and bias.dtype != torch.float32):
            raise TypeError("mpv_linear computes in fp32 (the reference's nn.Linear dtype)")
        if weight.dim() != 2 or (bias is not None and bias.shape != (weight.shape[0],)):
            raise ValueError(f"bad Linear parameters: weight {tuple(weight.shape)}, "
                             f"bias {None if bias is None else tuple(bias.shape)}")
        if x.dim() != 2:
            raise ValueError(f"mpv_linear takes (batch, features) inputs, got {tuple(x.shape)}")
        x = _rows(x)
        w = weight.contiguous()
        M, K = x.shape
        N = w.shape[0]
        if w.shape[1] != K:
            raise ValueError(f"mat1 and mat2 shapes cannot be multiplied ({M}x{K} and "
                             f"{w.shape[1]}x{N})")
        y = torch.empty((M, N), dtype=torch.float32, device=x.device)
        _launch(x.device, _problem(M, N, K, x, x.stride(0), 1, w, K, 1, y, N,
                                   bias=None if bias is None else bias.contiguous(), alpha=alpha,
                                   relu=relu))
        scale = alpha
        if drop_p > 0.0:
            if not relu or alpha != 1.0:
                raise ValueError("the folded dropout backward needs a ReLU layer with alpha 1")
            y, _ = torch.native_dropout(y, drop_p, True)
            # masked_scale's factor, as torch rounds it; p = 1 drops everything
            scale = float(torch.tensor(1.0 / (1.0 - drop_p), dtype=torch.float32)) \
                if drop_p < 1.0 else 0.0
        ctx.save_for_backward(x, w, y if relu else None)
        ctx.alpha, ctx.has_bias = scale, bias is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        gy = gy.contiguous()
        M, K = x.shape
        N = w.shape[0]
        gx = gw = gb = None
        problems = []
        if ctx.needs_input_grad[0]:
            # dx[m, k] = sum_n g[m, n] W[n, k],  g = alpha * dy * (y > 0)
            gx = torch.empty((M, K), dtype=torch.float32, device=x.device)
            problems.append(_problem(M, K, N, gy, N, 1, w, 1, K, gx, K, a_mask=y,
                                     a_scale=ctx.alpha))
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            # dW[n, k] = sum_m g[m, n] x[m, k]; db[n] = sum_m g[m, n] (ones column)
            gw = torch.empty((N, K), dtype=torch.float32, device=x.device)
            gb = torch.empty((N,), dtype=torch.float32, device=x.device) if ctx.has_bias else None
            problems.append(_problem(N, K + (1 if ctx.has_bias else 0), M, gy, 1, N, x, 1,
                                     x.stride(0), gw, K, a_mask=y, a_scale=ctx.alpha,
                                     ones_col=K if ctx.has_bias else -1, out_col=gb))
        if problems:
            _launch(x.device, *problems)  # dx and dW + db in one launch pair
        return gx, gw, gb, None, None, None


def _check_params(x, *wb):
    H.require_gpu(x, *wb)
    if x.dtype != torch.float32 or any(t is not None and t.dtype != torch.float32 for t in wb):
        raise TypeError("mpv_linear computes in fp32 (the reference's nn.Linear dtype)")
    if x.dim() != 2:
        raise ValueError(f"mpv_linear takes (batch, features) inputs, got {tuple(x.shape)}")
    for w, b in zip(wb[::2], wb[1::2]):
        if w.dim() != 2 or w.shape[1] != x.shape[1] or (b is not None and b.shape != (w.shape[0],)):
            raise ValueError(f"bad Linear parameters for input {tuple(x.shape)}: weight "
                             f"{tuple(w.shape)}, bias {None if b is None else tuple(b.shape)}")


class HipLinearHeads(torch.autograd.Function):
    """Two Linear heads of one input, ``(alpha * a(x), alpha * b(x))`` -- an
    encoder's mu and logvar (reference mpvae.py:54-55,63-64) -- in one launch
    pair; the backward's dW, db of both heads and both dx terms in one more."""

    @staticmethod
    def forward(ctx, x, wa, ba, wb, bb, alpha):
        _check_params(x, wa, ba, wb, bb)
        x = _rows(x)
        wa, wb = wa.contiguous(), wb.contiguous()
        M, K = x.shape
        ys = []
        problems = []
        for w, b in ((wa, ba), (wb, bb)):
            y = torch.empty((M, w.shape[0]), dtype=torch.float32, device=x.device)
            problems.append(_problem(M, w.shape[0], K, x, x.stride(0), 1, w, K, 1, y, w.shape[0],
                                     bias=None if b is None else b.contiguous(), alpha=alpha))
            ys.append(y)
        _launch(x.device, *problems)
        ctx.save_for_backward(x, wa, wb)
        ctx.alpha, ctx.has_bias = alpha, (ba is not None, bb is not None)
        return ys[0], ys[1]

    @staticmethod
    def backward(ctx, ga, gb_):
        x, wa, wb = ctx.saved_tensors
        M, K = x.shape
        dev = x.device
        need = ctx.needs_input_grad
        grads = [None] * 6
        problems = []
        ga, gb_ = ga.contiguous(), gb_.contiguous()
        dxs = []
        if need[0] and not HEADS_DX_ONE_GEMM:
            for w, g in ((wa, ga), (wb, gb_)):
                dxs.append(torch.empty((M, K), dtype=torch.float32, device=dev))
                problems.append(_problem(M, K, w.shape[0], g, w.shape[0], 1, w, 1, K, dxs[-1], K,
                                         a_scale=ctx.alpha))
        elif need[0]:
            # dx = ga Wa + gb Wb: one GEMM over the two heads' outputs (two
            # reduction segments), no separate sum
            Na, Nb = wa.shape[0], wb.shape[0]
            grads[0] = torch.empty((M, K), dtype=torch.float32, device=dev)
            problems.append(_problem(M, K, Na + Nb, ga, Na, 1, wa, 1, K, grads[0], K,
                                     a_scale=ctx.alpha, seg2=(Na, gb_, Nb, wb)))
        for k, (w, g) in enumerate(((wa, ga), (wb, gb_))):
            N = w.shape[0]
            if need[1 + 2 * k] or need[2 + 2 * k]:
                hb = ctx.has_bias[k]
                gw = torch.empty((N, K), dtype=torch.float32, device=dev)
                gbias = torch.empty((N,), dtype=torch.float32, device=dev) if hb else None
                problems.append(_problem(N, K + (1 if hb else 0), M, g, 1, N, x, 1, x.stride(0),
                                         gw, K, a_scale=ctx.alpha, ones_col=K if hb else -1,
                                         out_col=gbias))
                grads[1 + 2 * k], grads[2 + 2 * k] = gw, gbias
        if problems:
            _launch(dev, *problems)
        if dxs:
            grads[0] = dxs[0].add_(dxs[1])
        return tuple(grads)


class HipRowHeads(torch.autograd.Function):
    """Two Linear heads on the two row blocks of one stacked input,
    ``(a(h[:n_a]), b(h[n_a:]))`` -- the label and feature decoders' last
    layers after their shared fd_x1 / fd_x2 ran on both inputs stacked
    (reference mpvae.py:76-84) -- in one launch pair, and their backward (the
    stacked d h and both dW, db) in one more."""

    @staticmethod
    def forward(ctx, h, wa, ba, wb, bb, n_a):
        _check_params(h, wa, ba, wb, bb)
        h = _rows(h)
        wa, wb = wa.contiguous(), wb.contiguous()
        M, K = h.shape
        if not 0 <= n_a <= M:
            raise ValueError(f"row split {n_a} outside 0..{M}")
        blocks = ((0, n_a, wa, ba), (n_a, M - n_a, wb, bb))
        ys, problems = [], []
        for r0, m, w, b in blocks:
            y = torch.empty((m, w.shape[0]), dtype=torch.float32, device=h.device)
            problems.append(_problem(m, w.shape[0], K, h[r0:], h.stride(0), 1, w, K, 1, y,
                                     w.shape[0], bias=None if b is None else b.contiguous()))
            ys.append(y)
        _launch(h.device, *problems)
        ctx.save_for_backward(h, wa, wb)
        ctx.n_a, ctx.has_bias = n_a, (ba is not None, bb is not None)
        return ys[0], ys[1]

    @staticmethod
    def backward(ctx, ga, gb_):
        h, wa, wb = ctx.saved_tensors
        M, K = h.shape
        dev = h.device
        need = ctx.needs_input_grad
        grads = [None] * 6
        gh = torch.empty((M, K), dtype=torch.float32, device=dev) if need[0] else None
        problems = []
        for k, (r0, m, w, g) in enumerate(((0, ctx.n_a, wa, ga), (ctx.n_a, M - ctx.n_a, wb, gb_))):
            g = g.contiguous()
            N = w.shape[0]
            if need[0]:
                problems.append(_problem(m, K, N, g, N, 1, w, 1, K, gh[r0:], K))
            if need[1 + 2 * k] or need[2 + 2 * k]:
                hb = ctx.has_bias[k]
                gw = torch.empty((N, K), dtype=torch.float32, device=dev)
                gbias = torch.empty((N,), dtype=torch.float32, device=dev) if hb else None
                problems.append(_problem(N, K + (1 if hb else 0), m, g, 1, N, h[r0:], 1,
                                         h.stride(0), gw, K, ones_col=K if hb else -1,
                                         out_col=gbias))
                grads[1 + 2 * k], grads[2 + 2 * k] = gw, gbias
        if problems:
            _launch(dev, *problems)
        grads[0] = gh
        return tuple(grads)


def linear(x, layer, relu=False, alpha=1.0, drop_p=0.0):
    """act(alpha * layer(x)) on the matrix cores, act = ReLU if `relu`; then,
    if drop_p > 0, nn.Dropout(drop_p) in training mode (ReLU layers, alpha 1)."""
    return HipLinear.apply(x, layer.weight, layer.bias, bool(relu), float(alpha), float(drop_p))


def heads(x, a, b, alpha=1.0):
    """(alpha * a(x), alpha * b(x)) for two Linear layers of one input."""
    return HipLinearHeads.apply(x, a.weight, a.bias, b.weight, b.bias, float(alpha))


def row_heads(h, a, b, n_a):
    """(a(h[:n_a]), b(h[n_a:])) for two Linear layers on the row blocks of h."""
    return HipRowHeads.apply(h, a.weight, a.bias, b.weight, b.bias, int(n_a))
