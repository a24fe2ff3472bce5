"""Device-dispatching primitive API used by the explicit engine and the trainers.

CPU tensors run the PyTorch reference (:mod:`hfrep.ops.reference`); GPU tensors run the gfx950
kernels in ``_hfrep_native.so`` (``torch.ops.hfrep``).  There is no silent fallback on GPU: if the
library is missing, :func:`hfrep.ops._native.use_native_for` raises (see its docstring).

Shapes: activations are (..., features) with the feature axis contiguous; Dense/LSTM kernels
are Keras-layout (in, out) fp32 master weights; activations may be fp32 or bf16 (the compute
dtype of the explicit engine); gradients are always fp32.
"""
from __future__ import annotations

import contextlib

import torch

from . import _native
from . import reference as R


def _nat(t: torch.Tensor) -> bool:
    return _native.use_native_for(t)


def _ops():
    return _native.native()


def _2d(x: torch.Tensor) -> torch.Tensor:
    return x.reshape(-1, x.shape[-1])


# ---------------------------------------------------------------------------------------
# weight gradients off the reverse pass's critical path
# ---------------------------------------------------------------------------------------
class _WgradDefer:
    stream = None  # the side stream weight-gradient launches go to (None: inline)
    keep: list = []  # operands of the deferred launches, alive until the join


@contextlib.contextmanager
def wgrad_on(stream):
    """Inside the block every layer's weight-gradient launch (:func:`run_wgrad`) runs on ``stream``,
    after everything issued so far on the current stream, while the current stream goes on with the
    next layer's backward; at the end the current stream waits for ``stream``.  The launches keep
    their order on the one side stream, so every gradient accumulates in the sequential order (bitwise
    the same result).  Their operands stay referenced until the join, so the caching allocator never
    hands their blocks to the current stream while the side stream still reads them.  ``stream`` None:
    a no-op (the launches run inline)."""
    if stream is None or _WgradDefer.stream is not None:
        yield
        return
    cur = torch.cuda.current_stream(stream.device)
    _WgradDefer.stream, _WgradDefer.keep = stream, []
    try:
        yield
    finally:
        _WgradDefer.stream = None
        cur.wait_stream(stream)
        _WgradDefer.keep = []


def run_wgrad(fn, *args, **kw):
    """``fn(*args, **kw)`` (a weight-gradient launch), on the :func:`wgrad_on` stream when one is set."""
    s = _WgradDefer.stream
    if s is None:
        return fn(*args, **kw)
    s.wait_stream(torch.cuda.current_stream(s.device))
    with torch.cuda.stream(s):
        fn(*args, **kw)
    _WgradDefer.keep.append((args, kw))


# ---------------------------------------------------------------------------------------
# dense / GEMM family
# ---------------------------------------------------------------------------------------
# fp32 GEMMs run on native exact-fp32 kernels: K in {32, 36, 64, 100, 128} with 4 < N <= 112 (every Dense
# of the LSTM and MLP zoo at the bench shapes) on the register-resident narrow kernel, any other K % 4 == 0
# up to 320 and any N (the conv critic's im2col GEMMs, K = k C) on the LDS-staged wide kernel
# (csrc/skinny.hip narrowf_kernel / widef_kernel).


def linear(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor | None, act: int,
           out: torch.Tensor | None = None) -> torch.Tensor:
    """act(x @ W + b) on the last axis. Output dtype = x dtype.  ``out``: a contiguous destination
    of the output's shape (e.g. a row slice of a larger buffer); the result is written there."""
    if _nat(x):
        y = _ops().linear(_2d(x.contiguous()), W, b, int(act), out)
        return y.reshape(*x.shape[:-1], W.shape[1])
    y = torch.matmul(x, W.to(x.dtype))
    if b is not None:
        y = y + b.to(x.dtype)
    y = R.apply_act(y, act)
    return y if out is None else out.copy_(y)


# fp32 dZ (.., 400) @ W^T with W (K <= 112, 400): the LSTM layers' input gradient, on the native
# kernels of csrc/lstm_f32.hip (lstmf_dgrad_s4 split / lstmf_dgrad exact)


def linear_dgrad(dz: torch.Tensor, W: torch.Tensor) -> torch.Tensor:
    """dz @ W^T (input gradient)."""
    if (dz.dtype == torch.float32 and W.dtype == torch.float32 and dz.shape[-1] == 400
            and W.shape[0] <= 112 and _nat(dz)):
        return _ops().lstmf_dgrad(_2d(dz.contiguous()), W.contiguous()).reshape(*dz.shape[:-1], W.shape[0])
    if _nat(dz):
        return _ops().linear_dgrad(_2d(dz.contiguous()), W).reshape(*dz.shape[:-1], W.shape[0])
    return torch.matmul(dz, W.t().to(dz.dtype))


def linear_wgrad_(x: torch.Tensor, dz: torch.Tensor, gW: torch.Tensor, gb: torch.Tensor | None,
                  shift_T: int = 0) -> None:
    """gW += x^T dz (summed over all leading axes); gb += sum(dz).

    ``shift_T > 0``: x is a (B, T, K) sequence and the product uses x_{t-1} (zero at t=0) — the
    LSTM recurrent-kernel gradient sum_t h_{t-1}^T dz_t — without materialising the shift.
    """
    if _nat(dz):
        _ops().linear_wgrad_(_2d(x.contiguous()), _2d(dz.contiguous()), gW, gb, int(shift_T))
        return
    if shift_T:
        x = R.shift_prev(x)
    x2, d2 = _2d(x).to(gW.dtype), _2d(dz).to(gW.dtype)
    gW.add_(x2.t() @ d2)
    if gb is not None:
        gb.add_(d2.sum(0))


# ---------------------------------------------------------------------------------------
# elementwise activations
# ---------------------------------------------------------------------------------------
def act_forward(x: torch.Tensor, act: int) -> torch.Tensor:
    if _nat(x):
        return _ops().act_fwd(x.contiguous(), int(act))
    return R.apply_act(x, act)


def act_backward(dy: torch.Tensor, y: torch.Tensor, act: int) -> torch.Tensor:
    """dy * f'(x) written through y = f(x)."""
    if act == 0:
        return dy
    if _nat(dy):
        return _ops().act_bwd(dy.contiguous(), y.contiguous(), int(act))
    return dy * R.act_dy(y, act)


def act_tangent_backward(dy, dyd, y, zd, act: int):
    """Adjoint of z for y = f(z), ydot = f'(z) zdot:  dy f'(z) + dyd f''(z) zdot."""
    first = act_backward(dy, y, act) if dy is not None else None
    if act in (0, 3, 4):  # piecewise linear: f'' = 0
        return first if first is not None else torch.zeros_like(dyd)
    if _nat(dyd):
        sec = _ops().act_tangent_bwd(dyd.contiguous(), y.contiguous(), zd.contiguous(), int(act))
    else:
        sec = dyd * R.act_d2y(y, act) * zd
    return sec if first is None else first + sec


# ---------------------------------------------------------------------------------------
# LSTM recurrences (persistent kernels on GPU)
# ---------------------------------------------------------------------------------------
def lstm_seq_fwd(zx, U, act: int, save: bool):
    if _nat(zx):
        hs, gates, cs = _ops().lstm_fwd(zx.contiguous(), U, int(act), bool(save))
        return hs, (gates if save else None), (cs if save else None)
    return R.lstm_seq_fwd(zx, U.to(zx.dtype), act, save)


def lstm_seq_bwd(dh_seq, gates, cs, U, act: int):
    if _nat(dh_seq):
        return _ops().lstm_bwd(dh_seq.contiguous(), gates, cs, U, int(act))
    return R.lstm_seq_bwd(dh_seq, gates, cs, U.to(dh_seq.dtype), act)


def lstm_seq_tfwd(dzx, gates, cs, U, act: int):
    if _nat(dzx):
        return tuple(_ops().lstm_tfwd(dzx.contiguous(), gates, cs, U, int(act)))
    return R.lstm_seq_tfwd(dzx, gates, cs, U.to(dzx.dtype), act)


def lstm_seq_tbwd(dh_seq, dhd_seq, gates, cs, zds, cds, U, act: int):
    if _nat(dhd_seq):
        return tuple(_ops().lstm_tbwd(dh_seq.contiguous(), dhd_seq.contiguous(), gates, cs, zds, cds, U, int(act)))
    return R.lstm_seq_tbwd(dh_seq, dhd_seq, gates, cs, zds, cds, U.to(dhd_seq.dtype), act)


def shift_prev(h_seq: torch.Tensor) -> torch.Tensor:
    """h_{t-1} for every t (zeros at t=0).  (B, T, H)"""
    if _nat(h_seq):
        return _ops().shift_prev(h_seq.contiguous())
    return R.shift_prev(h_seq)


# ---------------------------------------------------------------------------------------
# LayerNorm
# ---------------------------------------------------------------------------------------
def layer_norm_fwd(x, gamma, beta, eps: float, save: bool = True):
    """(y, xhat, rstd); with save=False the native kernel skips xhat / rstd (returned empty)."""
    if _nat(x):
        y, xhat, rstd = _ops().layernorm_fwd(x.contiguous(), gamma, beta, float(eps), bool(save))
        return y, xhat, rstd
    return R.layer_norm_fwd(x, gamma.to(x.dtype), beta.to(x.dtype), eps)


def lrelu_layer_norm_fwd(x, gamma, beta, eps: float, alpha: float, save: bool = True):
    """LayerNorm(LeakyReLU(x)) as one kernel (the generator's LReLU -> LN pairs); the activation
    output is rounded to x.dtype exactly as the separate activation kernel stores it."""
    if _nat(x):
        return _ops().layernorm_fwd(x.contiguous(), gamma, beta, float(eps), bool(save), float(alpha))
    return layer_norm_fwd(R.leaky_relu(x, alpha), gamma, beta, eps, save)


def layer_norm_bwd_(dy, xhat, rstd, gamma, ggamma, gbeta):
    """Returns dx; accumulates dgamma/dbeta into the gradient views."""
    if _nat(dy):
        return _ops().layernorm_bwd_(dy.contiguous(), xhat, rstd, gamma, ggamma, gbeta)
    dx, dg, db = R.layer_norm_bwd(dy, xhat, rstd, gamma.to(dy.dtype))
    if ggamma is not None:
        ggamma.add_(dg.to(ggamma.dtype))
        gbeta.add_(db.to(gbeta.dtype))
    return dx


def layer_norm_tfwd(xd, xhat, rstd, gamma):
    """LayerNorm JVP from the saved forward (xhat, rstd): the GP critic's tangent pass."""
    if _nat(xd):
        return _ops().layernorm_tfwd(xd.contiguous(), xhat, rstd, gamma)
    return R.layer_norm_tfwd(xd, xhat, rstd, gamma.to(xd.dtype))


def layer_norm_tbwd_(dy, dyd, xd, xhat, rstd, gamma, ggamma, gbeta, need_dx: bool):
    """Reverse of the LN forward + JVP; accumulates dgamma / dbeta, returns (dx, dxd) or (None, None)."""
    if _nat(dyd):
        dx, dxd = _ops().layernorm_tbwd_(dy.contiguous() if dy is not None else None, dyd.contiguous(), xd, xhat,
                                         rstd, gamma, ggamma, gbeta, bool(need_dx))
        return (dx, dxd) if need_dx else (None, None)
    dx, dxd, dg, db = R.layer_norm_tbwd(dy, dyd, xd, xhat, rstd, gamma.to(dyd.dtype))
    ggamma.add_(dg.to(ggamma.dtype))
    gbeta.add_(db.to(gbeta.dtype))
    return (dx, dxd) if need_dx else (None, None)


# ---------------------------------------------------------------------------------------
# temporal conv helpers (im2col on the feature axis)
# ---------------------------------------------------------------------------------------
def im2col_causal(x: torch.Tensor, k: int, dil: int) -> torch.Tensor:
    """(B, T, C) -> (B, T, k*C) with column block j holding x[t - (k-1-j)*dil] (zero padded)."""
    if _nat(x):
        return _ops().im2col_causal(x.contiguous(), int(k), int(dil))
    B, T, C = x.shape
    pad = (k - 1) * dil
    xp = torch.nn.functional.pad(x, (0, 0, pad, 0))
    cols = [xp[:, j * dil:j * dil + T] for j in range(k)]
    return torch.cat(cols, dim=2)


def col2im_causal(dcols: torch.Tensor, k: int, dil: int, C: int) -> torch.Tensor:
    """Adjoint of :func:`im2col_causal` (a gather on the GPU: no atomics)."""
    if _nat(dcols):
        return _ops().col2im_causal(dcols.contiguous(), int(k), int(dil), int(C))
    B, T, _ = dcols.shape
    pad = (k - 1) * dil
    dxp = dcols.new_zeros(B, T + pad, C)
    for j in range(k):
        dxp[:, j * dil:j * dil + T] += dcols[:, :, j * C:(j + 1) * C]
    return dxp[:, pad:]


# ---------------------------------------------------------------------------------------
# WGAN-GP helpers
# ---------------------------------------------------------------------------------------
def gan_loss(p: torch.Tensor, split: int, la: float, lb: float, kind: int):
    """(per-segment losses [2], dL/dp) of a Wasserstein (kind 0) or BCE (kind 1) loss over the
    scores p split into two labelled segments (one launch for the W terms on [real; fake]).
    bf16 / fp32 on the GPU: one native pass (csrc/misc.hip gan_loss_kernel); else the reference."""
    if _nat(p) and p.dtype in (torch.bfloat16, torch.float32):
        return _ops().gan_loss(p.contiguous(), int(split), float(la), float(lb), int(kind))
    return R.gan_loss(p, int(split), float(la), float(lb), int(kind),
                      acc=torch.float64 if p.dtype == torch.float64 else torch.float32)


def head_cs_ok(x: torch.Tensor, W: torch.Tensor) -> bool:
    """Whether a linear Dense(1) head on x can run as the fused forward + known-gradient column sum."""
    return (x.dim() == 2 and W.dim() == 2 and W.shape[1] == 1 and x.dtype in (torch.bfloat16, torch.float32)
            and _nat(x) and not _native.fallback_allowed() and bool(_ops().linear_head_cs_supported(int(W.shape[0]))))


def loss_grad_value(label: float, n: int, dtype) -> float:
    """The per-row gradient gan_loss (kind 0) writes for a segment of n rows with this label: label * (1/n)
    in fp32, stored in the score dtype."""
    inv = torch.tensor(1.0, dtype=torch.float32) / torch.tensor(float(n), dtype=torch.float32)
    return float((torch.tensor(float(label), dtype=torch.float32) * inv).to(dtype).item())


def linear_head_cs(x, W, b, split: int, wa: float, wb: float, gW, gb):
    """y = x W + b for a linear Dense(1) head, and in the same pass gW += sum_r ds_r x_r, gb += sum_r ds_r
    for the known per-row loss gradient ds_r = wa (r < split) / wb (csrc/skinny.hip skinny_fwd_cs_kernel)."""
    return _ops().linear_head_cs(x.contiguous(), W, b, int(split), float(wa), float(wb), gW, gb)


def gp_coef(g: torch.Tensor, weight: float):
    """(penalty, v): penalty = mean((1-||g_b||)^2); v = d(weight*penalty)/dg."""
    if _nat(g):
        pen, v = _ops().gp_coef(g.contiguous(), float(weight))
        return pen, v
    return R.gp_coef(g, weight)


def gp_coef_pack(g: torch.Tensor, weight: float, w: torch.Tensor):
    """(pack, v): gp_coef plus the critic step's loss record pack = [w0 + w1 + weight*pen, w0, w1, pen]
    (fp32) from the step's two W terms ``w`` -- one native launch pair on the GPU, no torch glue."""
    if _nat(g) and w.dtype == torch.float32:
        return _ops().gp_coef_pack(g.contiguous(), float(weight), w.contiguous())
    pen, v = gp_coef(g, weight)
    w = w.to(torch.float64 if g.dtype == torch.float64 else torch.float32)
    pen = pen.to(w.dtype)
    return torch.stack([w[0] + w[1] + weight * pen, w[0], w[1], pen]), v


def gp_pack(pen: torch.Tensor, weight: float, w: torch.Tensor) -> torch.Tensor:
    """gp_coef_pack's loss record [w0 + w1 + weight*pen, w0, w1, pen] from gp_coef's penalty (the same
    arithmetic as the fused launch: the concurrent small-batch critic step forms it after its join)."""
    if _nat(pen) and pen.dtype == torch.float32 and w.dtype == torch.float32:
        return _ops().gp_pack(pen.reshape(1).contiguous(), float(weight), w.contiguous())
    w = w.to(pen.dtype)
    return torch.stack([w[0] + w[1] + weight * pen.reshape(()), w[0], w[1], pen.reshape(())])


def interpolate(real: torch.Tensor, fake: torch.Tensor, alpha: torch.Tensor) -> torch.Tensor:
    """alpha (B,) per-sample: alpha*real + (1-alpha)*fake (GAN/MTSS_WGAN_GP.py:197-199)."""
    if _nat(real):
        return _ops().interpolate(real.contiguous(), fake.contiguous(), alpha.contiguous())
    a = alpha.reshape(-1, *([1] * (real.dim() - 1))).to(real.dtype)
    return a * real + (1 - a) * fake


# ---------------------------------------------------------------------------------------
# LSTM layer-level API (input projection included).  The tape is opaque: a (gates, cells) tuple
# on the reference / fp32 path, or one blocked bf16 tensor on the fused v2 kernels (csrc/lstm2.hip).
# ---------------------------------------------------------------------------------------
def _use_lstm2(x: torch.Tensor, U: torch.Tensor) -> bool:
    return (x.dtype == torch.bfloat16 and U.shape[0] == 100 and x.shape[-1] <= 128 and _nat(x)
            and not _native.fallback_allowed())


def _use_lstmf(x: torch.Tensor, U: torch.Tensor, act: int) -> bool:
    """fp32 fused-projection kernels (csrc/lstm_f32.hip): H = 100, K in {32, 35, 36, 100}."""
    return (x.dtype == torch.float32 and _nat(x) and not _native.fallback_allowed()
            and bool(_ops().lstmf_supported(int(U.shape[0]), int(x.shape[-1]), int(act))))


class FTape:
    """fp32 tape of the fused fp32 kernels (csrc/lstm_f32.hip): one lane-native blocked tensor
    (per 32-row block and step: 4 waves x 14 slots x 64 lanes x {4 gate values, 1 cell value}), plus
    the (B, T) it was written for.  Primal tapes hold gate activations and c_t, tangent tapes the
    gate pre-activation tangents and cdot_t."""

    __slots__ = ("t", "B", "T")

    def __init__(self, t: torch.Tensor, B: int, T: int):
        self.t, self.B, self.T = t, int(B), int(T)


def lstm_layer_fwd(x, W, b, U, act: int, save: bool):
    """h_seq and a tape for act(x W + b ...) recurrences; x (B, T, K)."""
    if _use_lstm2(x, U):
        hs, tape = _ops().lstm2_fwd(x.contiguous(), W, b, U, int(act), bool(save))
        return hs, (tape if save else None)
    if _use_lstmf(x, U, act):
        hs, tape = _ops().lstmf_fwd(x.contiguous(), W, b, U, int(act), bool(save))
        return hs, (FTape(tape, x.shape[0], x.shape[1]) if save else None)
    zx = linear(x, W, b, 0)
    hs, gates, cs = lstm_seq_fwd(zx, U, act, save)
    return hs, ((gates, cs) if save else None)


class OuterAdjoint:
    """Lazy input adjoint of a linear Dense(1) head: dX[b, j] = d[b, 0] * w[j, 0], viewed with
    ``shape`` (after Flatten: (B, T, H)).  The LSTM reverse kernels generate it inside the kernel (bf16:
    csrc/lstm2.hip TileSrc; fp32: the HEAD instantiations of lstmf_bwds / lstmf_tbwdp), so the
    (B, T*H) head adjoint never exists in HBM; every other consumer calls :meth:`materialize` (the
    skinny dgrad kernel, same rounding)."""

    def __init__(self, d: torch.Tensor, w: torch.Tensor, shape=None):
        self.d, self.w = d, w
        self.shape = tuple(shape) if shape is not None else (d.shape[0], w.shape[0])

    def reshape(self, *shape):
        shape = tuple(shape[0]) if len(shape) == 1 and not isinstance(shape[0], int) else tuple(shape)
        return OuterAdjoint(self.d, self.w, shape)

    def materialize(self) -> torch.Tensor:
        return linear_dgrad(self.d, self.w).reshape(self.shape)


def outer_adjoint_ok(dz: torch.Tensor) -> bool:
    """Whether a Dense(1) head may hand its input adjoint on lazily (bf16 and fp32 on the native path:
    the LSTM reverse kernels of both precisions generate it; the exact-fp32 BPTT materialises it in the
    binding)."""
    return dz.dtype in (torch.bfloat16, torch.float32) and _nat(dz) and not _native.fallback_allowed()


def _mat(a):
    return a.materialize() if isinstance(a, OuterAdjoint) else a


def lstm_layer_bwd(dH, tape, U, act: int, W=None, need_dz: bool = True):
    """dZ = dL/d(x W + b + h U) for every step; with ``W`` also the input gradient dX = dZ W^T,
    returned as ``(dZ, dX)`` (the v2 kernel produces it in the same launch, csrc/lstm2.hip).
    ``need_dz=False`` (only dX wanted, e.g. the gradient penalty's dD/dx) lets the v2 kernel skip
    writing dZ to HBM; the returned dZ is then None."""
    if isinstance(tape, FTape):
        if isinstance(dH, OuterAdjoint) and dH.d.dtype == torch.float32:  # head adjoint generated in-kernel
            dZ = _ops().lstmf_bwd(None, tape.t, U, int(act), tape.B, tape.T, dH.d.contiguous(),
                                  dH.w.reshape(-1).contiguous())
        else:
            dH = _mat(dH)
            dZ = _ops().lstmf_bwd(None if dH is None else dH.contiguous(), tape.t, U, int(act), tape.B, tape.T)
        return dZ if W is None else (dZ, linear_dgrad(dZ, W))
    if isinstance(tape, torch.Tensor):
        nd = bool(need_dz or W is None)
        if isinstance(dH, OuterAdjoint):  # head adjoint generated in-kernel
            dZ, dX = _ops().lstm2_bwd(None, tape, U, int(act), W, nd, dH.d.contiguous(), dH.w.reshape(-1).contiguous())
        else:
            dZ, dX = _ops().lstm2_bwd(dH.contiguous(), tape, U, int(act), W, nd)
        if W is not None and not need_dz:
            dZ = None
        return dZ if W is None else (dZ, dX)
    dH = _mat(dH)
    gates, cs = tape
    dZ = lstm_seq_bwd(dH, gates, cs, U, act)
    return dZ if W is None else (dZ, linear_dgrad(dZ, W))


def lstm_layer_tfwd(xd, W, tape, U, act: int):
    if isinstance(tape, FTape):
        hds, ttape = _ops().lstmf_tfwd(xd.contiguous(), W, U, tape.t, int(act))
        return hds, FTape(ttape, tape.B, tape.T)
    if isinstance(tape, torch.Tensor):
        hds, ttape = _ops().lstm2_tfwd(xd.contiguous(), W, U, tape, int(act))
        return hds, ttape
    gates, cs = tape
    dzx = linear(xd, W, None, 0)
    hds, zds, cds = lstm_seq_tfwd(dzx, gates, cs, U, act)
    return hds, (zds, cds)


def lstm_wgrad_(x, hs, dZ, gW, gU, gb, xd=None, hds=None, dZd=None, impl: int = 0) -> None:
    """All weight gradients of one LSTM layer: gW += X^T dZ (+ Xd^T dZd), gU += H_{t-1}^T dZ (+ ...),
    gb += sum(dZ).  bf16 GPU: ONE fused launch (csrc/wgrad3.hip LDS-DMA streaming kernel where the
    shape is supported, csrc/gemm2.hip otherwise; ``impl=2`` forces the latter); fp32 GPU at the
    model widths (K in {32, 35, 36, 100}; 35-wide rows are read in place): ONE fused launch of
    csrc/lstm_f32.hip -- the fp32-accurate three-term bf16 split (every fp32 operand h + m + l, six
    products on the bf16 matrix pipe): lstmf_wgrad_split_kernel for K <= 36 (``impl=2``),
    lstmf_wgrad_q4_kernel for K = 100 (``impl=3``); the exact-fp32 MFMA kernel lstmf_wgrad_kernel
    under HFREP_FP32_EXACT=1 (``impl=1``); otherwise per-product calls."""
    f32 = (dZ.dtype == torch.float32 and x.shape[-1] in (32, 35, 36, 100) and hs.shape[-1] == 100
           and dZ.shape[-1] == 400)
    if (dZ.dtype == torch.bfloat16 or f32) and _nat(dZ):
        _ops().lstm_wgrad_(x.contiguous(), hs.contiguous(), dZ.contiguous(), gW, gU, gb,
                           None if xd is None else xd.contiguous(), None if hds is None else hds.contiguous(),
                           None if dZd is None else dZd.contiguous(), int(impl))
        return
    T = hs.shape[1]
    linear_wgrad_(x, dZ, gW, gb)
    linear_wgrad_(hs, dZ, gU, None, shift_T=T)
    if xd is not None:
        linear_wgrad_(xd, dZd, gW, None)
        linear_wgrad_(hds, dZd, gU, None, shift_T=T)


def lstm_layer_tbwd(dH, dHd, tape, ttape, U, act: int, W=None):
    """(dZ, dZd) of the reverse-over-tangent pass; with ``W`` also (dX, dXd) = (dZ W^T, dZd W^T)."""
    if isinstance(tape, FTape):
        heads = [a for a in (dH, dHd) if isinstance(a, OuterAdjoint)]
        if heads and all(a is None or (isinstance(a, OuterAdjoint) and a.w is heads[0].w and a.d.dtype == torch.float32)
                         for a in (dH, dHd)):  # head adjoints generated in-kernel
            dZ, dZd = _ops().lstmf_tbwd(None, None, tape.t, ttape.t, U, int(act), tape.B, tape.T,
                                        None if dH is None else dH.d.contiguous(),
                                        None if dHd is None else dHd.d.contiguous(), heads[0].w.reshape(-1).contiguous())
        else:
            dH, dHd = _mat(dH), _mat(dHd)
            dZ, dZd = _ops().lstmf_tbwd(None if dH is None else dH.contiguous(), None if dHd is None else dHd.contiguous(),
                                        tape.t, ttape.t, U, int(act), tape.B, tape.T)
        return (dZ, dZd) if W is None else (dZ, dZd, linear_dgrad(dZ, W), linear_dgrad(dZd, W))
    if isinstance(tape, torch.Tensor):
        heads = [a for a in (dH, dHd) if isinstance(a, OuterAdjoint)]
        # the in-kernel generated head adjoint, also with the fused input gradient (the DX + GEN
        # tangent reverse drifted run to run in r01-r02: a cross-opcode MFMA SrcC hazard, fixed in r03,
        # profiles/r03_race/README.md)
        if heads and all(a is None or (isinstance(a, OuterAdjoint) and a.w is heads[0].w)
                                       for a in (dH, dHd)):
            w = heads[0].w.reshape(-1).contiguous()
            dZ, dZd, dX, dXd = _ops().lstm2_tbwd(None, None, tape, ttape, U, int(act), W,
                                                 None if dH is None else dH.d.contiguous(),
                                                 None if dHd is None else dHd.d.contiguous(), w)
        else:
            dH, dHd = _mat(dH), _mat(dHd)
            dZ, dZd, dX, dXd = _ops().lstm2_tbwd(None if dH is None else dH.contiguous(), dHd.contiguous(), tape,
                                                 ttape, U, int(act), W)
        return (dZ, dZd) if W is None else (dZ, dZd, dX, dXd)
    dH, dHd = _mat(dH), _mat(dHd)
    gates, cs = tape
    zds, cds = ttape
    if dH is None:
        dH = torch.zeros_like(dHd)
    dZ, dZd = lstm_seq_tbwd(dH, dHd, gates, cs, zds, cds, U, act)
    return (dZ, dZd) if W is None else (dZ, dZd, linear_dgrad(dZ, W), linear_dgrad(dZd, W))
