"""Keras-semantics layers with flat parameter storage and an explicit differentiation engine.

Every model keeps ALL of its parameters in one contiguous fp32 buffer (``Sequential.flat``) and
all gradients in one matching buffer (``flat.grad``).  That single buffer is what the fused
optimizer kernels update in one launch and what data-parallel training all-reduces as one
bucket — the MI355X-first replacement for Keras' per-variable ``apply_gradients``.

Each layer offers two execution styles:

* ``forward(x)`` — composed, autograd-differentiable ops (``ops.reference``); the CPU oracle.
* the **explicit engine** — ``efwd`` (forward, saving what backward needs), ``ebwd`` (reverse),
  ``etfwd`` (tangent/JVP at the saved point) and ``etbwd`` (reverse of the tangent system).  The
  trainers are written against this engine; on GPU tensors every primitive dispatches to the
  hand-written gfx950 kernels through :mod:`hfrep.ops.functional`.  The WGAN-GP critic update
  (a second-order quantity, GAN/MTSS_WGAN_GP.py:205-216) is computed as reverse-over-tangent:
  ``d/dtheta <v, dD/dx>`` = ``etbwd`` of the tangent network seeded with ``v``.

Keras conventions: Dense kernel (in, out) on the last axis; LSTM gate order
[i, f, c, o], recurrent sigmoid, unit forget bias, orthogonal recurrent init; LayerNorm eps
1e-3; LeakyReLU 0.2; Flatten row-major.  Parameter names follow the Keras HDF5 layout
(``lstm_1/lstm_cell_1/kernel:0``) so checkpoints can be exchanged by name.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from ..ops import functional as Fn
from ..ops import reference as R


# ----------------------------------------------------------------------------------------
# Keras initialisers (deterministic, generated on CPU from a torch.Generator)
# ----------------------------------------------------------------------------------------
def glorot_uniform(shape, gen, fan_in=None, fan_out=None):
    if fan_in is None:
        fan_in, fan_out = shape[0], shape[-1]
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    return (torch.rand(shape, generator=gen, dtype=torch.float64) * 2 - 1) * lim


def orthogonal(shape, gen, gain=1.0):
    rows = int(np.prod(shape[:-1]))
    cols = shape[-1]
    a = torch.randn(max(rows, cols), min(rows, cols), generator=gen, dtype=torch.float64)
    q, r = torch.linalg.qr(a)
    q = q * torch.sign(torch.diagonal(r))
    if rows < cols:
        q = q.t()
    return (gain * q).reshape(shape)


@dataclass
class ParamSpec:
    name: str          # short name: kernel / recurrent_kernel / bias / gamma / beta
    shape: tuple
    init: str          # glorot / orthogonal / zeros / ones / lstm_bias
    keras: str = ""    # full Keras weight name, filled by the model
    offset: int = 0


class Layer:
    """Base class. Subclasses define ``param_specs``, ``output_shape`` and the op methods."""

    kind = "layer"
    index = 0  # per-kind counter for Keras-style names

    def __init__(self):
        self.model = None
        self.specs: list[ParamSpec] = []
        self.name = ""

    # -- construction ------------------------------------------------------------------------
    def build(self, in_shape):  # returns out_shape
        raise NotImplementedError

    def p(self, name):  # parameter view
        return self.model.view(self, name)

    def g(self, name):  # gradient view
        return self.model.gview(self, name)

    # -- autograd path ----------------------------------------------------------------------
    def forward(self, x):
        raise NotImplementedError

    # -- explicit engine ----------------------------------------------------------------------
    def efwd(self, x, save: bool):
        raise NotImplementedError

    def ebwd(self, ctx, dy, need_dx: bool, wgrad: bool = True):
        raise NotImplementedError

    # tangent (forward-mode) and its reverse at the taped point: the GP's reverse-over-tangent pass
    # (docs/ARCHITECTURE.md §1); every concrete layer implements both with native primitives
    def etfwd(self, ctx, xd):
        raise NotImplementedError

    def etbwd(self, ctx, tctx, dy, dyd, need_dx: bool):
        raise NotImplementedError

    def w(self, name):
        """Parameter as seen by ``forward`` (the autograd reference path)."""
        return self.p(name)


class Dense(Layer):
    kind = "dense"

    def __init__(self, units: int, activation=None, use_bias: bool = True):
        super().__init__()
        self.units, self.act, self.use_bias = units, activation, use_bias
        self.act_code = R.act_code(activation)

    def build(self, in_shape):
        fin = in_shape[-1]
        self.specs = [ParamSpec("kernel", (fin, self.units), "glorot")]
        if self.use_bias:
            self.specs.append(ParamSpec("bias", (self.units,), "zeros"))
        return tuple(in_shape[:-1]) + (self.units,)

    def forward(self, x):
        return R.dense(x, self.w("kernel"), self.w("bias") if self.use_bias else None, self.act)

    def efwd(self, x, save, out=None, compute=True, wgrad_rows=None):
        """``compute=False`` (linear head whose value the caller never reads, e.g. D(x_hat) of the
        gradient penalty: only its input adjoint is used): no kernel runs and ``y`` is an uninitialised
        placeholder of the output's shape -- the linear backward / tangent passes never read it."""
        if not compute:
            assert self.act_code == 0, "only a linear Dense output can be left uncomputed"
            y = torch.empty(tuple(x.shape[:-1]) + (self.units,), dtype=x.dtype, device=x.device)
            return y, ({"x": x, "y": y} if save else None)
        b = self.p("bias") if self.use_bias else None
        if (wgrad_rows is not None and save and out is None and self.units == 1 and self.act_code == 0
                and Fn.head_cs_ok(x, self.p("kernel"))):
            # the loss gradient of every row is known before the forward (Wasserstein segments): the
            # head's weight gradient is accumulated in the same pass over x and ebwd skips it
            split, wa, wb = wgrad_rows
            y = Fn.linear_head_cs(x, self.p("kernel"), b, split, wa, wb, self.g("kernel"),
                                  self.g("bias") if self.use_bias else None)
            return y, {"x": x, "y": y, "wgrad_done": True}
        y = Fn.linear(x, self.p("kernel"), b, self.act_code, out=out)
        return y, ({"x": x, "y": y} if save else None)

    def _dgrad(self, dz):
        # a Dense(1) head hands its input adjoint on as a lazy outer product (OuterAdjoint): the
        # LSTM reverse kernels generate it in-kernel, anything else materialises it
        if self.units == 1 and dz.dim() == 2 and Fn.outer_adjoint_ok(dz):  # (B, 1): a Flatten head
            return Fn.OuterAdjoint(dz, self.p("kernel"))
        return Fn.linear_dgrad(dz, self.p("kernel"))

    def ebwd(self, ctx, dy, need_dx, wgrad=True):
        dz = Fn.act_backward(dy, ctx["y"], self.act_code)
        if wgrad and not ctx.get("wgrad_done"):
            Fn.run_wgrad(Fn.linear_wgrad_, ctx["x"], dz, self.g("kernel"), self.g("bias") if self.use_bias else None)
        return self._dgrad(dz) if need_dx else None

    def etfwd(self, ctx, xd, compute=True):
        if not compute:  # linear head, tangent value unused (see efwd): shape-only placeholder
            assert self.act_code == 0, "only a linear Dense output can be left uncomputed"
            zd = torch.empty(tuple(xd.shape[:-1]) + (self.units,), dtype=xd.dtype, device=xd.device)
            return zd, {"xd": xd, "zd": zd}
        zd = Fn.linear(xd, self.p("kernel"), None, 0)
        yd = Fn.act_backward(zd, ctx["y"], self.act_code)  # act'(z) * zdot
        return yd, {"xd": xd, "zd": zd}

    def etbwd(self, ctx, tctx, dy, dyd, need_dx):
        dzd = Fn.act_backward(dyd, ctx["y"], self.act_code)
        # dy is None (no primal seed) with a piecewise-linear activation: dz == 0 (f'' = 0), so its weight
        # gradient term vanishes and dx is the zero adjoint (None) -- nothing is materialised
        zero_dz = dy is None and self.act_code in (0, 3, 4)
        if not zero_dz:
            dz = Fn.act_tangent_backward(dy, dyd, ctx["y"], tctx["zd"], self.act_code)
            Fn.run_wgrad(Fn.linear_wgrad_, ctx["x"], dz, self.g("kernel"), self.g("bias") if self.use_bias else None)
        Fn.run_wgrad(Fn.linear_wgrad_, tctx["xd"], dzd, self.g("kernel"), None)
        if not need_dx:
            return None, None
        return (None if zero_dz else self._dgrad(dz)), self._dgrad(dzd)


class LSTM(Layer):
    kind = "lstm"
    accepts_outer = True  # Fn.lstm_layer_bwd / _tbwd consume OuterAdjoint seeds

    def __init__(self, units: int, activation="tanh", return_sequences: bool = True):
        super().__init__()
        assert return_sequences, "the reference uses return_sequences=True everywhere"
        self.units, self.act = units, activation
        self.act_code = R.act_code(activation)

    def build(self, in_shape):
        fin = in_shape[-1]
        H = self.units
        self.specs = [
            ParamSpec("kernel", (fin, 4 * H), "glorot"),
            ParamSpec("recurrent_kernel", (H, 4 * H), "orthogonal"),
            ParamSpec("bias", (4 * H,), "lstm_bias"),
        ]
        return tuple(in_shape[:-1]) + (H,)

    def forward(self, x):
        return R.lstm(x, self.w("kernel"), self.w("recurrent_kernel"), self.w("bias"), act=self.act)

    def efwd(self, x, save):
        hs, tape = Fn.lstm_layer_fwd(x, self.p("kernel"), self.p("bias"), self.p("recurrent_kernel"), self.act_code,
                                     save)
        return hs, ({"x": x, "hs": hs, "tape": tape} if save else None)

    def ebwd(self, ctx, dy, need_dx, wgrad=True):
        U = self.p("recurrent_kernel")
        dx = None
        if need_dx:  # dX = dZ W^T comes out of the BPTT launch itself; dZ is only kept for wgrad
            dZ, dx = Fn.lstm_layer_bwd(dy, ctx["tape"], U, self.act_code, W=self.p("kernel"), need_dz=wgrad)
        else:
            dZ = Fn.lstm_layer_bwd(dy, ctx["tape"], U, self.act_code)
        if wgrad:
            Fn.run_wgrad(Fn.lstm_wgrad_, ctx["x"], ctx["hs"], dZ, self.g("kernel"), self.g("recurrent_kernel"), self.g("bias"))
        return dx

    def etfwd(self, ctx, xd):
        hds, ttape = Fn.lstm_layer_tfwd(xd, self.p("kernel"), ctx["tape"], self.p("recurrent_kernel"), self.act_code)
        return hds, {"xd": xd, "hds": hds, "ttape": ttape}

    def etbwd(self, ctx, tctx, dy, dyd, need_dx):
        U = self.p("recurrent_kernel")
        dx = dxd = None
        if need_dx:
            dZ, dZd, dx, dxd = Fn.lstm_layer_tbwd(dy, dyd, ctx["tape"], tctx["ttape"], U, self.act_code,
                                                  W=self.p("kernel"))
        else:
            dZ, dZd = Fn.lstm_layer_tbwd(dy, dyd, ctx["tape"], tctx["ttape"], U, self.act_code)
        Fn.run_wgrad(Fn.lstm_wgrad_, ctx["x"], ctx["hs"], dZ, self.g("kernel"), self.g("recurrent_kernel"), self.g("bias"),
                       tctx["xd"], tctx["hds"], dZd)
        return dx, dxd


class LayerNormalization(Layer):
    kind = "layer_normalization"

    def __init__(self, epsilon: float = R.LN_EPS):
        super().__init__()
        self.eps = epsilon

    def build(self, in_shape):
        d = in_shape[-1]
        self.specs = [ParamSpec("gamma", (d,), "ones"), ParamSpec("beta", (d,), "zeros")]
        return tuple(in_shape)

    def forward(self, x):
        return R.layer_norm(x, self.w("gamma"), self.w("beta"), self.eps)

    def efwd(self, x, save):
        y, xhat, rstd = Fn.layer_norm_fwd(x, self.p("gamma"), self.p("beta"), self.eps, save=save)
        return y, ({"x": x, "xhat": xhat, "rstd": rstd} if save else None)

    def ebwd(self, ctx, dy, need_dx, wgrad=True):
        gg, gb = (self.g("gamma"), self.g("beta")) if wgrad else (None, None)
        dx = Fn.layer_norm_bwd_(dy, ctx["xhat"], ctx["rstd"], self.p("gamma"), gg, gb)
        return dx if need_dx else None

    # tangent pass of a GP critic with LayerNorm (lstm_critic_clip + wgan_gp): closed-form JVP and
    # reverse kernels on the saved xhat / rstd (works after a fused LReLU -> LN forward too, whose
    # tape holds xhat / rstd but not the LN input)
    def etfwd(self, ctx, xd):
        return Fn.layer_norm_tfwd(xd, ctx["xhat"], ctx["rstd"], self.p("gamma")), {"xd": xd}

    def etbwd(self, ctx, tctx, dy, dyd, need_dx):
        return Fn.layer_norm_tbwd_(dy, dyd, tctx["xd"], ctx["xhat"], ctx["rstd"], self.p("gamma"), self.g("gamma"),
                                   self.g("beta"), need_dx)


class LeakyReLU(Layer):
    kind = "leaky_re_lu"

    def __init__(self, alpha: float = R.LRELU_ALPHA):
        super().__init__()
        self.alpha = alpha

    def build(self, in_shape):
        return tuple(in_shape)

    def forward(self, x):
        return R.leaky_relu(x, self.alpha)

    def efwd(self, x, save):
        y = Fn.act_forward(x, 3)
        return y, ({"y": y} if save else None)

    def ebwd(self, ctx, dy, need_dx, wgrad=True):
        return Fn.act_backward(dy, ctx["y"], 3) if need_dx else None

    def etfwd(self, ctx, xd):
        return Fn.act_backward(xd, ctx["y"], 3), {}

    def etbwd(self, ctx, tctx, dy, dyd, need_dx):
        if not need_dx:
            return None, None
        dx = Fn.act_backward(dy, ctx["y"], 3) if dy is not None else None
        return dx, Fn.act_backward(dyd, ctx["y"], 3)


class Flatten(Layer):
    kind = "flatten"
    accepts_outer = True  # reshape of a lazy OuterAdjoint stays lazy

    def build(self, in_shape):
        self.in_shape = tuple(in_shape)
        return (int(np.prod(in_shape)),)

    def forward(self, x):
        return x.reshape(x.shape[0], -1)

    def efwd(self, x, save):
        return x.reshape(x.shape[0], -1), ({"shape": x.shape} if save else None)

    def ebwd(self, ctx, dy, need_dx, wgrad=True):
        return dy.reshape(ctx["shape"]) if need_dx else None

    def etfwd(self, ctx, xd):
        return xd.reshape(xd.shape[0], -1), {}

    def etbwd(self, ctx, tctx, dy, dyd, need_dx):
        if not need_dx:
            return None, None
        return (dy.reshape(ctx["shape"]) if dy is not None else None), dyd.reshape(ctx["shape"])


class Conv1D(Layer):
    """Causal temporal convolution (K14 north-star variant; not used by the reference scripts).

    Implemented as im2col + the native GEMM: kernel (K, C_in, C_out) is viewed as a Dense kernel
    (K*C_in, C_out) over unfolded windows, so every explicit-engine method reuses Dense's.
    """

    kind = "conv1d"

    def __init__(self, filters: int, kernel_size: int, activation=None, dilation: int = 1):
        super().__init__()
        self.filters, self.k, self.act, self.dil = filters, kernel_size, activation, dilation
        self.act_code = R.act_code(activation)

    def build(self, in_shape):
        T, cin = in_shape[-2], in_shape[-1]
        self.cin = cin
        self.specs = [ParamSpec("kernel", (self.k, cin, self.filters), "glorot_conv"),
                      ParamSpec("bias", (self.filters,), "zeros")]
        return (T, self.filters)

    def forward(self, x):
        return R.conv1d_causal(x, self.w("kernel"), self.w("bias"), self.act, self.dil)

    def _unfold(self, x):
        return Fn.im2col_causal(x, self.k, self.dil)

    def efwd(self, x, save):
        cols = self._unfold(x)
        y = Fn.linear(cols, self.p("kernel").reshape(-1, self.filters), self.p("bias"), self.act_code)
        return y, ({"x": x, "cols": cols, "y": y} if save else None)

    def ebwd(self, ctx, dy, need_dx, wgrad=True):
        dz = Fn.act_backward(dy, ctx["y"], self.act_code)
        if wgrad:
            Fn.run_wgrad(Fn.linear_wgrad_, ctx["cols"], dz, self.g("kernel").reshape(-1, self.filters), self.g("bias"))
        if not need_dx:
            return None
        dcols = Fn.linear_dgrad(dz, self.p("kernel").reshape(-1, self.filters))
        return Fn.col2im_causal(dcols, self.k, self.dil, self.cin)

    def etfwd(self, ctx, xd):
        cols_d = self._unfold(xd)
        zd = Fn.linear(cols_d, self.p("kernel").reshape(-1, self.filters), None, 0)
        return Fn.act_backward(zd, ctx["y"], self.act_code), {"cols_d": cols_d, "zd": zd}

    def etbwd(self, ctx, tctx, dy, dyd, need_dx):
        Wk = self.p("kernel").reshape(-1, self.filters)
        gk = self.g("kernel").reshape(-1, self.filters)
        if dy is None:
            dy = torch.zeros_like(ctx["y"])
        dzd = Fn.act_backward(dyd, ctx["y"], self.act_code)
        dz = Fn.act_tangent_backward(dy, dyd, ctx["y"], tctx["zd"], self.act_code)
        Fn.run_wgrad(Fn.linear_wgrad_, ctx["cols"], dz, gk, self.g("bias"))
        Fn.run_wgrad(Fn.linear_wgrad_, tctx["cols_d"], dzd, gk, None)
        if not need_dx:
            return None, None
        return (Fn.col2im_causal(Fn.linear_dgrad(dz, Wk), self.k, self.dil, self.cin),
                Fn.col2im_causal(Fn.linear_dgrad(dzd, Wk), self.k, self.dil, self.cin))


def _init_tensor(spec: ParamSpec, gen, layer: Layer) -> torch.Tensor:
    if spec.init == "glorot":
        return glorot_uniform(spec.shape, gen)
    if spec.init == "glorot_conv":
        k, cin, cout = spec.shape
        return glorot_uniform(spec.shape, gen, fan_in=k * cin, fan_out=k * cout)
    if spec.init == "orthogonal":
        return orthogonal(spec.shape, gen)
    if spec.init == "zeros":
        return torch.zeros(spec.shape, dtype=torch.float64)
    if spec.init == "ones":
        return torch.ones(spec.shape, dtype=torch.float64)
    if spec.init == "lstm_bias":
        H = spec.shape[0] // 4
        b = torch.zeros(spec.shape, dtype=torch.float64)
        b[H:2 * H] = 1.0  # unit_forget_bias
        return b
    raise ValueError(spec.init)


_ALIGN = 64  # floats; keeps every parameter view 256-B aligned for vector loads


class Sequential(torch.nn.Module):
    """A Keras ``Sequential`` with flat parameter/gradient storage and the explicit engine."""

    _name_counters: dict = {}

    def __init__(self, layers: list[Layer], input_shape, name: str = "sequential", seed: int | None = None,
                 device="cpu", dtype=torch.float32, keras_names: bool = True):
        super().__init__()
        self.layers = list(layers)
        self.input_shape = tuple(input_shape)
        self.model_name = name
        shape = self.input_shape
        off = 0
        self._index: dict = {}
        for li, layer in enumerate(self.layers):
            layer.model = self
            cnt = Sequential._name_counters.get(layer.kind, 0) + 1 if keras_names else li + 1
            Sequential._name_counters[layer.kind] = cnt
            sfx = "" if cnt == 1 else f"_{cnt - 1}"  # Keras uniquifies as x, x_1, x_2, ...
            layer.name = f"{layer.kind}{sfx}"
            layer.in_shape_, shape = shape, layer.build(shape)
            layer.out_shape_ = shape
            for s in layer.specs:
                n = int(np.prod(s.shape))
                s.offset = off
                cell = f"{layer.name}/lstm_cell{sfx}/" if layer.kind == "lstm" else f"{layer.name}/"
                s.keras = f"{cell}{s.name}:0"
                self._index[(id(layer), s.name)] = s
                off += (n + _ALIGN - 1) // _ALIGN * _ALIGN
        self.output_shape = shape
        self.numel_padded = max(off, _ALIGN)
        gen = torch.Generator().manual_seed(seed if seed is not None else 123)
        flat = torch.zeros(self.numel_padded, dtype=torch.float64)
        for layer in self.layers:
            for s in layer.specs:
                n = int(np.prod(s.shape))
                flat[s.offset:s.offset + n] = _init_tensor(s, gen, layer).reshape(-1)
        self.flat = torch.nn.Parameter(flat.to(dtype=dtype, device=device))
        self.flat.grad = torch.zeros_like(self.flat)
        self.compute_dtype = dtype

    # ---- parameter access ----------------------------------------------------------------
    def spec(self, layer, name) -> ParamSpec:
        return self._index[(id(layer), name)]

    def view(self, layer, name):
        s = self.spec(layer, name)
        n = int(np.prod(s.shape))
        return self.flat[s.offset:s.offset + n].view(s.shape)

    def gview(self, layer, name):
        s = self.spec(layer, name)
        n = int(np.prod(s.shape))
        return self.flat.grad[s.offset:s.offset + n].view(s.shape)

    def named_weights(self):
        """[(keras_name, view)] in Keras ``get_weights`` order."""
        return [(s.keras, self.view(l, s.name)) for l in self.layers for s in l.specs]

    def get_weights(self):
        return [v.detach().cpu().numpy().copy() for _, v in self.named_weights()]

    def set_weights(self, arrays):
        with torch.no_grad():
            for (_, v), a in zip(self.named_weights(), arrays):
                v.copy_(torch.as_tensor(np.asarray(a), dtype=v.dtype).reshape(v.shape))

    def count_params(self) -> int:
        return sum(int(np.prod(s.shape)) for l in self.layers for s in l.specs)

    def zero_grad(self, set_to_none: bool = False):  # noqa: D401 - keep the flat grad buffer alive
        self.flat.grad.zero_()

    def to(self, *args, **kwargs):  # keep .grad allocated after moves
        super().to(*args, **kwargs)
        if self.flat.grad is None or self.flat.grad.shape != self.flat.shape or self.flat.grad.device != self.flat.device:
            self.flat.grad = torch.zeros_like(self.flat)
        return self

    def summary(self) -> str:
        lines = [f'Model: "{self.model_name}"', f"{'Layer':<28}{'Output':<20}{'Params':>10}"]
        for l in self.layers:
            n = sum(int(np.prod(s.shape)) for s in l.specs)
            lines.append(f"{l.name:<28}{str((None,) + tuple(l.out_shape_)):<20}{n:>10}")
        lines.append(f"Total params: {self.count_params()}")
        return "\n".join(lines)

    # ---- autograd path -------------------------------------------------------------------
    def forward(self, x):
        for l in self.layers:
            x = l.forward(x)
        return x

    # ---- explicit engine -----------------------------------------------------------------
    def _head_skippable(self) -> bool:
        last = self.layers[-1] if self.layers else None
        return isinstance(last, Dense) and last.act_code == 0

    def efwd(self, x, save: bool = True, out=None, head_out: bool = True, head_wgrad=None):
        """``out``: destination of the model output, used when the last layer can write into it
        (Dense); otherwise the output is copied there.  ``head_out=False``: the caller only needs the
        tape (e.g. the gradient penalty's forward on x_hat, whose score nothing reads): a linear Dense
        head is not evaluated and the returned output is a shape-only placeholder.  ``head_wgrad=(split,
        wa, wb)``: the loss gradient of the output rows is known already (wa for rows < split, wb after:
        the Wasserstein critic terms); a linear Dense(1) head then accumulates its own weight gradient
        in the forward pass (one read of its input) and ``ebwd`` skips it."""
        skip_head = not head_out and self._head_skippable()
        tape = []
        i, n = 0, len(self.layers)
        while i < n:
            l = self.layers[i]
            if isinstance(l, LeakyReLU) and i + 1 < n and isinstance(self.layers[i + 1], LayerNormalization):
                # fused LReLU -> LN pair: one pass, the activation never hits HBM.  The LReLU tape
                # keeps the pre-activation input: its sign is the output's (alpha > 0), which is
                # all the LReLU backward / tangent passes read.
                ln = self.layers[i + 1]
                y, xhat, rstd = Fn.lrelu_layer_norm_fwd(x, ln.p("gamma"), ln.p("beta"), ln.eps, l.alpha, save)
                tape.append({"y": x} if save else None)
                tape.append({"x": None, "x_pre": x, "alpha": l.alpha, "xhat": xhat, "rstd": rstd} if save else None)
                x = y
                i += 2
                continue
            if skip_head and i == n - 1:
                x, ctx = l.efwd(x, save, compute=False)
            elif head_wgrad is not None and i == n - 1 and isinstance(l, Dense) and out is None:
                x, ctx = l.efwd(x, save, wgrad_rows=head_wgrad)
            elif out is not None and i == n - 1 and isinstance(l, Dense):
                x, ctx = l.efwd(x, save, out=out)
            else:
                x, ctx = l.efwd(x, save)
            tape.append(ctx)
            i += 1
        if out is not None and x.data_ptr() != out.data_ptr():
            x = out.copy_(x)
        return x, tape

    @torch.no_grad()
    def predict(self, x, out=None):
        return self.efwd(x, save=False, out=out)[0]

    @staticmethod
    def _adj(layer, dy):
        if isinstance(dy, Fn.OuterAdjoint) and not getattr(layer, "accepts_outer", False):
            return dy.materialize()
        return dy

    def ebwd(self, tape, dy, need_dx: bool = False, wgrad: bool = True, hook=None):
        """Reverse pass; ``hook(i)`` runs after layer i (its gradients are then final)."""
        for i in range(len(self.layers) - 1, -1, -1):
            need = need_dx or i > 0
            layer = self.layers[i]
            dy = layer.ebwd(tape[i], self._adj(layer, dy), need, wgrad)
            if hook is not None:
                hook(i)
        return Fn._mat(dy)

    def etfwd(self, tape, xd, head_out: bool = True):
        """``head_out=False``: the tangent of a linear Dense head is not evaluated (placeholder), as in
        ``efwd``."""
        skip_head = not head_out and self._head_skippable()
        ttape = []
        n = len(self.layers)
        for i, (l, ctx) in enumerate(zip(self.layers, tape)):
            if skip_head and i == n - 1:
                xd, tctx = l.etfwd(ctx, xd, compute=False)
            else:
                xd, tctx = l.etfwd(ctx, xd)
            ttape.append(tctx)
        return xd, ttape

    def etbwd(self, tape, ttape, dy, dyd, need_dx: bool = False, hook=None):
        for i in range(len(self.layers) - 1, -1, -1):
            need = need_dx or i > 0
            layer = self.layers[i]
            dy, dyd = layer.etbwd(tape[i], ttape[i], self._adj(layer, dy), self._adj(layer, dyd), need)
            if hook is not None:
                hook(i)
        return Fn._mat(dy), Fn._mat(dyd)

    def grad_buckets(self, n: int = 2) -> list[tuple[int, int, int]]:
        """Split the flat gradient buffer at layer boundaries into <= n buckets of similar size.

        Returns ``[(first_layer, start, end)]`` in reverse-pass completion order (the bucket of
        the LAST layers first): bucket b is final as soon as the reverse pass has processed its
        ``first_layer``, so its all-reduce can overlap the backward of the earlier layers.
        """
        starts = []
        for li, l in enumerate(self.layers):
            if l.specs:
                starts.append((li, min(s.offset for s in l.specs)))
        if not starts:
            return []
        total = self.numel_padded
        cuts = [starts[0]]
        for k in range(1, max(n, 1)):  # the layer boundary closest to k/n of the buffer
            goal = total * k / n
            li, off = min(starts[1:] or starts, key=lambda c: abs(c[1] - goal))
            if off > cuts[-1][1]:
                cuts.append((li, off))
        out = []
        for j, (li, off) in enumerate(cuts):
            end = cuts[j + 1][1] if j + 1 < len(cuts) else total
            out.append((li, off, end))
        return out[::-1]
