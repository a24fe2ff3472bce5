"""Pure-PyTorch reference implementations (Keras 2.7 semantics).

Two families live here:

1. **Composed, autograd-differentiable ops** (`dense`, `lstm`, `layer_norm`, losses, ...).  They
   are the numerical oracle for the HIP kernels and the CPU execution path; autograd through them
   supports double-backward, so a WGAN-GP gradient penalty can be formed with
   ``torch.autograd.grad(create_graph=True)`` exactly like the reference's ``K.gradients``
   (GAN/MTSS_WGAN_GP.py:201-216).

2. **Explicit primitive kernels** (`lstm_seq_fwd`, `lstm_seq_bwd`, `lstm_seq_tfwd`,
   `lstm_seq_tbwd`, ...).  These define the exact contract of the native HIP kernels: a
   persistent LSTM forward that saves gate activations and cell states, its BPTT backward, the
   *tangent* (forward-mode) LSTM at a saved primal point and the reverse pass of that tangent
   system.  The WGAN-GP critic update needs d/dtheta <v, dD/dx> (a Hessian-vector product);
   computing it as reverse-over-tangent turns the second-order pass into four first-order
   recurrences with hand-derived adjoints.  The CPU versions are vectorised over the batch and
   loop over time only.

Keras conventions reproduced: gate order [i, f, c(g), o]; ``z = x W + h U + b``;
recurrent activation sigmoid; cell activation in {tanh, sigmoid, linear}; LayerNorm eps 1e-3;
LeakyReLU alpha 0.2; BCE clipping at 1e-7; Wasserstein loss mean(y_true * y_pred).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

ACT_CODES = {"linear": 0, None: 0, "sigmoid": 1, "tanh": 2, "leaky_relu": 3, "relu": 4}
LRELU_ALPHA = 0.2
LN_EPS = 1e-3
KERAS_EPS = 1e-7


def act_code(name) -> int:
    return ACT_CODES[name]


def apply_act(x: torch.Tensor, act) -> torch.Tensor:
    a = act_code(act) if not isinstance(act, int) else act
    if a == 0:
        return x
    if a == 1:
        return torch.sigmoid(x)
    if a == 2:
        return torch.tanh(x)
    if a == 3:
        return F.leaky_relu(x, LRELU_ALPHA)
    if a == 4:
        return torch.relu(x)
    raise ValueError(act)


def act_dy(y: torch.Tensor, act) -> torch.Tensor:
    """f'(x) expressed through y = f(x)."""
    a = act_code(act) if not isinstance(act, int) else act
    if a == 0:
        return torch.ones_like(y)
    if a == 1:
        return y * (1 - y)
    if a == 2:
        return 1 - y * y
    if a == 3:
        return torch.where(y >= 0, torch.ones_like(y), torch.full_like(y, LRELU_ALPHA))
    if a == 4:
        return (y > 0).to(y.dtype)
    raise ValueError(act)


def act_d2y(y: torch.Tensor, act) -> torch.Tensor:
    """f''(x) expressed through y = f(x) (zero for piecewise-linear acts)."""
    a = act_code(act) if not isinstance(act, int) else act
    if a == 1:
        return y * (1 - y) * (1 - 2 * y)
    if a == 2:
        return -2 * y * (1 - y * y)
    return torch.zeros_like(y)


# ======================================================================================
# 1. composed differentiable ops
# ======================================================================================
def dense(x: torch.Tensor, kernel: torch.Tensor, bias: torch.Tensor | None = None, act=None) -> torch.Tensor:
    """Keras Dense on the last axis; kernel layout (in, out)."""
    y = torch.matmul(x, kernel)
    if bias is not None:
        y = y + bias
    return apply_act(y, act)


def lstm(x: torch.Tensor, kernel, recurrent_kernel, bias, act="tanh", rec_act="sigmoid",
         h0=None, c0=None, return_state=False):
    """Keras LSTM(return_sequences=True), implementation 2 (fused gates). x: (B, T, in)."""
    B, T, _ = x.shape
    H = recurrent_kernel.shape[0]
    zx = torch.matmul(x, kernel) + bias
    h = x.new_zeros(B, H) if h0 is None else h0
    c = x.new_zeros(B, H) if c0 is None else c0
    outs = []
    for t in range(T):
        z = zx[:, t] + h @ recurrent_kernel
        zi, zf, zg, zo = z.split(H, dim=-1)
        i = apply_act(zi, rec_act)
        f = apply_act(zf, rec_act)
        g = apply_act(zg, act)
        o = apply_act(zo, rec_act)
        c = f * c + i * g
        h = o * apply_act(c, act)
        outs.append(h)
    y = torch.stack(outs, dim=1)
    return (y, (h, c)) if return_state else y


def layer_norm(x: torch.Tensor, gamma, beta, eps: float = LN_EPS) -> torch.Tensor:
    mu = x.mean(dim=-1, keepdim=True)
    var = ((x - mu) ** 2).mean(dim=-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * gamma + beta


def leaky_relu(x: torch.Tensor, alpha: float = LRELU_ALPHA) -> torch.Tensor:
    return F.leaky_relu(x, alpha)


def conv1d_causal(x: torch.Tensor, kernel: torch.Tensor, bias=None, act=None, dilation: int = 1):
    """Temporal conv over (B, T, C_in) with kernel (K, C_in, C_out), causal (left) padding."""
    K = kernel.shape[0]
    pad = (K - 1) * dilation
    xt = F.pad(x.transpose(1, 2), (pad, 0))
    w = kernel.permute(2, 1, 0)  # (C_out, C_in, K)
    y = F.conv1d(xt, w, bias=bias, dilation=dilation).transpose(1, 2)
    return apply_act(y, act)


# ---- losses (Keras 2.7) ----
def wasserstein_loss(y_true: torch.Tensor, y_pred: torch.Tensor) -> torch.Tensor:
    """K.mean(y_true * y_pred) with Keras' rank alignment: (B,1) labels vs (B,T,1) preds."""
    if y_pred.dim() == y_true.dim() + 1 and y_pred.shape[-1] == 1:
        y_pred = y_pred.squeeze(-1)
    return torch.mean(y_true * y_pred)


def binary_crossentropy(y_true: torch.Tensor, y_pred: torch.Tensor) -> torch.Tensor:
    if y_pred.dim() == y_true.dim() + 1 and y_pred.shape[-1] == 1:
        y_pred = y_pred.squeeze(-1)
    o = torch.clamp(y_pred, KERAS_EPS, 1 - KERAS_EPS)
    bce = y_true * torch.log(o + KERAS_EPS) + (1 - y_true) * torch.log(1 - o + KERAS_EPS)
    return -bce.mean()


def mse(y_true, y_pred):
    return torch.mean((y_true - y_pred) ** 2)


def gradient_penalty_from_grad(g: torch.Tensor) -> torch.Tensor:
    """mean((1 - ||g||_2)^2) with the norm over every non-batch axis (GAN/MTSS_WGAN_GP.py:201-216)."""
    n = torch.sqrt(torch.sum(g.reshape(g.shape[0], -1) ** 2, dim=1))
    return torch.mean((1 - n) ** 2)


def gan_loss(p: torch.Tensor, split: int, la: float, lb: float, kind: int, acc=torch.float32):
    """Contract of the native ``gan_loss`` op (csrc/misc.hip): the flattened scores p are two
    segments, [0, split) with label ``la`` and [split, n) with label ``lb``; returns
    (per-segment mean losses [2] in ``acc``, dL/dp like p) for L = loss_0 + loss_1.
    kind 0: Wasserstein ``mean(y * p)`` (GAN/WGAN.py:126-127); kind 1: Keras binary cross-entropy
    on probabilities with the [eps, 1 - eps] clip (zero gradient where the clip is active)."""
    pf = p.reshape(-1).to(acc)
    n = pf.numel()
    y = torch.full_like(pf, lb)
    y[:split] = la
    inv = torch.full_like(pf, 1.0 / max(n - split, 1))
    inv[:split] = 1.0 / max(split, 1)
    if kind == 0:
        lo, g = y * pf, y * inv
    else:
        o = pf.clamp(KERAS_EPS, 1 - KERAS_EPS)
        lo = -(y * torch.log(o + KERAS_EPS) + (1 - y) * torch.log(1 - o + KERAS_EPS))
        inside = ((pf > KERAS_EPS) & (pf < 1 - KERAS_EPS)).to(acc)
        g = -(y / (o + KERAS_EPS) - (1 - y) / (1 - o + KERAS_EPS)) * inside * inv
    li = lo * inv
    out = torch.stack([li[:split].sum(), li[split:].sum()])
    return out, g.to(p.dtype).reshape(p.shape)


def gp_coef(g: torch.Tensor, weight: float):
    """Explicit GP adjoint: returns (penalty value, v = dL/dg) for L = weight*mean((1-||g||)^2)."""
    B = g.shape[0]
    gf = g.reshape(B, -1)
    n = torch.sqrt(torch.sum(gf * gf, dim=1))
    pen = torch.mean((1 - n) ** 2)
    scale = -(2.0 * weight / B) * (1 - n) / torch.clamp(n, min=1e-30)
    v = (gf * scale[:, None]).reshape(g.shape)
    return pen, v


# ======================================================================================
# 2. explicit primitives (contracts of the native kernels)
# ======================================================================================
def lstm_seq_fwd(zx: torch.Tensor, U: torch.Tensor, act: int, save: bool = True):
    """Recurrence given the input projection ``zx = x W + b`` (B, T, 4H).

    Returns ``h_seq`` (B,T,H) and, if ``save``, gate activations (B,T,4H) [i,f,g,o] and cell
    states (B,T,H).
    """
    B, T, G = zx.shape
    H = G // 4
    h = zx.new_zeros(B, H)
    c = zx.new_zeros(B, H)
    hs = zx.new_empty(B, T, H)
    gates = zx.new_empty(B, T, G) if save else None
    cs = zx.new_empty(B, T, H) if save else None
    for t in range(T):
        z = zx[:, t] + h @ U
        i = torch.sigmoid(z[:, :H])
        f = torch.sigmoid(z[:, H:2 * H])
        g = apply_act(z[:, 2 * H:3 * H], act)
        o = torch.sigmoid(z[:, 3 * H:])
        c = f * c + i * g
        h = o * apply_act(c, act)
        hs[:, t] = h
        if save:
            gates[:, t] = torch.cat([i, f, g, o], dim=1)
            cs[:, t] = c
    return hs, gates, cs


def lstm_seq_bwd(dh_seq: torch.Tensor, gates: torch.Tensor, cs: torch.Tensor, U: torch.Tensor, act: int):
    """BPTT through the recurrence: returns dZ (B,T,4H) = dL/d(zx) for every step."""
    B, T, G = gates.shape
    H = G // 4
    dz_all = torch.empty_like(gates)
    dh = dh_seq.new_zeros(B, H)
    dc = dh_seq.new_zeros(B, H)
    Ut = U.t()
    for t in range(T - 1, -1, -1):
        i, f, g, o = gates[:, t].split(H, dim=1)
        c = cs[:, t]
        cp = cs[:, t - 1] if t > 0 else torch.zeros_like(c)
        ca = apply_act(c, act)
        dht = dh_seq[:, t] + dh
        do = dht * ca
        dct = dc + dht * o * act_dy(ca, act)
        di, dg, df = dct * g, dct * i, dct * cp
        dc = dct * f
        dz = torch.cat([di * i * (1 - i), df * f * (1 - f), dg * act_dy(g, act), do * o * (1 - o)], dim=1)
        dz_all[:, t] = dz
        dh = dz @ Ut
    return dz_all


def lstm_seq_tfwd(dzx: torch.Tensor, gates: torch.Tensor, cs: torch.Tensor, U: torch.Tensor, act: int):
    """Tangent (JVP) of the recurrence at a saved primal point.

    ``dzx`` = xdot W (no bias).  Returns (hdot_seq (B,T,H), zdot (B,T,4H), cdot (B,T,H)).
    """
    B, T, G = gates.shape
    H = G // 4
    hd = dzx.new_zeros(B, H)
    cd = dzx.new_zeros(B, H)
    hds = dzx.new_empty(B, T, H)
    zds = dzx.new_empty(B, T, G)
    cds = dzx.new_empty(B, T, H)
    for t in range(T):
        zd = dzx[:, t] + hd @ U
        i, f, g, o = gates[:, t].split(H, dim=1)
        c = cs[:, t]
        cp = cs[:, t - 1] if t > 0 else torch.zeros_like(c)
        idot = i * (1 - i) * zd[:, :H]
        fdot = f * (1 - f) * zd[:, H:2 * H]
        gdot = act_dy(g, act) * zd[:, 2 * H:3 * H]
        odot = o * (1 - o) * zd[:, 3 * H:]
        cd = fdot * cp + f * cd + idot * g + i * gdot
        ca = apply_act(c, act)
        hd = odot * ca + o * act_dy(ca, act) * cd
        hds[:, t] = hd
        zds[:, t] = zd
        cds[:, t] = cd
    return hds, zds, cds


def lstm_seq_tbwd(dh_seq, dhd_seq, gates, cs, zds, cds, U, act: int):
    """Reverse pass of the tangent system.

    Given adjoints of the primal outputs (``dh_seq``) and of the tangent outputs (``dhd_seq``),
    returns (dZ, dZdot): adjoints of ``zx`` and of ``dzx`` for every step.
    """
    B, T, G = gates.shape
    H = G // 4
    dZ = torch.empty_like(gates)
    dZd = torch.empty_like(gates)
    ah_n = gates.new_zeros(B, H)   # h-bar carried from step t+1
    ahd_n = gates.new_zeros(B, H)  # hdot-bar carried
    ac_n = gates.new_zeros(B, H)   # c-bar carried
    acd_n = gates.new_zeros(B, H)  # cdot-bar carried
    Ut = U.t()
    for t in range(T - 1, -1, -1):
        i, f, g, o = gates[:, t].split(H, dim=1)
        c = cs[:, t]
        cd = cds[:, t]
        cp = cs[:, t - 1] if t > 0 else torch.zeros_like(c)
        cdp = cds[:, t - 1] if t > 0 else torch.zeros_like(c)
        zd = zds[:, t]
        zdi, zdf, zdg, zdo = zd.split(H, dim=1)
        si, sf, so = i * (1 - i), f * (1 - f), o * (1 - o)
        sg = act_dy(g, act)
        idot, fdot, gdot, odot = si * zdi, sf * zdf, sg * zdg, so * zdo
        ca = apply_act(c, act)
        d1 = act_dy(ca, act)
        d2 = act_d2y(ca, act)
        a_h = dh_seq[:, t] + ah_n
        a_hd = dhd_seq[:, t] + ahd_n
        a_od = a_hd * ca
        a_o = a_h * ca + a_hd * d1 * cd
        a_cd = acd_n + a_hd * o * d1
        a_c = ac_n + a_h * o * d1 + a_hd * (odot * d1 + o * d2 * cd)
        a_fd = a_cd * cp
        a_id = a_cd * g
        a_gd = a_cd * i
        a_f = a_c * cp + a_cd * cdp
        a_i = a_c * g + a_cd * gdot
        a_g = a_c * i + a_cd * idot
        ac_n = a_c * f + a_cd * fdot
        acd_n = a_cd * f
        s2i = si * (1 - 2 * i)
        s2f = sf * (1 - 2 * f)
        s2o = so * (1 - 2 * o)
        s2g = act_d2y(g, act)
        dzd = torch.cat([a_id * si, a_fd * sf, a_gd * sg, a_od * so], dim=1)
        dz = torch.cat([a_i * si + a_id * s2i * zdi, a_f * sf + a_fd * s2f * zdf,
                        a_g * sg + a_gd * s2g * zdg, a_o * so + a_od * s2o * zdo], dim=1)
        dZ[:, t] = dz
        dZd[:, t] = dzd
        ah_n = dz @ Ut
        ahd_n = dzd @ Ut
    return dZ, dZd


def shift_prev(h_seq: torch.Tensor) -> torch.Tensor:
    """h_{t-1} sequence with h_{-1} = 0."""
    out = torch.zeros_like(h_seq)
    out[:, 1:] = h_seq[:, :-1]
    return out


def layer_norm_fwd(x: torch.Tensor, gamma, beta, eps: float = LN_EPS):
    """Returns (y, xhat, rstd) for an explicit backward."""
    mu = x.mean(dim=-1, keepdim=True)
    var = ((x - mu) ** 2).mean(dim=-1, keepdim=True)
    rstd = torch.rsqrt(var + eps)
    xhat = (x - mu) * rstd
    return xhat * gamma + beta, xhat, rstd


def layer_norm_bwd(dy: torch.Tensor, xhat: torch.Tensor, rstd: torch.Tensor, gamma):
    """Returns (dx, dgamma, dbeta)."""
    g = dy * gamma
    n = xhat.shape[-1]
    dx = rstd * (g - g.mean(dim=-1, keepdim=True) - xhat * (g * xhat).mean(dim=-1, keepdim=True))
    red = tuple(range(dy.dim() - 1))
    return dx, (dy * xhat).sum(dim=red), dy.sum(dim=red)


def layer_norm_tfwd(xd: torch.Tensor, xhat: torch.Tensor, rstd: torch.Tensor, gamma):
    """JVP of LayerNorm w.r.t. its input: gamma * r (xd - mean(xd) - xhat mean(xhat xd))."""
    m = (xhat * xd).mean(dim=-1, keepdim=True)
    return gamma * (rstd * (xd - xd.mean(dim=-1, keepdim=True) - xhat * m))


def layer_norm_tbwd(dy, dyd: torch.Tensor, xd: torch.Tensor, xhat: torch.Tensor, rstd: torch.Tensor, gamma):
    """Reverse of (y, yd) = (LN(x), JVP(x; xd)) with seeds (dy, dyd); dy None = zero.

    Returns (dx, dxd, dgamma, dbeta); the closed form the native kernel evaluates (csrc/misc.hip).
    """
    D = xhat.shape[-1]
    r = rstd
    mxd = xd.mean(dim=-1, keepdim=True)
    m = (xhat * xd).mean(dim=-1, keepdim=True)
    xhatd = r * (xd - mxd - xhat * m)
    h = dyd * gamma
    mh = h.mean(dim=-1, keepdim=True)
    S = (h * xhat).sum(dim=-1, keepdim=True)
    P = (h * xd).sum(dim=-1, keepdim=True)
    dxd = r * (h - mh - xhat * S / D)
    g = dy * gamma if dy is not None else torch.zeros_like(h)
    G = g - r * m * h - (r * S / D) * xd
    dx = r * (G - G.mean(dim=-1, keepdim=True) - xhat * (G * xhat).mean(dim=-1, keepdim=True)) \
        - r * r * xhat * (P - D * mxd * mh - m * S) / D
    red = tuple(range(dyd.dim() - 1))
    dgamma = (dyd * xhatd).sum(dim=red)
    dbeta = torch.zeros_like(dgamma)
    if dy is not None:
        dgamma = dgamma + (dy * xhat).sum(dim=red)
        dbeta = dy.sum(dim=red)
    return dx, dxd, dgamma, dbeta
