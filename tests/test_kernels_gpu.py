"""HIP kernel numerics vs plain PyTorch fp32/fp64 references (run on an MI355X with -m gpu).

Every native op in ``torch.ops.hfrep`` is compared against the reference implementation of the
same op (``hfrep.ops.reference``) evaluated in fp64 on the CPU.  fp32 kernels run either on the
exact-f32 MFMA (16x16x4 f32) or -- the default for the recurrent products, weight gradients and the
K = 100 input gradient -- as the fp32-accurate three-term bf16 split (every operand h + m + l, six
products); both are held to fp32-level tolerances, and the split kernels to <= 2x the exact kernel's
error vs fp64 (``test_lstmf_*split*``).  bf16 kernels are compared with bf16-level tolerances relative
to the output scale.
"""
import numpy as np
import pytest
import torch

from hfrep.ops import reference as R

pytestmark = pytest.mark.gpu

TOL = {torch.float32: dict(rtol=2e-4, atol=2e-5), torch.bfloat16: dict(rtol=5e-2, atol=3e-2)}


def _close(got, ref, dt, scale=None):
    got = got.double().cpu()
    ref = ref.double().cpu()
    s = scale if scale is not None else max(ref.abs().max().item(), 1e-3)
    t = TOL[dt]
    err = (got - ref).abs().max().item()
    assert err <= t["atol"] * max(1.0, s) + t["rtol"] * s, f"max err {err:.3e} (scale {s:.3e})"


def _ops():
    from hfrep.ops import _native

    return _native.native()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,K,N,act", [(1000, 32, 400, 0), (777, 100, 400, 0), (300, 35, 100, 1), (64, 2400, 1, 0),
                                       (257, 100, 35, 3), (40, 100, 100, 2), (70001, 100, 32, 0), (333, 36, 36, 1),
                                       (129, 22, 7, 3), (70001, 300, 100, 3), (1000, 96, 100, 3), (33, 300, 100, 0),
                                       (517, 200, 250, 1), (77, 1, 22, 3), (130, 3, 22, 3), (65, 5, 22, 0), (99, 4, 22, 3)])
def test_linear(cuda, dt, M, K, N, act):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(M, K, generator=g) * 0.5
    W = torch.randn(K, N, generator=g) * (1.0 / K ** 0.5)
    b = torch.randn(N, generator=g) * 0.1
    y = _ops().linear(x.to(cuda, dt), W.to(cuda), b.to(cuda), act)
    ref = R.apply_act(x.double().to(dt).double() @ W.double() + b.double(), act)
    _close(y, ref, dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(1000, 400, 100), (513, 400, 32), (64, 1, 2400), (70001, 100, 300),
                                   (999, 100, 96), (17, 300, 300)])
def test_linear_dgrad(cuda, dt, M, N, K):
    g = torch.Generator().manual_seed(1)
    dz = torch.randn(M, N, generator=g)
    W = torch.randn(K, N, generator=g) * 0.1
    dx = _ops().linear_dgrad(dz.to(cuda, dt), W.to(cuda))
    _close(dx, dz.to(dt).double() @ W.double().t(), dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,K,N,shift", [(5000, 100, 400, 0), (4800, 100, 400, 24), (96, 32, 400, 0), (64, 2400, 1, 0),
                                         (70001, 100, 32, 0), (777, 32, 20, 0), (300, 36, 7, 0)])
def test_wgrad(cuda, dt, M, K, N, shift):
    g = torch.Generator().manual_seed(2)
    x = torch.randn(M, K, generator=g)
    dz = torch.randn(M, N, generator=g) * 0.1
    gW0 = torch.randn(K, N, generator=g)
    gb0 = torch.randn(N, generator=g)
    gW, gb = gW0.clone().to(cuda), gb0.clone().to(cuda)
    _ops().linear_wgrad_(x.to(cuda, dt), dz.to(cuda, dt), gW, gb, shift)
    xr = x.to(dt).double()
    if shift:
        xr = R.shift_prev(xr.reshape(-1, shift, K)).reshape(M, K)
    d = dz.to(dt).double()
    _close(gW, gW0.double() + xr.t() @ d, dt, scale=(xr.abs().t() @ d.abs()).max().item())
    _close(gb, gb0.double() + d.sum(0), dt, scale=d.abs().sum(0).max().item())


def _lstm_inputs(B, T, H, seed, dt):
    g = torch.Generator().manual_seed(seed)
    zx = torch.randn(B, T, 4 * H, generator=g) * 0.7
    U = torch.randn(H, 4 * H, generator=g) * (1.0 / H ** 0.5)
    return zx, U


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act", [2, 1, 0])
@pytest.mark.parametrize("B,T,H", [(33, 24, 100), (70, 7, 100), (32, 48, 64)])
def test_lstm_fwd_bwd(cuda, dt, act, B, T, H):
    zx, U = _lstm_inputs(B, T, H, 3, dt)
    zxd = zx.to(dt)
    hs, gates, cs = _ops().lstm_fwd(zxd.to(cuda), U.to(cuda), act, True)
    rh, rg, rc = R.lstm_seq_fwd(zxd.double(), U.to(dt).double() if dt == torch.bfloat16 else U.double(), act)
    _close(hs, rh, dt)
    _close(gates, rg, dt)
    _close(cs, rc, dt)
    dH = torch.randn(B, T, H, generator=torch.Generator().manual_seed(4)).to(dt)
    dZ = _ops().lstm_bwd(dH.to(cuda), gates, cs, U.to(cuda), act)
    ref = R.lstm_seq_bwd(dH.double(), gates.double().cpu(), cs.double().cpu(), U.double(), act)
    _close(dZ, ref, dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act", [2, 1, 0])
def test_lstm_tangent(cuda, dt, act):
    B, T, H = 45, 12, 100
    zx, U = _lstm_inputs(B, T, H, 5, dt)
    zxd = zx.to(dt)
    hs, gates, cs = _ops().lstm_fwd(zxd.to(cuda), U.to(cuda), act, True)
    g = torch.Generator().manual_seed(6)
    dzx = (torch.randn(B, T, 4 * H, generator=g) * 0.3).to(dt)
    hds, zds, cds = _ops().lstm_tfwd(dzx.to(cuda), gates, cs, U.to(cuda), act)
    G64, C64 = gates.double().cpu(), cs.double().cpu()
    rh, rz, rc = R.lstm_seq_tfwd(dzx.double(), G64, C64, U.double(), act)
    _close(hds, rh, dt)
    _close(cds, rc, dt)
    dH = (torch.randn(B, T, H, generator=g) * 0.5).to(dt)
    dHd = torch.randn(B, T, H, generator=g).to(dt)
    dZ, dZd = _ops().lstm_tbwd(dH.to(cuda), dHd.to(cuda), gates, cs, zds, cds, U.to(cuda), act)
    rZ, rZd = R.lstm_seq_tbwd(dH.double(), dHd.double(), G64, C64, zds.double().cpu(), cds.double().cpu(), U.double(), act)
    _close(dZ, rZ, dt)
    _close(dZd, rZd, dt)
    # dH = None path (pure tangent adjoint)
    dZ0, dZd0 = _ops().lstm_tbwd(None, dHd.to(cuda), gates, cs, zds, cds, U.to(cuda), act)
    rZ0, rZd0 = R.lstm_seq_tbwd(torch.zeros_like(dH).double(), dHd.double(), G64, C64, zds.double().cpu(),
                                cds.double().cpu(), U.double(), act)
    _close(dZ0, rZ0, dt)
    _close(dZd0, rZd0, dt)


@pytest.mark.parametrize("D", [100, 35])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_layernorm(cuda, dt, D):
    g = torch.Generator().manual_seed(7)
    x = (torch.randn(37, 11, D, generator=g) * 2 + 0.5).to(dt)
    gamma, beta = torch.randn(D, generator=g), torch.randn(D, generator=g)
    y, xhat, rstd = _ops().layernorm_fwd(x.to(cuda), gamma.to(cuda), beta.to(cuda), 1e-3)
    ry, rxh, rrs = R.layer_norm_fwd(x.double(), gamma.double(), beta.double(), 1e-3)
    _close(y, ry, dt)
    _close(xhat, rxh, dt)
    _close(rstd, rrs, dt)
    # no-grad form: same y, nothing saved
    y2, xh2, rs2 = _ops().layernorm_fwd(x.to(cuda), gamma.to(cuda), beta.to(cuda), 1e-3, False)
    assert torch.equal(y2, y) and xh2.numel() == 0 and rs2.numel() == 0
    # fused LeakyReLU -> LN == the activation kernel followed by LN, bitwise
    xa = _ops().act_fwd(x.to(cuda), 3)
    ya, xha, rsa = _ops().layernorm_fwd(xa, gamma.to(cuda), beta.to(cuda), 1e-3)
    for save in (True, False):
        yf, xhf, rsf = _ops().layernorm_fwd(x.to(cuda), gamma.to(cuda), beta.to(cuda), 1e-3, save, 0.2)
        assert torch.equal(yf, ya)
        if save:
            assert torch.equal(xhf, xha) and torch.equal(rsf, rsa)
    dy = torch.randn(37, 11, D, generator=g).to(dt)
    gg, gb = torch.zeros(D, device=cuda), torch.zeros(D, device=cuda)
    dx = _ops().layernorm_bwd_(dy.to(cuda), xhat, rstd, gamma.to(cuda), gg, gb)
    rdx, rdg, rdb = R.layer_norm_bwd(dy.double(), xhat.double().cpu(), rstd.double().cpu(), gamma.double())
    _close(dx, rdx, dt)
    _close(gg, rdg, dt, scale=(dy.double().abs() * xhat.double().cpu().abs()).sum((0, 1)).max().item())
    _close(gb, rdb, dt, scale=dy.double().abs().sum((0, 1)).max().item())


@pytest.mark.parametrize("D", [100, 35, 256])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_layernorm_tangent(cuda, dt, D):
    """LN JVP + its reverse (the GP critic's LayerNorm) vs torch.func over the fp64 LN: the
    closed form in csrc/misc.hip against nested autodiff, with and without a primal seed."""
    g = torch.Generator().manual_seed(17)
    x = (torch.randn(29, 13, D, generator=g) * 2 + 0.5).double()
    xd = torch.randn(29, 13, D, generator=g).double()
    gamma, beta = torch.randn(D, generator=g).double(), torch.randn(D, generator=g).double()
    dy, dyd = torch.randn(29, 13, D, generator=g).double(), torch.randn(29, 13, D, generator=g).double()
    _, xhat, rstd = _ops().layernorm_fwd(x.to(dt).to(cuda), gamma.float().to(cuda), beta.float().to(cuda), 1e-3)
    xq = x.to(dt).double()  # the kernel's input as rounded to dt
    yd = _ops().layernorm_tfwd(xd.to(dt).to(cuda), xhat, rstd, gamma.float().to(cuda))

    def ln(q, ga, be):
        return R.layer_norm(q, ga, be, 1e-3)

    for with_dy in (True, False):
        xs, xds = xq.clone().requires_grad_(True), xd.to(dt).double().requires_grad_(True)
        gs, bs = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
        y, ryd = torch.func.jvp(lambda q: ln(q, gs, bs), (xs,), (xds,))
        seeds = [dy.to(dt).double() if with_dy else torch.zeros_like(dy), dyd.to(dt).double()]
        rdx, rdxd, rdg, rdb = torch.autograd.grad([y, ryd], [xs, xds, gs, bs], seeds)
        if with_dy:
            _close(yd, ryd.detach(), dt)
        gg, gb = torch.zeros(D, device=cuda), torch.zeros(D, device=cuda)
        dx, dxd = _ops().layernorm_tbwd_(dy.to(dt).to(cuda) if with_dy else None, dyd.to(dt).to(cuda),
                                         xd.to(dt).to(cuda), xhat, rstd, gamma.float().to(cuda), gg, gb, True)
        _close(dx, rdx, dt)
        _close(dxd, rdxd, dt)
        _close(gg, rdg, dt, scale=(dyd.abs() * 4).sum((0, 1)).max().item())
        _close(gb, rdb, dt, scale=dy.abs().sum((0, 1)).max().item())
        # parameter-gradient-only form: same dgamma / dbeta, nothing written for dx / dxd
        gg2, gb2 = torch.zeros(D, device=cuda), torch.zeros(D, device=cuda)
        e1, e2 = _ops().layernorm_tbwd_(dy.to(dt).to(cuda) if with_dy else None, dyd.to(dt).to(cuda),
                                        xd.to(dt).to(cuda), xhat, rstd, gamma.float().to(cuda), gg2, gb2, False)
        assert e1.numel() == 0 and e2.numel() == 0
        assert torch.equal(gg2, gg) and torch.equal(gb2, gb)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gp_coef_and_interpolate(cuda, dt):
    g = torch.Generator().manual_seed(8)
    gr = (torch.randn(64, 24, 32, generator=g) * 0.05).to(dt)
    pen, v = _ops().gp_coef(gr.to(cuda), 10.0)
    rp, rv = R.gp_coef(gr.double(), 10.0)
    assert abs(pen.item() - rp.item()) <= 1e-4 * max(1, abs(rp.item()))
    _close(v, rv, dt)
    # the critic step's loss record from the same launch pair: [w0 + w1 + 10 pen, w0, w1, pen]
    w = torch.tensor([0.25, -1.5], device=cuda)
    pack, v2 = _ops().gp_coef_pack(gr.to(cuda), 10.0, w)
    assert torch.equal(v2, v) and pack[3].item() == pen.item()
    want = torch.tensor([0.25 - 1.5 + 10.0 * pen.item(), 0.25, -1.5, pen.item()])
    assert torch.allclose(pack.cpu(), want, rtol=1e-6, atol=1e-6), (pack, want)
    a, b = torch.rand(64, 24, 32, generator=g).to(dt), torch.rand(64, 24, 32, generator=g).to(dt)
    al = torch.rand(64, generator=g)
    out = _ops().interpolate(a.to(cuda), b.to(cuda), al.to(cuda))
    _close(out, al.double()[:, None, None] * a.double() + (1 - al.double()[:, None, None]) * b.double(), dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_act_kernels(cuda, dt):
    x = torch.randn(10007, generator=torch.Generator().manual_seed(9)).to(dt)
    for act in (1, 2, 3, 4):
        y = _ops().act_fwd(x.to(cuda), act)
        _close(y, R.apply_act(x.double(), act), dt)
        dy = torch.randn_like(x, dtype=torch.float32).to(dt)
        dx = _ops().act_bwd(dy.to(cuda), y, act)
        _close(dx, dy.double() * R.act_dy(y.double().cpu(), act), dt)


def test_rng_and_sampling(cuda):
    from hfrep.utils.rng import DeviceRNG

    r = DeviceRNG(123, cuda)
    z = r.normal((200000,))
    assert abs(z.mean().item()) < 0.01 and abs(z.std().item() - 1) < 0.01
    z2 = r.normal((200000,))
    assert not torch.equal(z, z2), "counter must advance between draws"
    u = r.uniform((100000,))
    assert 0 < u.min().item() and u.max().item() <= 1 and abs(u.mean().item() - 0.5) < 0.01
    data = torch.arange(50 * 6, dtype=torch.float32, device=cuda).reshape(50, 3, 2)
    s = r.sample_windows(data, 4096)
    idx = (s[:, 0, 0] / 6).long()
    assert torch.equal(s, data[idx])
    counts = torch.bincount(idx, minlength=50).float()
    assert counts.min().item() > 40  # roughly uniform over the 50 windows
    # determinism: same seed/stream -> same stream of numbers
    a, b = DeviceRNG(7, cuda), DeviceRNG(7, cuda)
    assert torch.equal(a.normal((1000,)), b.normal((1000,)))


def test_rng_and_sampling_vector_paths(cuda):
    """The 16-byte paths of the sampler (one wave per window, D % 4 == 0: the bench's 24 x 32 windows)
    and of the Philox fill: bf16 draws are the RNE rounding of the fp32 draws of the same stream (odd
    length: vector body + scalar tail), and sample b's window depends only on (seed, counter + b), not
    on the launch shape."""
    from hfrep.utils.rng import DeviceRNG

    for dt in (torch.float32, torch.bfloat16):
        zf = DeviceRNG(5, cuda).normal((1001,))
        zb = DeviceRNG(5, cuda).normal((1001,), dtype=dt)
        assert zb.dtype == dt and torch.equal(zb, zf.to(dt))
        uf, ub = DeviceRNG(6, cuda).uniform((333,)), DeviceRNG(6, cuda).uniform((333,), dtype=dt)
        assert torch.equal(ub, uf.to(dt))
    data = torch.randn(300, 24, 32, device=cuda)
    for dt in (torch.float32, torch.bfloat16):
        a, b = DeviceRNG(9, cuda), DeviceRNG(9, cuda)
        sa = a.sample_windows(data, 100, out_dtype=dt)
        sb = b.sample_windows(data, 5000, out_dtype=dt)
        assert sa.dtype == dt and torch.equal(sa, sb[:100])
        # recover each sample's window index from its first two values, then compare whole windows
        ref = data.to(dt).float().reshape(300, -1)[:, :2]
        idx = (sb.float().reshape(5000, 1, -1)[:, :, :2] - ref[None]).abs().sum(-1).argmin(-1)
        assert torch.equal(sb, data.to(dt)[idx])


def test_optimizers_match_cpu(cuda):
    from hfrep.train.optim import KerasOptimizer

    for kind in ("rmsprop", "adam", "nadam"):
        g = torch.Generator().manual_seed(10)
        p0 = torch.randn(1003, generator=g)
        grads = [torch.randn(1003, generator=g) for _ in range(4)]
        pc, pg = p0.clone(), p0.clone().to(cuda)
        oc = KerasOptimizer(kind, 1e-2)
        og = KerasOptimizer(kind, 1e-2, device=cuda)
        for gr in grads:
            oc.apply(pc, gr.clone(), clip=0.5 if kind == "rmsprop" else 0.0)
            og.apply(pg, gr.clone().to(cuda), clip=0.5 if kind == "rmsprop" else 0.0)
        torch.testing.assert_close(pg.cpu(), pc, rtol=1e-5, atol=1e-6)
        assert og.iterations.item() == 4


@pytest.mark.parametrize("key,T,F,lrelu", [(("lstm", "wgan_gp"), 24, 32, False), (("mlp", "wgan_gp"), 24, 32, False),
                                           (("lstm", "wgan"), 24, 32, False), (("mlp", "gan"), 24, 32, False),
                                           (("lstm", "gan"), 24, 32, False), (("conv", "wgan_gp"), 24, 32, False),
                                           (("lstm_ln", "wgan_gp"), 24, 32, False),
                                           (("lstm", "wgan_gp"), 168, 36, True)])
def test_trainer_gradients_gpu_vs_cpu(cuda, key, T, F, lrelu):
    """The full explicit critic/generator gradient programs on GPU (native fp32 kernels) vs CPU fp64,
    incl. the production generator shape (T = 168, F = 36, LeakyReLU after the first LSTM)."""
    from hfrep.train.gan_trainer import GANConfig, GANTrainer

    B = 48
    ds = np.random.RandomState(0).rand(64, T, F).astype(np.float32)
    kw = dict(arch=key[0], loss=key[1], window=T, features=F, batch_size=B, lrelu_after_first=lrelu)
    cfg_g = GANConfig(dtype="float32", **kw)
    cfg_c = GANConfig(dtype="float64", **kw)
    tg = GANTrainer(cfg_g, ds, device=cuda)
    tc = GANTrainer(cfg_c, ds, param_dtype=torch.float64)
    with torch.no_grad():
        tc.generator.flat.copy_(tg.generator.flat.double().cpu())
        tc.critic.flat.copy_(tg.critic.flat.double().cpu())
    g = torch.Generator().manual_seed(11)
    real = torch.rand(B, T, F, generator=g)
    noise = torch.randn(B, T, F, generator=g)
    alpha = torch.rand(B, generator=g)
    with torch.no_grad():
        if key[1] == "wgan_gp":
            fg = tg.generator.predict(noise.to(cuda))
            fc = tc.generator.predict(noise.double())
            _close(fg, fc, torch.float32)
            tg.critic_gp_grads(real.to(cuda), fg, alpha.to(cuda))
            tc.critic_gp_grads(real.double(), fg.double().cpu(), alpha.double())
            gg, gc = tg.critic.flat.grad.cpu().double(), tc.critic.flat.grad
            rel = (gg - gc).norm() / gc.norm()
            assert rel < 2e-4, f"critic grad rel err {rel:.2e}"
        lg = tg.generator_grads(noise.to(cuda))
        lc = tc.generator_grads(noise.double())
        gg, gc = tg.generator.flat.grad.cpu().double(), tc.generator.flat.grad
        rel = (gg - gc).norm() / max(gc.norm(), 1e-30)
        assert rel < 2e-4, f"generator grad rel err {rel:.2e}"
        assert abs(lg.item() - lc.item()) < 1e-4 * max(1, abs(lc.item()))


@pytest.mark.parametrize("act", [2, 1, 0])
@pytest.mark.parametrize("B,T,K", [(70, 24, 32), (33, 12, 100), (64, 7, 35)])
def test_lstm2_fused_layer(cuda, act, B, T, K):
    """v2 fused bf16 kernels (input projection in-kernel, blocked tapes) vs the fp64 reference."""
    from hfrep.ops import functional as Fn

    H = 100
    g = torch.Generator().manual_seed(20)
    x = (torch.randn(B, T, K, generator=g) * 0.5).to(torch.bfloat16)
    W = torch.randn(K, 4 * H, generator=g) * (1.0 / K ** 0.5)
    b = torch.randn(4 * H, generator=g) * 0.1
    U = torch.randn(H, 4 * H, generator=g) * (1.0 / H ** 0.5)
    hs, tape = Fn.lstm_layer_fwd(x.to(cuda), W.to(cuda), b.to(cuda), U.to(cuda), act, True)
    assert isinstance(tape, torch.Tensor), "bf16 H=100 must take the fused v2 path"
    zx = x.double() @ W.double() + b.double()
    rh, rg, rc = R.lstm_seq_fwd(zx, U.double(), act)
    _close(hs, rh, torch.bfloat16)
    dH = torch.randn(B, T, H, generator=g).to(torch.bfloat16)
    dZ = Fn.lstm_layer_bwd(dH.to(cuda), tape, U.to(cuda), act)
    rdz = R.lstm_seq_bwd(dH.double(), rg, rc, U.double(), act)
    _close(dZ, rdz, torch.bfloat16)
    # fused input gradient: dX = dZ W^T from the same launch (K <= 128)
    dZ1, dX = Fn.lstm_layer_bwd(dH.to(cuda), tape, U.to(cuda), act, W=W.to(cuda))
    assert torch.equal(dZ1, dZ)
    _close(dX, rdz @ W.double().t(), torch.bfloat16, scale=(rdz.abs() @ W.double().abs().t()).max().item())
    xd = (torch.randn(B, T, K, generator=g) * 0.3).to(torch.bfloat16)
    hds, ttape = Fn.lstm_layer_tfwd(xd.to(cuda), W.to(cuda), tape, U.to(cuda), act)
    th, tz, tc = R.lstm_seq_tfwd(xd.double() @ W.double(), rg, rc, U.double(), act)
    _close(hds, th, torch.bfloat16)
    dHd = torch.randn(B, T, H, generator=g).to(torch.bfloat16)
    for with_dh in (True, False):
        dZ2, dZd2 = Fn.lstm_layer_tbwd(dH.to(cuda) if with_dh else None, dHd.to(cuda), tape, ttape, U.to(cuda), act)
        rz, rzd = R.lstm_seq_tbwd(dH.double() if with_dh else torch.zeros(B, T, H, dtype=torch.float64),
                                  dHd.double(), rg, rc, tz, tc, U.double(), act)
        _close(dZ2, rz, torch.bfloat16)
        _close(dZd2, rzd, torch.bfloat16)
        dZ3, dZd3, dX3, dXd3 = Fn.lstm_layer_tbwd(dH.to(cuda) if with_dh else None, dHd.to(cuda), tape, ttape,
                                                  U.to(cuda), act, W=W.to(cuda))
        # the DX instantiation may contract the gate math differently (1-ulp bf16 differences
        # that the recurrence carries back in time): compare both variants to the reference
        _close(dZ3, rz, torch.bfloat16)
        _close(dZd3, rzd, torch.bfloat16)
        Wd = W.double()
        _close(dX3, rz @ Wd.t(), torch.bfloat16, scale=(rz.abs() @ Wd.abs().t()).max().item())
        _close(dXd3, rzd @ Wd.t(), torch.bfloat16, scale=(rzd.abs() @ Wd.abs().t()).max().item())


def _block_errors(model_g, model_c):
    """(global relative L2 error, worst per-parameter-block relative L2 error, block name) of the
    flat gradients of two copies of one model (every Keras weight is its own block, so an error in
    one layer cannot be averaged away by the others)."""
    a_all, b_all = model_g.flat.grad.cpu().double(), model_c.flat.grad.double().cpu()
    # a block whose exact gradient vanishes (the critic head bias under the Wasserstein terms:
    # sum of -1/B over real + 1/B over fake = 0) is measured against 1e-3 of the whole gradient
    floor = 1e-3 * b_all.norm().item()
    worst, wname = 0.0, ""
    for (name, _), (_, _) in zip(model_g.named_weights(), model_c.named_weights()):
        lay = [l for l in model_g.layers for s_ in l.specs if s_.keras == name][0]
        spec = [s_ for s_ in lay.specs if s_.keras == name][0]
        n = int(np.prod(spec.shape))
        a, b = a_all[spec.offset:spec.offset + n], b_all[spec.offset:spec.offset + n]
        rel = ((a - b).norm() / max(b.norm().item(), floor, 1e-30)).item()
        if rel > worst:
            worst, wname = rel, name
    return ((a_all - b_all).norm() / max(b_all.norm().item(), 1e-30)).item(), worst, wname


# bf16 bounds.  Measured on MI355X (r02, profiles/r02_tests/bf16_errors.txt): global 2.7e-3 .. 5.9e-3,
# worst block 4.0e-3 .. 2.3e-2 (the generator's first LSTM kernel at T = 168).  The compute is bf16
# MFMA with bf16 activations / tapes against an fp64 reference of the same inputs, so ~1e-2 is the
# bf16 noise floor; a stale or wrong row tile moves these by O(0.1 .. 1)
BF16_GLOBAL, BF16_BLOCK = 1.5e-2, 5e-2


@pytest.mark.parametrize("key,T,F,B,lrelu", [(("lstm", "wgan_gp"), 24, 32, 64, False), (("lstm", "wgan"), 24, 32, 64, False),
                                             (("lstm", "wgan_gp"), 24, 32, 256 * 32 + 70, False),
                                             (("lstm", "wgan_gp"), 168, 36, 40, True),
                                             (("lstm_ln", "wgan_gp"), 24, 32, 64, False)])
def test_trainer_gradients_bf16_fused(cuda, key, T, F, B, lrelu):
    """bf16 training step (fused LSTM kernels) vs the fp64 CPU engine: norm-relative error of the
    whole gradient and of every parameter block.  Cases: the bench shape at small B, a multi-pass
    batch (more 32-row tiles than CUs + a partial tile), and the production generator shape
    (T = 168, F = 36, LeakyReLU after the first LSTM)."""
    from hfrep.train.gan_trainer import GANConfig, GANTrainer

    ds = np.random.RandomState(0).rand(64, T, F).astype(np.float32)
    kw = dict(arch=key[0], loss=key[1], window=T, features=F, batch_size=B, lrelu_after_first=lrelu)
    tg = GANTrainer(GANConfig(dtype="bfloat16", **kw), ds, device=cuda)
    tc = GANTrainer(GANConfig(dtype="float64", **kw), ds, param_dtype=torch.float64)
    with torch.no_grad():
        tc.generator.flat.copy_(tg.generator.flat.double().cpu())
        tc.critic.flat.copy_(tg.critic.flat.double().cpu())
    g = torch.Generator().manual_seed(12)
    real = torch.rand(B, T, F, generator=g)
    noise = torch.randn(B, T, F, generator=g)
    alpha = torch.rand(B, generator=g)
    with torch.no_grad():
        if key[1] == "wgan_gp":
            fg = tg.generator.predict(noise.to(cuda, torch.bfloat16))
            tg.critic_gp_grads(real.to(cuda, torch.bfloat16), fg, alpha.to(cuda))
            tc.critic_gp_grads(real.to(torch.bfloat16).double(), fg.double().cpu(), alpha.double())
            rel, worst, name = _block_errors(tg.critic, tc.critic)
            print(f"critic bf16 rel {rel:.3e} worst block {worst:.3e} ({name})")
            assert rel < BF16_GLOBAL and worst < BF16_BLOCK, (rel, worst, name)
        tg.generator_grads(noise.to(cuda, torch.bfloat16))
        tc.generator_grads(noise.to(torch.bfloat16).double())
        rel, worst, name = _block_errors(tg.generator, tc.generator)
        print(f"generator bf16 rel {rel:.3e} worst block {worst:.3e} ({name})")
        assert rel < BF16_GLOBAL and worst < BF16_BLOCK, (rel, worst, name)


@pytest.mark.parametrize("impl", [0, 2])
@pytest.mark.parametrize("B,T,K,tangent", [(70, 24, 32, False), (33, 24, 100, True), (200, 12, 35, True), (5, 3, 100, False),
                                           (1000, 24, 32, True), (2051, 24, 100, True), (4096, 24, 100, False)])
def test_lstm_wgrad_fused(cuda, B, T, K, tangent, impl):
    """One-launch LSTM weight gradients vs fp64 products: impl 0 = LDS-DMA streaming kernel
    (wgrad3.hip) where the shape allows it, impl 2 = the tr-read tile kernel (gemm2.hip)."""
    from hfrep.ops import functional as Fn

    H, N = 100, 400
    g = torch.Generator().manual_seed(30)
    bf = lambda *s: torch.randn(*s, generator=g).to(torch.bfloat16)
    x, hs, dZ = bf(B, T, K), bf(B, T, H), bf(B, T, N)
    xd, hds, dZd = bf(B, T, K), bf(B, T, H), bf(B, T, N)
    gW0, gU0, gb0 = torch.randn(K, N, generator=g), torch.randn(H, N, generator=g), torch.randn(N, generator=g)
    gW, gU, gb = gW0.clone().to(cuda), gU0.clone().to(cuda), gb0.clone().to(cuda)
    Fn.lstm_wgrad_(x.to(cuda), hs.to(cuda), dZ.to(cuda), gW, gU, gb, *(
        (xd.to(cuda), hds.to(cuda), dZd.to(cuda)) if tangent else (None, None, None)), impl=impl)
    d = lambda t: t.double().reshape(-1, t.shape[-1])
    rW = gW0.double() + d(x).t() @ d(dZ)
    rU = gU0.double() + d(R.shift_prev(hs.double())).t() @ d(dZ)
    rb = gb0.double() + d(dZ).sum(0)
    if tangent:
        rW += d(xd).t() @ d(dZd)
        rU += d(R.shift_prev(hds.double())).t() @ d(dZd)
    sc = lambda a, b: (d(a).abs().t() @ d(b).abs()).max().item() * (2 if tangent else 1)
    _close(gW, rW, torch.bfloat16, scale=sc(x, dZ))
    _close(gU, rU, torch.bfloat16, scale=sc(hs, dZ))
    _close(gb, rb, torch.bfloat16, scale=d(dZ).abs().sum(0).max().item())
    # tight check against fp32 accumulation of the same bf16 inputs (the kernel's exact math)
    err = (gW.cpu().double() - rW).abs().max().item()
    assert err < 1e-3 * sc(x, dZ), err


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,K,N", [(37, 2400, 1), (1000, 2400, 1), (513, 64, 3), (70, 8, 4), (4099, 800, 2),
                                   (70001, 2400, 1)])
def test_skinny_dense_ops(cuda, dt, M, K, N):
    """Flatten -> Dense(N <= 4) head kernels (csrc/skinny.hip, bf16 and fp32): forward, input grad,
    weight+bias grad vs fp64 products of the same inputs."""
    from hfrep.ops import functional as Fn

    g = torch.Generator().manual_seed(40)
    x = torch.randn(M, K, generator=g).to(dt)
    W = torch.randn(K, N, generator=g) * K ** -0.5
    b = torch.randn(N, generator=g)
    y = Fn.linear(x.to(cuda), W.to(cuda), b.to(cuda), 0)
    ry = x.double() @ W.double() + b.double()
    _close(y, ry, dt, scale=(x.double().abs() @ W.double().abs()).max().item())
    d = torch.randn(M, N, generator=g).to(dt)
    dx = Fn.linear_dgrad(d.to(cuda), W.to(cuda))
    _close(dx, d.double() @ W.double().t(), dt)
    gW0, gb0 = torch.randn(K, N, generator=g), torch.randn(N, generator=g)
    gW, gb = gW0.clone().to(cuda), gb0.clone().to(cuda)
    Fn.linear_wgrad_(x.to(cuda), d.to(cuda), gW, gb)
    rW = gW0.double() + x.double().t() @ d.double()
    rb = gb0.double() + d.double().sum(0)
    tol = 1e-3 if dt == torch.bfloat16 else 2e-5
    assert (gW.cpu().double() - rW).abs().max().item() < tol * max(1.0, (x.double().abs().t() @ d.double().abs()).max().item())
    assert (gb.cpu().double() - rb).abs().max().item() < tol * max(1.0, d.double().abs().sum(0).max().item())


@pytest.mark.parametrize("B,D", [(7, 768), (16384, 768), (33, 100), (40000, 768), (5, 1680), (9, 102)])
def test_gp_coef_many_rows(cuda, B, D):
    """Vector path (D % 4 == 0, D <= 1024; B = 40 000 takes several grid-stride rounds) and the scalar
    two-pass path (D = 1680: the T = 48, F = 35 preset; D = 102) against fp64."""
    from hfrep.ops import functional as Fn

    g = torch.Generator().manual_seed(41)
    x = (torch.randn(B, D, generator=g) * 0.05).to(torch.bfloat16)
    pen, v = Fn.gp_coef(x.to(cuda), 10.0)
    xd = x.double()
    nrm = xd.norm(dim=1)
    rpen = ((1 - nrm) ** 2).mean()
    rv = -(2 * 10.0 / B) * ((1 - nrm) / nrm)[:, None] * xd
    assert abs(pen.item() - rpen.item()) < 1e-3 * max(1.0, rpen.item())
    _close(v, rv, torch.bfloat16)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,T,C,k,dil", [(3, 24, 32, 3, 1), (5, 17, 100, 3, 2), (2, 5, 7, 4, 3)])
def test_conv1d_im2col_col2im(cuda, dt, B, T, C, k, dil):
    """Native causal im2col / col2im (csrc/misc.hip) vs the PyTorch formulation; col2im is the
    adjoint of im2col: <im2col(x), y> == <x, col2im(y)>."""
    from hfrep.ops import functional as Fn

    g = torch.Generator().manual_seed(50)
    x = torch.randn(B, T, C, generator=g).to(dt)
    y = torch.randn(B, T, k * C, generator=g).to(dt)
    cols = Fn.im2col_causal(x.to(cuda), k, dil).cpu()
    ref = Fn.im2col_causal(x, k, dil)
    assert torch.equal(cols, ref)
    dx = Fn.col2im_causal(y.to(cuda), k, dil, C).cpu()
    rdx = Fn.col2im_causal(y.double(), k, dil, C)
    _close(dx, rdx, dt, scale=k * y.double().abs().max().item())
    lhs = (ref.double() * y.double()).sum()
    rhs = (x.double() * rdx).sum()
    assert abs(lhs - rhs) < 1e-6 * max(1.0, abs(lhs.item()))


def test_conv_critic_trains_native(cuda):
    """conv WGAN-GP variant (K14): a bf16 training iteration on the GPU runs and stays finite."""
    from hfrep.train.gan_trainer import GANConfig, GANTrainer

    ds = np.random.RandomState(0).rand(256, 24, 32).astype(np.float32)
    tr = GANTrainer(GANConfig(arch="conv", loss="wgan_gp", window=24, features=32, batch_size=128, dtype="bfloat16"),
                    ds, device=cuda)
    for _ in range(2):
        tr.train_step()
    rec = tr.losses()
    assert all(np.isfinite(v) for k, v in rec.items() if k != "iteration")


def test_lstm2_bwd_dx_only(cuda):
    """need_dz=False (gradient-penalty input gradient): same dX, no dZ written."""
    from hfrep.ops import functional as Fn

    B, T, K, H = 40, 12, 32, 100
    g = torch.Generator().manual_seed(60)
    x = (torch.randn(B, T, K, generator=g) * 0.5).to(torch.bfloat16).to(cuda)
    W = (torch.randn(K, 4 * H, generator=g) * K ** -0.5).to(cuda)
    U = (torch.randn(H, 4 * H, generator=g) * H ** -0.5).to(cuda)
    b = torch.zeros(4 * H, device=cuda)
    _, tape = Fn.lstm_layer_fwd(x, W, b, U, 2, True)
    dH = torch.randn(B, T, H, generator=g).to(torch.bfloat16).to(cuda)
    dZ, dX = Fn.lstm_layer_bwd(dH, tape, U, 2, W=W)
    dZ2, dX2 = Fn.lstm_layer_bwd(dH, tape, U, 2, W=W, need_dz=False)
    assert dZ2 is None and torch.equal(dX, dX2)


def test_lstm2_persistent_multi_pass(cuda):
    """Persistent v2 kernels when every workgroup walks several row blocks (B > 2 * 32 * CUs) and
    the last block is partial: buffer-descriptor range checks replace the per-row branches."""
    from hfrep.ops import functional as Fn

    H, T, K, act = 100, 3, 32, 2
    B = 2 * 32 * 2 * torch.cuda.get_device_properties(0).multi_processor_count + 37
    g = torch.Generator().manual_seed(61)
    x = (torch.randn(B, T, K, generator=g) * 0.5).to(torch.bfloat16)
    W = torch.randn(K, 4 * H, generator=g) * K ** -0.5
    b = torch.randn(4 * H, generator=g) * 0.1
    U = torch.randn(H, 4 * H, generator=g) * H ** -0.5
    hs, tape = Fn.lstm_layer_fwd(x.to(cuda), W.to(cuda), b.to(cuda), U.to(cuda), act, True)
    rh, rg, rc = R.lstm_seq_fwd(x.double() @ W.double() + b.double(), U.double(), act)
    _close(hs, rh, torch.bfloat16)
    dH = torch.randn(B, T, H, generator=g).to(torch.bfloat16)
    dZ, dX = Fn.lstm_layer_bwd(dH.to(cuda), tape, U.to(cuda), act, W=W.to(cuda))
    rdz = R.lstm_seq_bwd(dH.double(), rg, rc, U.double(), act)
    _close(dZ, rdz, torch.bfloat16)
    _close(dX, rdz @ W.double().t(), torch.bfloat16, scale=(rdz.abs() @ W.double().abs().t()).max().item())
    xd = (torch.randn(B, T, K, generator=g) * 0.3).to(torch.bfloat16)
    hds, ttape = Fn.lstm_layer_tfwd(xd.to(cuda), W.to(cuda), tape, U.to(cuda), act)
    th, tz, tc = R.lstm_seq_tfwd(xd.double() @ W.double(), rg, rc, U.double(), act)
    _close(hds, th, torch.bfloat16)
    dHd = torch.randn(B, T, H, generator=g).to(torch.bfloat16)
    dZ2, dZd2, dX2, dXd2 = Fn.lstm_layer_tbwd(dH.to(cuda), dHd.to(cuda), tape, ttape, U.to(cuda), act, W=W.to(cuda))
    rz, rzd = R.lstm_seq_tbwd(dH.double(), dHd.double(), rg, rc, tz, tc, U.double(), act)
    _close(dZ2, rz, torch.bfloat16)
    _close(dZd2, rzd, torch.bfloat16)
    _close(dXd2, rzd @ W.double().t(), torch.bfloat16, scale=(rzd.abs() @ W.double().abs().t()).max().item())


def test_lstm2_head_adjoint_in_kernel(cuda):
    """Flatten -> Dense(1) head adjoint generated inside the reverse kernels == the materialised
    outer product (bitwise: same bf16 rounding as the skinny dgrad kernel)."""
    from hfrep.ops import functional as Fn

    H, T, K, act = 100, 24, 100, 2
    B = 97
    g = torch.Generator().manual_seed(62)
    x = (torch.randn(B, T, K, generator=g) * 0.5).to(torch.bfloat16).to(cuda)
    W = (torch.randn(K, 4 * H, generator=g) * K ** -0.5).to(cuda)
    U = (torch.randn(H, 4 * H, generator=g) * H ** -0.5).to(cuda)
    b = torch.zeros(4 * H, device=cuda)
    _, tape = Fn.lstm_layer_fwd(x, W, b, U, act, True)
    xd = (torch.randn(B, T, K, generator=g) * 0.3).to(torch.bfloat16).to(cuda)
    _, ttape = Fn.lstm_layer_tfwd(xd, W, tape, U, act)
    w = (torch.randn(T * H, 1, generator=g) * 0.05).to(cuda)
    d = torch.randn(B, 1, generator=g).to(torch.bfloat16).to(cuda)
    dd = torch.randn(B, 1, generator=g).to(torch.bfloat16).to(cuda)
    oa, oad = Fn.OuterAdjoint(d, w, (B, T, H)), Fn.OuterAdjoint(dd, w, (B, T, H))
    dHm, dHdm = oa.materialize(), oad.materialize()
    assert torch.equal(dHm, Fn.linear_dgrad(d, w).reshape(B, T, H))
    for Wx in (None, W):
        r1 = Fn.lstm_layer_bwd(oa, tape, U, act, W=Wx)
        r2 = Fn.lstm_layer_bwd(dHm, tape, U, act, W=Wx)
        for a, c in zip(r1 if Wx is not None else (r1,), r2 if Wx is not None else (r2,)):
            assert torch.equal(a, c)
        for seeds, mats in (((None, oad), (None, dHdm)), ((oa, oad), (dHm, dHdm))):
            t1 = Fn.lstm_layer_tbwd(seeds[0], seeds[1], tape, ttape, U, act, W=Wx)
            t2 = Fn.lstm_layer_tbwd(mats[0], mats[1], tape, ttape, U, act, W=Wx)
            # run-to-run bitwise (the generated-adjoint DX instantiation was not in r01-r02: stale
            # accumulator reads from the cross-opcode MFMA SrcC hazard, profiles/r03_race)
            t1b = Fn.lstm_layer_tbwd(seeds[0], seeds[1], tape, ttape, U, act, W=Wx)
            assert all(torch.equal(a, c) for a, c in zip(t1, t1b))
            # (the GEN and tensor-fed instantiations may contract the gate math differently: 1-ulp
            # bf16 differences that the recurrence carries back, so compare at bf16 tolerance)
            for a, c in zip(t1, t2):
                _close(a, c.double(), torch.bfloat16)
    # the native op with W and the head runs the DX + generated-head instantiation (shipped since the
    # r03 SrcC fix): bitwise the tensor-fed launch here, and run to run
    ops = _ops()
    o1 = ops.lstm2_tbwd(None, None, tape, ttape, U, act, W, d, dd, w.reshape(-1))
    o2 = ops.lstm2_tbwd(dHm, dHdm, tape, ttape, U, act, W)
    assert all(torch.equal(a, c) for a, c in zip(o1, o2))
    o3 = ops.lstm2_tbwd(None, None, tape, ttape, U, act, W, d, dd, w.reshape(-1))
    assert all(torch.equal(a, c) for a, c in zip(o1, o3))


@pytest.mark.parametrize("act", [1, 2])
def test_lstm2_tbwd_bitwise_large_batch(cuda, act):
    """The bf16 tangent reverse run twice on ONE pair of tapes at B = 32 772 is bitwise equal, with a
    tensor-fed adjoint and with the generated head adjoint + fused dX.  Before the r03 fix of the
    cross-opcode MFMA SrcC hazard (a 16x16x16 tail chained onto a 16x16x32 accumulator 1-4 wait states
    after it) act = sigmoid differed in ~2e5 dZ elements per run, rows 4 g + {0, 1} of a 32-row block
    (profiles/r03_race/README.md)."""
    from hfrep.ops import functional as Fn

    H, T, K, B = 100, 24, 32, 32772
    g = torch.Generator(device=cuda).manual_seed(0)
    mk = lambda *s_, sc=0.5: (torch.randn(*s_, device=cuda, generator=g) * sc).to(torch.bfloat16)
    x, xd, dH = mk(B, T, K), mk(B, T, K), mk(B, T, H)
    W = torch.randn(K, 4 * H, device=cuda, generator=g) * 0.1
    U = torch.randn(H, 4 * H, device=cuda, generator=g) * 0.1
    b = torch.randn(4 * H, device=cuda, generator=g) * 0.1
    _, tape = Fn.lstm_layer_fwd(x, W, b, U, act, True)
    _, ttape = Fn.lstm_layer_tfwd(xd, W, tape, U, act)
    z0 = Fn.lstm_layer_tbwd(dH, dH, tape, ttape, U, act)
    for _ in range(2):
        z1 = Fn.lstm_layer_tbwd(dH, dH, tape, ttape, U, act)
        assert all(torch.equal(a, c) for a, c in zip(z0, z1))
    oa = Fn.OuterAdjoint(mk(B, 1), torch.randn(T * H, 1, device=cuda, generator=g) * 0.1, (B, T, H))
    y0 = Fn.lstm_layer_tbwd(oa, oa, tape, ttape, U, act, W=W)
    y1 = Fn.lstm_layer_tbwd(oa, oa, tape, ttape, U, act, W=W)
    assert all(torch.equal(a, c) for a, c in zip(y0, y1))


@pytest.mark.parametrize("act", [0, 1, 2])  # 0: the MTSS-WGAN linear critic
@pytest.mark.parametrize("K", [32, 100])
def test_lstm2_bwd_bitwise_large_batch(cuda, act, K):
    """The bf16 BPTT (lstm_tbwd4 with its tangent stream compiled out, round 5) run three times at
    B = 32 772 on one tape is bitwise equal: dZ alone, dZ + fused dX, and dX from the generated head
    adjoint (the paths of the critic's W-terms backward, GP input gradient and generator step)."""
    from hfrep.ops import functional as Fn

    H, T, B = 100, 24, 32772
    g = torch.Generator(device=cuda).manual_seed(2)
    mk = lambda *s_, sc=0.5: (torch.randn(*s_, device=cuda, generator=g) * sc).to(torch.bfloat16)
    x, dH = mk(B, T, K), mk(B, T, H)
    W = torch.randn(K, 4 * H, device=cuda, generator=g) * 0.1
    U = torch.randn(H, 4 * H, device=cuda, generator=g) * 0.1
    b = torch.randn(4 * H, device=cuda, generator=g) * 0.1
    _, tape = Fn.lstm_layer_fwd(x, W, b, U, act, True)
    oa = Fn.OuterAdjoint(mk(B, 1), torch.randn(T * H, 1, device=cuda, generator=g) * 0.1, (B, T, H))
    runs = []
    for _ in range(3):
        z = Fn.lstm_layer_bwd(dH, tape, U, act)
        zx = Fn.lstm_layer_bwd(dH, tape, U, act, W=W, need_dz=True)
        gx = Fn.lstm_layer_bwd(oa, tape, U, act, W=W, need_dz=False)
        runs.append([z, *zx, *(gx if isinstance(gx, tuple) else (gx,))])
    for r in runs[1:]:
        assert all(a is None and c is None or torch.equal(a, c) for a, c in zip(runs[0], r))
    assert torch.isfinite(runs[0][0].float()).all() and runs[0][0].abs().max() > 0


@pytest.mark.parametrize("act", [1, 2])
@pytest.mark.parametrize("K", [32, 100])
def test_lstm2_tfwd_bitwise_large_batch(cuda, act, K):
    """The bf16 tangent forward (hdot and the tangent tape) run three times at B = 32 772 on one primal
    tape is bitwise equal (act = sigmoid differed run to run in rows 30 / 31 of a few row blocks with
    lstm_fwd4_kernel<TAN> in r03, profiles/r03_race/README.md)."""
    from hfrep.ops import functional as Fn

    H, T, B = 100, 24, 32772
    g = torch.Generator(device=cuda).manual_seed(1)
    mk = lambda *s_, sc=0.5: (torch.randn(*s_, device=cuda, generator=g) * sc).to(torch.bfloat16)
    x, xd = mk(B, T, K), mk(B, T, K)
    W = torch.randn(K, 4 * H, device=cuda, generator=g) * 0.1
    U = torch.randn(H, 4 * H, device=cuda, generator=g) * 0.1
    b = torch.randn(4 * H, device=cuda, generator=g) * 0.1
    _, tape = Fn.lstm_layer_fwd(x, W, b, U, act, True)
    dH = mk(B, T, H)
    # (the tangent tape's padded-unit slots are never written: compare what reads it, the tangent reverse)
    h0, t0 = Fn.lstm_layer_tfwd(xd, W, tape, U, act)
    z0 = Fn.lstm_layer_tbwd(dH, dH, tape, t0, U, act)
    for _ in range(2):
        h1, t1 = Fn.lstm_layer_tfwd(xd, W, tape, U, act)
        assert torch.equal(h0, h1), "tangent forward hdot not bitwise run to run"
        z1 = Fn.lstm_layer_tbwd(dH, dH, tape, t1, U, act)
        assert all(torch.equal(a, c) for a, c in zip(z0, z1)), "tangent tape not bitwise run to run"


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("n,split", [(64, 32), (70 * 24, 35 * 24), (1 << 20, 1 << 19), (1000, 1000)])
def test_gan_loss_native(cuda, dt, kind, n, split):
    """Native loss value + gradient (csrc/misc.hip gan_loss_kernel) vs the fp32 reference contract,
    and bitwise run-to-run."""
    from hfrep.ops import functional as Fn

    g = torch.Generator().manual_seed(n + kind)
    p = torch.rand(n, 1, generator=g) if kind == 1 else torch.randn(n, 1, generator=g)
    if kind == 1:
        p[:3] = torch.tensor([[0.0], [1.0], [1e-9]])  # clip boundaries
    p = p.to(dt)
    la, lb = (-1.0, 1.0) if kind == 0 else (1.0, 0.0)
    out, grad = Fn.gan_loss(p.to(cuda), split, la, lb, kind)
    rout, rgrad = R.gan_loss(p, split, la, lb, kind)
    assert torch.allclose(out.cpu(), rout, rtol=1e-5, atol=1e-6), (out, rout)
    _close(grad, rgrad.double(), dt)
    out2, grad2 = Fn.gan_loss(p.to(cuda), split, la, lb, kind)
    assert torch.equal(out, out2) and torch.equal(grad, grad2)


@pytest.mark.parametrize("act", [2, 1, 0])
@pytest.mark.parametrize("B,T,K", [(70, 24, 32), (33, 12, 100), (64, 7, 35), (40, 5, 36)])
def test_lstmf_fused_layer(cuda, act, B, T, K):
    """fp32 fused kernels (csrc/lstm_f32.hip: exact-f32 16x16x4 MFMA, gate-interleaved tiles + quad
    transpose, lane-native blocked tapes) vs the fp64 reference: forward, BPTT (+ input gradient),
    tangent forward and tangent reverse, each bitwise reproducible run to run."""
    from hfrep.ops import functional as Fn

    H = 100
    g = torch.Generator().manual_seed(21)
    x = torch.randn(B, T, K, generator=g) * 0.5
    W = torch.randn(K, 4 * H, generator=g) * (1.0 / K ** 0.5)
    b = torch.randn(4 * H, generator=g) * 0.1
    U = torch.randn(H, 4 * H, generator=g) * (1.0 / H ** 0.5)
    assert _ops().lstmf_supported(H, K, act)
    dev = lambda *ts: [t_.to(cuda) for t_ in ts]  # noqa: E731
    xg, Wg, bg, Ug = dev(x, W, b, U)
    hs, tape = Fn.lstm_layer_fwd(xg, Wg, bg, Ug, act, True)
    assert isinstance(tape, Fn.FTape)
    zx = x.double() @ W.double() + b.double()
    rh, rg, rc = R.lstm_seq_fwd(zx, U.double(), act)
    f32 = torch.float32
    _close(hs, rh, f32)
    hs0, none = Fn.lstm_layer_fwd(xg, Wg, bg, Ug, act, False)
    assert none is None and torch.equal(hs0, hs)
    # BPTT (+ dX through the input-gradient GEMM)
    dH = torch.randn(B, T, H, generator=g)
    dZ, dX = Fn.lstm_layer_bwd(dH.to(cuda), tape, Ug, act, W=Wg)
    rdz = R.lstm_seq_bwd(dH.double(), rg, rc, U.double(), act)
    _close(dZ, rdz, f32)
    _close(dX, rdz @ W.double().t(), f32, scale=(rdz.abs() @ W.double().abs().t()).max().item())
    # tangent forward + tangent reverse (with and without the primal adjoint)
    xd = torch.randn(B, T, K, generator=g) * 0.3
    hds, ttape = Fn.lstm_layer_tfwd(xd.to(cuda), Wg, tape, Ug, act)
    th, tz, tc = R.lstm_seq_tfwd(xd.double() @ W.double(), rg, rc, U.double(), act)
    _close(hds, th, f32)
    dHd = torch.randn(B, T, H, generator=g)
    for with_dh in (True, False):
        dZ2, dZd2, dX2, dXd2 = Fn.lstm_layer_tbwd(dH.to(cuda) if with_dh else None, dHd.to(cuda), tape, ttape, Ug, act,
                                                  W=Wg)
        rz, rzd = R.lstm_seq_tbwd(dH.double() if with_dh else torch.zeros(B, T, H, dtype=torch.float64),
                                  dHd.double(), rg, rc, tz, tc, U.double(), act)
        _close(dZ2, rz, f32)
        _close(dZd2, rzd, f32)
        Wd = W.double()
        _close(dXd2, rzd @ Wd.t(), f32, scale=(rzd.abs() @ Wd.abs().t()).max().item())
    # bitwise run-to-run reproducibility
    # (the tapes' padding slots are never written, so the tapes are compared through their readers)
    hs2, tape2 = Fn.lstm_layer_fwd(xg, Wg, bg, Ug, act, True)
    hds2, ttape2 = Fn.lstm_layer_tfwd(xd.to(cuda), Wg, tape2, Ug, act)
    assert torch.equal(hs, hs2) and torch.equal(hds, hds2)
    assert torch.equal(dZ, Fn.lstm_layer_bwd(dH.to(cuda), tape2, Ug, act))
    dZ3, dZd3 = Fn.lstm_layer_tbwd(None, dHd.to(cuda), tape2, ttape2, Ug, act)
    assert torch.equal(dZ3, dZ2) and torch.equal(dZd3, dZd2)


def test_lstmf_persistent_multi_pass(cuda):
    """More row tiles than CUs (every persistent workgroup walks several tiles) and a partial last
    tile: B = 256 * 32 + 45 rows (the 16-row tangent reverse walks twice as many)."""
    from hfrep.ops import functional as Fn

    H, K, T, B = 100, 32, 6, 256 * 32 + 45
    g = torch.Generator().manual_seed(22)
    x = torch.randn(B, T, K, generator=g) * 0.5
    W = torch.randn(K, 4 * H, generator=g) * (1.0 / K ** 0.5)
    b = torch.randn(4 * H, generator=g) * 0.1
    U = torch.randn(H, 4 * H, generator=g) * (1.0 / H ** 0.5)
    hs, tape = Fn.lstm_layer_fwd(x.to(cuda), W.to(cuda), b.to(cuda), U.to(cuda), 2, True)
    rh, rg, rc = R.lstm_seq_fwd(x.double() @ W.double() + b.double(), U.double(), 2)
    _close(hs, rh, torch.float32)
    dH = torch.randn(B, T, H, generator=g) * 0.3
    dZ = Fn.lstm_layer_bwd(dH.to(cuda), tape, U.to(cuda), 2)
    _close(dZ, R.lstm_seq_bwd(dH.double(), rg, rc, U.double(), 2), torch.float32)
    xd = torch.randn(B, T, K, generator=g) * 0.3
    hds, ttape = Fn.lstm_layer_tfwd(xd.to(cuda), W.to(cuda), tape, U.to(cuda), 2)
    th, tz, tc = R.lstm_seq_tfwd(xd.double() @ W.double(), rg, rc, U.double(), 2)
    _close(hds, th, torch.float32)
    dHd = torch.randn(B, T, H, generator=g)
    dZ2, dZd2 = Fn.lstm_layer_tbwd(dH.to(cuda), dHd.to(cuda), tape, ttape, U.to(cuda), 2)
    rz, rzd = R.lstm_seq_tbwd(dH.double(), dHd.double(), rg, rc, tz, tc, U.double(), 2)
    _close(dZ2, rz, torch.float32)
    _close(dZd2, rzd, torch.float32)


@pytest.mark.parametrize("B,T,K,tangent", [(70, 24, 32, False), (33, 12, 100, True), (1000, 24, 100, False),
                                           (41, 5, 36, True), (32, 48, 35, True), (65, 48, 35, False)])
def test_lstmf_wgrad_fused(cuda, B, T, K, tangent):
    """fp32 fused LSTM weight gradient (one launch for every product) vs fp64."""
    from hfrep.ops import functional as Fn

    H, N = 100, 400
    g = torch.Generator().manual_seed(23)
    x, hs, dz = torch.randn(B, T, K, generator=g), torch.randn(B, T, H, generator=g), torch.randn(B, T, N, generator=g)
    xd, hds, dzd = (torch.randn(B, T, K, generator=g), torch.randn(B, T, H, generator=g),
                    torch.randn(B, T, N, generator=g)) if tangent else (None, None, None)
    gW0, gU0, gb0 = torch.randn(K, N, generator=g), torch.randn(H, N, generator=g), torch.randn(N, generator=g)
    gW, gU, gb = gW0.clone().to(cuda), gU0.clone().to(cuda), gb0.clone().to(cuda)
    dev = lambda t: None if t is None else t.to(cuda)  # noqa: E731
    Fn.lstm_wgrad_(dev(x), dev(hs), dev(dz), gW, gU, gb, dev(xd), dev(hds), dev(dzd))
    X, Hp, D = x.double().reshape(-1, K), R.shift_prev(hs.double()).reshape(-1, H), dz.double().reshape(-1, N)
    rW, rU, rb = gW0.double() + X.t() @ D, gU0.double() + Hp.t() @ D, gb0.double() + D.sum(0)
    sW, sU = (X.abs().t() @ D.abs()).max().item(), (Hp.abs().t() @ D.abs()).max().item()
    if tangent:
        Xd, Hdp, Dd = xd.double().reshape(-1, K), R.shift_prev(hds.double()).reshape(-1, H), dzd.double().reshape(-1, N)
        rW, rU = rW + Xd.t() @ Dd, rU + Hdp.t() @ Dd
        sW, sU = sW + (Xd.abs().t() @ Dd.abs()).max().item(), sU + (Hdp.abs().t() @ Dd.abs()).max().item()
    _close(gW, rW, torch.float32, scale=sW)
    _close(gU, rU, torch.float32, scale=sU)
    _close(gb, rb, torch.float32, scale=D.abs().sum(0).max().item())


@pytest.mark.parametrize("B,T,K,tangent", [(1, 5, 100, False), (70, 24, 32, False), (33, 12, 100, True),
                                           (41, 5, 36, True), (1000, 24, 100, True), (4500, 24, 32, False),
                                           (20000, 24, 100, True), (41, 5, 35, True), (3001, 24, 35, False)])
def test_lstmf_wgrad_split_vs_exact(cuda, B, T, K, tangent):
    """The three-term bf16 split weight gradients (impl 2 pair, 3 quad) and the exact-fp32
    MFMA kernel (impl 1) vs fp64: all inside the fp32 tolerance and the splits' error within 2x the exact
    kernel's (the dropped split terms are <= 2^-24 of each product); bitwise run-to-run.  K = 35: the
    reference's 35-feature rows read in place (dword loads, a 36-column image; impl 3 falls back to 2)."""
    from hfrep.ops import functional as Fn

    H, N = 100, 400
    g = torch.Generator().manual_seed(37)
    t = lambda *s: torch.randn(*s, generator=g).to(cuda)  # noqa: E731
    x, hs, dz = t(B, T, K), t(B, T, H), t(B, T, N)
    xd, hds, dzd = (t(B, T, K), t(B, T, H), t(B, T, N)) if tangent else (None, None, None)
    X, Hp, Dm = x.double().reshape(-1, K), R.shift_prev(hs.double()).reshape(-1, H), dz.double().reshape(-1, N)
    rW, rU, rb = X.t() @ Dm, Hp.t() @ Dm, Dm.sum(0)
    if tangent:
        rW = rW + xd.double().reshape(-1, K).t() @ dzd.double().reshape(-1, N)
        rU = rU + R.shift_prev(hds.double()).reshape(-1, H).t() @ dzd.double().reshape(-1, N)
    errs = {}
    for impl in (1, 2, 2, 3, 3):
        gW, gU, gb = torch.zeros(K, N, device=cuda), torch.zeros(H, N, device=cuda), torch.zeros(N, device=cuda)
        Fn.lstm_wgrad_(x, hs, dz, gW, gU, gb, xd, hds, dzd, impl=impl)
        out = torch.cat([gW.reshape(-1), gU.reshape(-1), gb])
        if impl in errs:
            assert torch.equal(out, errs[impl][1]), "split wgrad not bitwise run-to-run"
            continue
        ref = torch.cat([rW.reshape(-1), rU.reshape(-1), rb])
        errs[impl] = ((out.double() - ref).abs().max().item(), out)
    refmax = max(rW.abs().max().item(), rU.abs().max().item(), rb.abs().max().item())
    e1, e2, e3 = errs[1][0], errs[2][0], errs[3][0]
    print(f"max abs err exact {e1:.3e} split {e2:.3e} quad {e3:.3e} (max |ref| {refmax:.3e})")
    assert e1 <= 1e-5 * refmax + 1e-5 and e2 <= 2 * e1 + 1e-6 * refmax, (e1, e2, refmax)
    assert e3 <= 2 * e1 + 1e-6 * refmax, (e1, e3, refmax)


@pytest.mark.parametrize("K,tangent", [(100, False), (32, True)])
def test_lstmf_wgrad_large_m(cuda, K, tangent):
    """fp32 fused weight gradient past 4 GiB of dZ (M = 3 M rows: a whole-tensor buffer descriptor
    wrapped its 32-bit size there and read zeros for the later rows) vs an fp64 GPU reference."""
    from hfrep.ops import functional as Fn

    B, T, H, N = 120000, 25, 100, 400
    g = torch.Generator(device=cuda).manual_seed(31)
    rn = lambda *s: torch.randn(*s, device=cuda, generator=g)  # noqa: E731
    x, hs, dz = rn(B, T, K), rn(B, T, H), rn(B, T, N)
    xd, hds, dzd = (rn(B, T, K), rn(B, T, H), rn(B, T, N)) if tangent else (None, None, None)
    rW = torch.zeros(K, N, dtype=torch.float64, device=cuda)
    rU = torch.zeros(H, N, dtype=torch.float64, device=cuda)
    for xx, hh, dd in ((x, hs, dz), (xd, hds, dzd)) if tangent else ((x, hs, dz),):
        D = dd.double().reshape(-1, N)
        rW += xx.double().reshape(-1, K).t() @ D
        rU += R.shift_prev(hh.double()).reshape(-1, H).t() @ D
    rb = dz.double().reshape(-1, N).sum(0)
    # random-sign sums of 3 M products: scale by the root-sum-square, not the absolute sum
    tol = 2e-5 * (B * T) ** 0.5 * (2 if tangent else 1)
    for impl in (1, 2, 3):
        gW, gU, gb = (torch.zeros(K, N, device=cuda), torch.zeros(H, N, device=cuda), torch.zeros(N, device=cuda))
        Fn.lstm_wgrad_(x, hs, dz, gW, gU, gb, xd, hds, dzd, impl=impl)
        for got, ref in ((gW, rW), (gU, rU), (gb, rb)):
            err = (got.double() - ref).abs().max().item()
            print(f"impl {impl}: max abs err {err:.3e} (tol {tol:.3e})")
            assert err < tol, (impl, err, tol)


@pytest.mark.parametrize("M,KO", [(1, 100), (17, 32), (1000, 100), (4099, 36), (20000, 100), (333, 7), (100000, 112)])
def test_lstmf_dgrad(cuda, M, KO):
    """fp32 LSTM input gradient dZ W^T, the exact-fp32 kernel and the three-term bf16 split kernel,
    vs fp64, bitwise run-to-run, including partial row chunks and column tiles."""
    from hfrep.ops import _native

    g = torch.Generator().manual_seed(29)
    dz, W = torch.randn(M, 400, generator=g), torch.randn(KO, 400, generator=g) * 0.1
    ref = dz.double() @ W.double().t()
    scale = (dz.abs().double() @ W.abs().double().t()).max().item()
    errs = {}
    for impl in (1, 3):  # exact-fp32 MFMA kernel, LDS-staged three-term bf16 split kernel
        out = _native.native().lstmf_dgrad(dz.to(cuda), W.to(cuda), impl)
        _close(out, ref, torch.float32, scale=scale)
        again = _native.native().lstmf_dgrad(dz.to(cuda), W.to(cuda), impl)
        assert torch.equal(out, again)
        errs[impl] = (out.double().cpu() - ref).abs().max().item()
    # the split's dropped terms are <= 2^-24 of each product: within 2x the exact kernel's error
    assert errs[3] <= 2 * errs[1] + 1e-6 * scale, errs


def test_gan_eval_device_path(cuda):
    """GANEval(..., device='cuda'): FID covariances through the native wgrad kernel and the MMD
    sample means on the GPU agree with the fp64 CPU reference path."""
    from hfrep.eval.gan_eval import GANEval

    rs = np.random.RandomState(3)
    real, fake = rs.rand(4000, 24, 32), rs.rand(4000, 24, 32) * 0.9 + 0.05
    cpu = GANEval(real, fake, real, ["f"], ["m"])
    gpu = GANEval(real, fake, real, ["f"], ["m"], device=cuda)
    for name in ("FID", "linear_MMD", "gaussian_MMD", "poly_MMD"):
        a, b = getattr(gpu, name)(), getattr(cpu, name)()
        assert abs(a - b) <= 1e-4 * max(abs(b), 1e-3), (name, a, b)


def _block_rel(model, a, b):
    """{keras weight name: relative L2 error} of two flat gradients of ``model``."""
    out = {}
    for lay in model.layers:
        for sp in lay.specs:
            n = int(np.prod(sp.shape))
            x, y = a[sp.offset:sp.offset + n], b[sp.offset:sp.offset + n]
            out[sp.keras] = ((x - y).norm() / max(y.norm().item(), 1e-30)).item()
    return out


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("B,T,F,lrelu", [(16384, 24, 32, False), (262144, 24, 32, False), (32768, 168, 36, True)])
def test_bench_scale_gradients_are_slice_averages(cuda, dtype, B, T, F, lrelu):
    """At the bench batch (B = 262,144: dZ of the critic's W terms is 20 GB) the critic GP and the
    generator gradients equal the average of the gradients of four row slices: every row's
    contribution is computed identically, only the reduction order differs.  Catches any kernel
    whose addressing breaks past 2 / 4 GiB (the fp32 weight gradient did, before r02).  Also at the
    production generator shape (T = 168, F = 36, LeakyReLU after LSTM1: dZ 17.6 GB at 32k windows)."""
    from hfrep.train.gan_trainer import GANConfig, GANTrainer

    S = 4
    ds = np.random.RandomState(0).rand(64, T, F).astype(np.float32)
    tr = GANTrainer(GANConfig(arch="lstm", loss="wgan_gp", window=T, features=F, batch_size=B, dtype=dtype,
                              lrelu_after_first=lrelu), ds, device=cuda)
    dt = torch.float32 if dtype == "float32" else torch.bfloat16
    g = torch.Generator(device=cuda).manual_seed(41)
    real = torch.rand(B, T, F, device=cuda, generator=g).to(dt)
    noise = torch.randn(B, T, F, device=cuda, generator=g).to(dt)
    alpha = torch.rand(B, device=cuda, generator=g)
    tol = 1e-4 if dtype == "float32" else 1e-3
    sl = lambda t, i: t[i * (B // S):(i + 1) * (B // S)].contiguous()  # noqa: E731

    def grads(model, fn, *args):
        if model.flat.grad is not None:
            model.flat.grad.zero_()
        fn(*args)
        torch.cuda.synchronize()
        return model.flat.grad.double().clone()

    with torch.no_grad():
        fake = tr.generator.predict(noise)
        full = grads(tr.critic, tr.critic_gp_grads, real, fake, alpha)
        # run-to-run bitwise at the full batch (the store-data hazard made reruns differ at 2 x 262k rows)
        assert torch.equal(full, grads(tr.critic, tr.critic_gp_grads, real, fake, alpha)), "critic rerun differs"
        avg = sum(grads(tr.critic, tr.critic_gp_grads, sl(real, i), sl(fake, i), sl(alpha, i)) for i in range(S)) / S
        rel = ((full - avg).norm() / avg.norm()).item()
        assert torch.isfinite(full).all() and rel < tol, (f"critic: full-batch vs slice-average rel {rel:.2e}",
                                                          _block_rel(tr.critic, full, avg))
        full = grads(tr.generator, tr.generator_grads, noise)
        avg = sum(grads(tr.generator, tr.generator_grads, sl(noise, i)) for i in range(S)) / S
        rel = ((full - avg).norm() / avg.norm()).item()
        assert torch.isfinite(full).all() and rel < tol, (f"generator: full-batch vs slice-average rel {rel:.2e}",
                                                          _block_rel(tr.generator, full, avg))


@pytest.mark.parametrize("M,K,N,act", [(6291456 + 5, 100, 32, 0), (1000, 36, 36, 1), (333, 64, 112, 2),
                                       (77, 128, 5, 3), (4099, 32, 100, 0)])
def test_narrowf_linear(cuda, M, K, N, act):
    """Exact-fp32 narrow GEMM (csrc/skinny.hip narrowf_kernel) on the Dense forward: the generator's
    Dense(32) at the bench's 6.3 M rows (B = 262144 x T = 24) and every K / partial-tile case; fp64
    reference computed on the device; bitwise run-to-run."""
    assert _ops().narrowf_supported(K, N)
    g = torch.Generator(device=cuda).manual_seed(41)
    x = torch.randn(M, K, generator=g, device=cuda)
    W = torch.randn(K, N, generator=g, device=cuda) * (1.0 / K ** 0.5)
    b = torch.randn(N, generator=g, device=cuda) * 0.1
    y = _ops().linear(x, W, b, act)
    ref = R.apply_act(x.double() @ W.double() + b.double(), act)
    err = (y.double() - ref).abs().max().item()
    scale = max(ref.abs().max().item(), 1e-3)
    assert err <= TOL[torch.float32]["atol"] * max(1.0, scale) + TOL[torch.float32]["rtol"] * scale, (err, scale)
    assert torch.equal(y, _ops().linear(x, W, b, act))
    del x, y, ref


@pytest.mark.parametrize("M,K,N", [(6291456 + 3, 32, 100), (513, 36, 100), (70, 100, 32)])
def test_narrowf_dgrad(cuda, M, K, N):
    """dz W^T on the narrow fp32 kernel (the generator's Dense(32) input gradient at 6.3 M rows)."""
    assert _ops().narrowf_supported(K, N)
    g = torch.Generator(device=cuda).manual_seed(43)
    dz = torch.randn(M, K, generator=g, device=cuda)
    W = torch.randn(N, K, generator=g, device=cuda) * 0.1
    dx = _ops().linear_dgrad(dz, W)
    ref = dz.double() @ W.double().t()
    err = (dx.double() - ref).abs().max().item()
    scale = max(ref.abs().max().item(), 1e-3)
    assert err <= TOL[torch.float32]["atol"] * max(1.0, scale) + TOL[torch.float32]["rtol"] * scale, (err, scale)
    assert torch.equal(dx, _ops().linear_dgrad(dz, W))


@pytest.mark.parametrize("act", [2, 1, 0])
@pytest.mark.parametrize("B,T,K", [(70, 24, 32), (8192 + 45, 6, 32), (64, 7, 35), (40, 5, 36)])
def test_lstmf_split_forward_vs_exact(cuda, act, B, T, K):
    """The split-recurrent forward (lstmf_fwds_kernel: h_{t-1} U as the exact three-term bf16 split on
    v_mfma_f32_16x16x32_bf16 for k < 96, fp32 for the tail) vs the exact-fp32 forward and fp64: primal and tangent forward within 2x the exact kernel's error (+ fp32
    noise), bitwise run to run."""
    from hfrep.ops import functional as Fn

    H = 100
    g = torch.Generator().manual_seed(57)
    x = torch.randn(B, T, K, generator=g) * 0.5
    W = torch.randn(K, 4 * H, generator=g) * (1.0 / K ** 0.5)
    b = torch.randn(4 * H, generator=g) * 0.1
    U = torch.randn(H, 4 * H, generator=g) * (1.0 / H ** 0.5)
    xd = torch.randn(B, T, K, generator=g) * 0.3
    xg, Wg, bg, Ug, xdg = (t_.to(cuda) for t_ in (x, W, b, U, xd))
    zx = x.double() @ W.double() + b.double()
    rh, rg, rc = R.lstm_seq_fwd(zx, U.double(), act)
    th, _, _ = R.lstm_seq_tfwd(xd.double() @ W.double(), rg, rc, U.double(), act)
    ops = _ops()
    out, errs = {}, {}
    prev = ops.set_lstmf_fwd_impl(1)
    try:
        for impl in (1, 2, 2):
            ops.set_lstmf_fwd_impl(impl)
            hs, tape = Fn.lstm_layer_fwd(xg, Wg, bg, Ug, act, True)
            hs0, _ = Fn.lstm_layer_fwd(xg, Wg, bg, Ug, act, False)
            hds, _ = Fn.lstm_layer_tfwd(xdg, Wg, tape, Ug, act)
            if impl in out:
                assert all(torch.equal(a_, b_) for a_, b_ in zip(out[impl], (hs, hs0, hds))), "not bitwise"
                continue
            out[impl] = (hs, hs0, hds)
            errs[impl] = ((hs.double().cpu() - rh).abs().max().item(), (hs0.double().cpu() - rh).abs().max().item(),
                          (hds.double().cpu() - th).abs().max().item())
    finally:
        ops.set_lstmf_fwd_impl(prev)
    print(f"max abs err exact {errs[1]} split {errs[2]}")
    for e1, e2 in zip(errs[1], errs[2]):
        assert e2 <= 2 * e1 + 2e-6, (errs[1], errs[2])


@pytest.mark.parametrize("B,T", [(70, 24), (8192 + 45, 6)])
def test_lstmf_head_adjoint_in_kernel(cuda, B, T):
    """fp32: the critic head's adjoint dH = d (x) w generated inside lstmf_bwds / lstmf_tbwdp (HEAD
    instantiations) vs the materialised dH (skinny dgrad + the plain kernels), for the BPTT (split impl 3;
    the exact impl 2 materialises in the binding: bitwise) and the tangent reverse with a primal head
    seed, a tangent one, or both.  The in-kernel product may contract into its consumer's add (one
    rounding fewer), so the two agree to fp32 rounding and both are checked against fp64."""
    from hfrep.ops import functional as Fn

    H, K, act = 100, 100, 2
    g = torch.Generator().manual_seed(71)
    x, xd = torch.randn(B, T, K, generator=g) * 0.5, torch.randn(B, T, K, generator=g) * 0.5
    W = torch.randn(K, 4 * H, generator=g) * (1.0 / K ** 0.5)
    b = torch.randn(4 * H, generator=g) * 0.1
    U = torch.randn(H, 4 * H, generator=g) * (1.0 / H ** 0.5)
    d1, d2 = torch.randn(B, 1, generator=g), torch.randn(B, 1, generator=g)
    w = torch.randn(T * H, 1, generator=g)
    xg, xdg, Wg, bg, Ug, d1g, d2g, wg = (t_.to(cuda) for t_ in (x, xd, W, b, U, d1, d2, w))
    o1, o2 = Fn.OuterAdjoint(d1g, wg, (B, T, H)), Fn.OuterAdjoint(d2g, wg, (B, T, H))
    m1, m2 = o1.materialize(), o2.materialize()
    # fp64 reference of the BPTT with the exact outer-product adjoint
    zx = x.double() @ W.double() + b.double()
    _, rg, rc = R.lstm_seq_fwd(zx, U.double(), act)
    rdz = R.lstm_seq_bwd((d1.double() * w.double().reshape(1, -1)).reshape(B, T, H), rg, rc, U.double(), act)

    def close(a, c, what):
        scale = c.abs().max().item()
        assert (a - c).abs().max().item() <= 1e-5 * scale, what

    ops = _ops()
    pb = ops.set_lstmf_bwd_impl(3)
    try:
        _, tape = Fn.lstm_layer_fwd(xg, Wg, bg, Ug, act, True)
        for impl in (3, 2):
            ops.set_lstmf_bwd_impl(impl)
            a, c = Fn.lstm_layer_bwd(o1, tape, Ug, act), Fn.lstm_layer_bwd(m1, tape, Ug, act)
            if impl == 2:
                assert torch.equal(a, c)
            else:
                close(a, c, "bwd")
                ea = (a.double().cpu() - rdz).abs().max().item()
                ec = (c.double().cpu() - rdz).abs().max().item()
                assert ea <= 1.05 * ec + 1e-7, (ea, ec)
            assert torch.equal(a, Fn.lstm_layer_bwd(o1, tape, Ug, act))  # run to run
        ops.set_lstmf_bwd_impl(3)
        _, ttape = Fn.lstm_layer_tfwd(xdg, Wg, tape, Ug, act)
        for a, c in (((None, o2), (None, m2)), ((o1, None), (m1, None)), ((o1, o2), (m1, m2))):
            za, zad = Fn.lstm_layer_tbwd(a[0], a[1], tape, ttape, Ug, act)
            zc, zcd = Fn.lstm_layer_tbwd(c[0], c[1] if c[1] is not None else torch.zeros_like(m1), tape, ttape, Ug, act)
            close(za, zc, "tbwd dZ")
            close(zad, zcd, "tbwd dZd")
    finally:
        ops.set_lstmf_bwd_impl(pb)


@pytest.mark.parametrize("act", [2, 1, 0])
@pytest.mark.parametrize("B,T", [(70, 24), (8192 + 45, 6), (33, 1), (40, 5)])
def test_lstmf_split_bptt_vs_exact(cuda, act, B, T):
    """The split-recurrent BPTT (lstmf_bwds_kernel: dz_{t+1} U^T as the exact three-term bf16 split on
    v_mfma_f32_16x16x32_bf16) vs the exact-fp32 role-split BPTT (lstmf_bwdp_kernel) and fp64: dZ (and the
    fused dX) within 2x the exact kernel's error (+ fp32 noise), bitwise run to run; the tape comes from
    the exact forward so both kernels see the same input."""
    from hfrep.ops import functional as Fn

    H, K = 100, 32
    g = torch.Generator().manual_seed(61)
    x = torch.randn(B, T, K, generator=g) * 0.5
    W = torch.randn(K, 4 * H, generator=g) * (1.0 / K ** 0.5)
    b = torch.randn(4 * H, generator=g) * 0.1
    U = torch.randn(H, 4 * H, generator=g) * (1.0 / H ** 0.5)
    dH = torch.randn(B, T, H, generator=g)
    xg, Wg, bg, Ug, dHg = (t_.to(cuda) for t_ in (x, W, b, U, dH))
    zx = x.double() @ W.double() + b.double()
    _, rg, rc = R.lstm_seq_fwd(zx, U.double(), act)
    rdz = R.lstm_seq_bwd(dH.double(), rg, rc, U.double(), act)
    ops = _ops()
    pf = ops.set_lstmf_fwd_impl(1)
    pb = ops.set_lstmf_bwd_impl(2)
    out, errs = {}, {}
    try:
        _, tape = Fn.lstm_layer_fwd(xg, Wg, bg, Ug, act, True)
        for impl in (2, 3, 3):
            ops.set_lstmf_bwd_impl(impl)
            dZ = Fn.lstm_layer_bwd(dHg, tape, Ug, act)
            if impl in out:
                assert torch.equal(out[impl], dZ), "not bitwise"
                continue
            out[impl] = dZ
            errs[impl] = (dZ.double().cpu() - rdz).abs().max().item()
    finally:
        ops.set_lstmf_fwd_impl(pf)
        ops.set_lstmf_bwd_impl(pb)
    print(f"max abs err exact {errs[2]:.3e} split {errs[3]:.3e}")
    assert torch.isfinite(out[3]).all()
    assert errs[3] <= 2 * errs[2] + 2e-6, errs


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("B", [37, 3000])
def test_critic_head_wgrad_fused_in_forward(cuda, dtype, B, monkeypatch):
    """The W terms' critic head: with the loss gradient of every row known (-1/B real, +1/B fake) the
    head's weight gradient is accumulated by the head forward itself (skinny_fwd_cs_kernel: one pass over
    the layer-2 output instead of skinny_fwd + skinny_wgrad).  Against the unfused path on the same GP
    critic step: the loss pack is bitwise equal (same score arithmetic) and the critic gradient agrees to
    the fp32 summation order; two fused runs are bitwise equal."""
    import numpy as np

    from hfrep.ops import functional as Fn
    from hfrep.train.gan_trainer import GANConfig, GANTrainer

    T, F = 24, 32
    ds = np.random.RandomState(5).rand(64, T, F).astype(np.float32)
    tr = GANTrainer(GANConfig(arch="lstm", loss="wgan_gp", window=T, features=F, batch_size=B, dtype=dtype), ds,
                    device=cuda)
    g = torch.Generator().manual_seed(4)
    real = torch.rand(B, T, F, generator=g).to(cuda, tr.dtype)
    fake = torch.rand(B, T, F, generator=g).to(cuda, tr.dtype)
    alpha = torch.rand(B, generator=g).to(cuda)
    runs = []
    for fused in (True, True, False):
        if not fused:
            monkeypatch.setattr(Fn, "head_cs_ok", lambda x, W: False)
        tr.critic.zero_grad()
        with torch.no_grad():
            pack = tr.critic_gp_grads(real, fake, alpha)
        torch.cuda.synchronize()
        runs.append((pack.clone(), tr.critic.flat.grad.clone()))
    assert Fn.head_cs_ok is not None
    (p0, g0), (p1, g1), (p2, g2) = runs
    assert torch.equal(p0, p1) and torch.equal(g0, g1)
    assert torch.equal(p0, p2), (p0, p2)
    rel = ((g0 - g2).norm() / g2.norm()).item()
    assert rel < 1e-5, rel
