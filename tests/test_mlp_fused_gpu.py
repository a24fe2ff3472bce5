"""Fused MLP-GAN kernels (csrc/mlp.hip, train/mlp_fused.py) vs the CPU fp64 explicit engine.

BASELINE configs 3 / 4: the vanilla GAN (GAN/GAN.py) and the MLP WGAN-GP (GAN/WGAN_GP.py).  Every
fused pass is checked against the layer-by-layer fp64 reference of the same quantity: the generator
forward, the WGAN-GP critic gradient (W terms + reverse-over-tangent penalty), the GAN discriminator
gradient, the generator gradient through the frozen critic and the loss values; plus run-to-run
bitwise determinism and whole training steps against the GPU engine path (HFREP_MLP_FUSED=0).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = {"float32": 2e-4, "bfloat16": 3e-2}


def _rel(got, ref):
    got, ref = got.double().cpu(), ref.double().cpu()
    return ((got - ref).norm() / max(ref.norm().item(), 1e-30)).item()


def _pair(cuda, loss, dtype, B, T=24, F=32):
    from hfrep.train.gan_trainer import GANConfig, GANTrainer

    ds = np.random.RandomState(0).rand(64, T, F).astype(np.float32)
    kw = dict(arch="mlp", loss=loss, window=T, features=F, batch_size=B)
    tg = GANTrainer(GANConfig(dtype=dtype, **kw), ds, device=cuda)
    assert tg._fused is not None, "the fused MLP path must be selected on the GPU"
    tc = GANTrainer(GANConfig(dtype="float64", **kw), ds, param_dtype=torch.float64)
    with torch.no_grad():
        tc.generator.flat.copy_(tg.generator.flat.double().cpu())
        tc.critic.flat.copy_(tg.critic.flat.double().cpu())
    return tg, tc


def _inputs(B, T, F, seed=11):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(B, T, F, generator=g), torch.randn(B, T, F, generator=g), torch.rand(B, generator=g)


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("B,T,F", [(48, 24, 32), (37, 24, 32), (20, 48, 36)])
def test_mlp_wgan_gp_fused_grads(cuda, dtype, B, T, F):
    """Config 4: generator forward, the critic update's gradient and loss pack, and the generator
    gradient, fused kernels vs the fp64 engine (same weights, same batch)."""
    tg, tc = _pair(cuda, "wgan_gp", dtype, B, T, F)
    fz = tg._fused
    ops = torch.ops.hfrep
    dt = tg.dtype
    real, noise, alpha = _inputs(B, T, F)
    with torch.no_grad():
        fake = ops.mlp_gen_fwd(noise.to(cuda, dt), fz.gw)
        fc = tc.generator.predict(noise.double())
        assert _rel(fake, fc) < TOL[dtype], f"G(z) rel err {_rel(fake, fc):.2e}"
        pack_g = fz._wgp_critic_grads(real.to(cuda, dt), fake)
        pack_c = tc.critic_gp_grads(real.double(), fake.double().cpu(), alpha.double())
        rel = _rel(tg.critic.flat.grad, tc.critic.flat.grad)
        assert rel < TOL[dtype], f"critic grad rel err {rel:.2e}"
        lt = 1e-4 if dtype == "float32" else 2e-2
        for a, b in zip(pack_g.cpu().tolist(), pack_c.tolist()):
            assert abs(a - b) <= lt * max(1.0, abs(b)), (pack_g, pack_c)
        lg = fz._generator_grads(noise.to(cuda, dt), fake)
        lc = tc.generator_grads(noise.double())
        rel = _rel(tg.generator.flat.grad, tc.generator.flat.grad)
        assert rel < TOL[dtype], f"generator grad rel err {rel:.2e}"
        assert abs(lg.item() - lc.item()) <= lt * max(1.0, abs(lc.item()))


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("B", [48, 37])
def test_mlp_gan_fused_grads(cuda, dtype, B):
    """Config 3: the discriminator update on real (label 1) and fake (label 0) and the generator update
    (label 1 through the frozen discriminator), fused vs the fp64 engine."""
    from hfrep.ops import functional as Fn

    T, F = 24, 32
    tg, tc = _pair(cuda, "gan", dtype, B, T, F)
    fz = tg._fused
    dt = tg.dtype
    real, noise, _ = _inputs(B, T, F)
    lt = 1e-4 if dtype == "float32" else 2e-2
    with torch.no_grad():
        for x, label in ((real, 1.0), (torch.sigmoid(noise), 0.0)):
            tg.critic.zero_grad()
            tc.critic.zero_grad()
            lg = fz._gan_d_grads(x.to(cuda, dt), label)
            p, tape = tc.critic.efwd(x.double(), save=True)
            out, dp = Fn.gan_loss(p, p.numel(), label, label, 1)
            tc.critic.ebwd(tape, dp)
            rel = _rel(tg.critic.flat.grad, tc.critic.flat.grad)
            assert rel < TOL[dtype], f"D grad rel err {rel:.2e} (label {label})"
            assert abs(lg.item() - out[0].item()) <= lt * max(1.0, abs(out[0].item()))
        fake = torch.ops.hfrep.mlp_gen_fwd(noise.to(cuda, dt), fz.gw)
        lg = fz._generator_grads(noise.to(cuda, dt), fake)
        lc = tc.generator_grads(noise.double())
        rel = _rel(tg.generator.flat.grad, tc.generator.flat.grad)
        assert rel < TOL[dtype], f"generator grad rel err {rel:.2e}"
        assert abs(lg.item() - lc.item()) <= lt * max(1.0, abs(lc.item()))


@pytest.mark.parametrize("loss", ["wgan_gp", "gan"])
def test_mlp_fused_bitwise_and_engine_parity(cuda, loss, monkeypatch):
    """Three training iterations: two fused runs are bitwise identical (fixed-order reductions, no
    atomics); the fused run tracks the GPU engine path (HFREP_MLP_FUSED=0) on the same RNG stream."""
    from hfrep.train.gan_trainer import GANConfig, GANTrainer

    T, F, B = 24, 32, 96
    ds = np.random.RandomState(1).rand(256, T, F).astype(np.float32)
    cfg = GANConfig(arch="mlp", loss=loss, window=T, features=F, batch_size=B, dtype="float32")

    def run(fused):
        monkeypatch.setenv("HFREP_MLP_FUSED", "1" if fused else "0")
        tr = GANTrainer(cfg, ds, device=cuda)
        assert (tr._fused is not None) == fused
        for _ in range(3):
            tr.train_step()
        torch.cuda.synchronize()
        return tr

    a, b, e = run(True), run(True), run(False)
    assert torch.equal(a.critic.flat, b.critic.flat) and torch.equal(a.generator.flat, b.generator.flat)
    assert torch.equal(a._d_acc, b._d_acc) and torch.equal(a._g_acc, b._g_acc)
    for m in ("critic", "generator"):
        pa, pe = getattr(a, m).flat, getattr(e, m).flat
        assert _rel(pa, pe) < 1e-4, f"{m} params drift from the engine path: {_rel(pa, pe):.2e}"
    la, le = a.losses(), e.losses()
    for k in ("d_loss", "g_loss"):
        assert abs(la[k] - le[k]) <= 1e-3 * max(1.0, abs(le[k])), (la, le)


def test_mlp_fused_large_batch_slices(cuda):
    """At a batch spanning many persistent-grid rounds the fused critic gradient is the average of
    the gradients of its four quarter batches (bf16 and fp32)."""
    T, F = 24, 32
    for dtype in ("float32", "bfloat16"):
        B = 4 * 8192
        tg, _ = _pair(cuda, "wgan_gp", dtype, B, T, F)
        fz, dt = tg._fused, tg.dtype
        real, noise, _ = _inputs(B, T, F, seed=3)
        with torch.no_grad():
            fake = torch.ops.hfrep.mlp_gen_fwd(noise.to(cuda, dt), fz.gw)
            tg.critic.zero_grad()
            fz._wgp_critic_grads(real.to(cuda, dt), fake)
            full = tg.critic.flat.grad.clone()
            acc = torch.zeros_like(full)
            r = real.to(cuda, dt)
            for q in range(4):
                tg.critic.zero_grad()
                sl = slice(q * B // 4, (q + 1) * B // 4)
                fz._wgp_critic_grads(r[sl].contiguous(), fake[sl].contiguous())
                acc += tg.critic.flat.grad / 4
        rel = _rel(full, acc)
        assert rel < (1e-5 if dtype == "float32" else 2e-2), f"{dtype}: full vs slice-average rel {rel:.2e}"


@pytest.mark.parametrize("B,T,F", [(37, 24, 32), (300, 32, 32), (45, 16, 36), (6000, 24, 32)])
def test_mlp_wgp_inkernel_wgrad_matches_operand_path(cuda, B, T, F):
    """bf16 config 4: the GP critic update with the weight gradients accumulated in the kernel
    (mlp_wgp_critic_w: 128-row block tiles staged transposed in LDS, per-t tables for w3_t and
    W2 w3_t, one-hot MFMA for gw3) vs the operand path (mlp_wgp_critic + linear_wgrad_) on the same
    batch.  Both round the same operands to bf16 and differ only in the fp32 summation order; two
    in-kernel runs are bitwise identical.  Shapes: partial block tile, T = 32 (a full t tile), F = 36,
    and a batch that takes several grid rounds."""
    ops = torch.ops.hfrep
    assert not ops.mlp_wgpw_supported(36, 48) and not ops.mlp_wgpw_supported(32, 40)  # the LDS plan
    tg, _ = _pair(cuda, "wgan_gp", "bfloat16", B, T, F)
    fz, dt = tg._fused, tg.dtype
    assert fz.wgrad_tsum and not fz.wgrad_inkernel  # the t-major kernel is the default
    fz.affine = False  # the per-row kernels under test
    real, noise, _ = _inputs(B, T, F, seed=5)
    grads, packs = [], []
    with torch.no_grad():
        fake = ops.mlp_gen_fwd(noise.to(cuda, dt), fz.gw)
        r = real.to(cuda, dt)
        for inkernel in (True, True, False):
            fz.wgrad_inkernel, fz.wgrad_tsum = inkernel, False
            tg.critic.zero_grad()
            packs.append(fz._wgp_critic_grads(r, fake).clone())
            grads.append(tg.critic.flat.grad.clone())
    assert torch.equal(grads[0], grads[1]) and torch.equal(packs[0], packs[1])
    rel = _rel(grads[0], grads[2])
    assert rel < 1e-4, f"in-kernel vs operand-path critic gradient rel {rel:.2e}"
    torch.testing.assert_close(packs[0], packs[2], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("loss,B,T,F", [("wgan_gp", 37, 24, 32), ("gan", 300, 40, 32), ("wgan_gp", 45, 24, 36),
                                        ("gan", 6000, 24, 32)])
def test_mlp_gen_bwd_inkernel_matches_operand_path(cuda, loss, B, T, F):
    """bf16 configs 3 / 4: the generator reverse with its ten parameter gradients accumulated in the
    kernel (mlp_gen_bwd_w: u1 / u2 / dz1 / dz2 / dfake / noise staged transposed in LDS, bias gradients
    from a ones row of each X image) vs the operand path (mlp_gen_bwd + linear_wgrad_ + slab sums):
    same bf16 operands, different fp32 summation order; two in-kernel runs bitwise identical."""
    ops = torch.ops.hfrep
    tg, _ = _pair(cuda, loss, "bfloat16", B, T, F)
    fz, dt = tg._fused, tg.dtype
    assert fz.gen_wgrad_inkernel
    _, noise, _ = _inputs(B, T, F, seed=9)
    grads, losses = [], []
    with torch.no_grad():
        z = noise.to(cuda, dt)
        fake = ops.mlp_gen_fwd(z, fz.gw)
        for inkernel in (True, True, False):
            fz.gen_wgrad_inkernel = inkernel
            tg.generator.zero_grad()
            losses.append(fz._generator_grads(z, fake).clone())
            grads.append(tg.generator.flat.grad.clone())
    assert torch.equal(grads[0], grads[1]) and torch.equal(losses[0], losses[2])
    rel = _rel(grads[0], grads[2])
    assert rel < 1e-4, f"in-kernel vs operand-path generator gradient rel {rel:.2e}"
    # every parameter tensor is covered (a missed slab segment would show as a zero block)
    for (l, n), v in zip([(l, n) for l in tg.generator.layers for n in getattr(l, "param_names", [])], []):
        pass
    for a, b in zip(fz.gg, fz.gg):
        assert a.abs().sum() > 0


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("B,F", [(37, 32), (5000, 32), (45, 36)])
def test_mlp_gan_critic_colsum_matches_operand_path(cuda, dtype, B, F):
    """Config 3: the discriminator update with its gradients as dz-weighted column sums in the kernel
    (mlp_gan_critic_g) vs the operand path (mlp_gan_critic + linear_wgrad_), labels 1 and 0; two
    column-sum runs are bitwise identical."""
    T = 24
    tg, _ = _pair(cuda, "gan", dtype, B, T, F)
    fz, dt = tg._fused, tg.dtype
    assert fz.gan_colsum
    real, noise, _ = _inputs(B, T, F, seed=13)
    with torch.no_grad():
        for x, label in ((real, 1.0), (torch.sigmoid(noise), 0.0)):
            xg = x.to(cuda, dt)
            grads, losses = [], []
            for colsum in (True, True, False):
                fz.gan_colsum = colsum
                tg.critic.zero_grad()
                losses.append(fz._gan_d_grads(xg, label).clone())
                grads.append(tg.critic.flat.grad.clone())
            assert torch.equal(grads[0], grads[1]) and torch.equal(losses[0], losses[1])
            rel = _rel(grads[0], grads[2])
            assert rel < (1e-5 if dtype == "float32" else 5e-3), f"label {label}: column-sum vs operand rel {rel:.2e}"
            torch.testing.assert_close(losses[0], losses[2], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("B,T,F", [(37, 24, 32), (300, 40, 32), (45, 48, 36), (6000, 24, 32)])
def test_mlp_wgp_tsum_matches_operand_path(cuda, dtype, B, T, F):
    """Config 4: the GP critic update with rows walked t-major and the weight gradients as per-t column
    sums (mlp_wgp_critic_t: gW2 = sum_t S2[t] (x) w3_t, gW1 = sum_t S1[t] (x) W2 w3_t, gw3_t = S3[t]) vs
    the operand path on the same batch: the loss pack to fp32 rounding (the score sums run in another
    order), the gradient to the summation order (fp32) / the operand path's bf16 operand rounding (bf16);
    two runs bitwise identical."""
    tg, tc = _pair(cuda, "wgan_gp", dtype, B, T, F)
    fz, dt = tg._fused, tg.dtype
    fz.affine = False  # the per-row kernels under test
    real, noise, alpha = _inputs(B, T, F, seed=7)
    packs, grads = [], []
    with torch.no_grad():
        fake = torch.ops.hfrep.mlp_gen_fwd(noise.to(cuda, dt), fz.gw)
        r = real.to(cuda, dt)
        for mode in ("t", "t", "op"):
            fz.wgrad_inkernel, fz.wgrad_tsum = False, mode == "t"
            tg.critic.zero_grad()
            packs.append(fz._wgp_critic_grads(r, fake).clone())
            grads.append(tg.critic.flat.grad.clone())
        pack_c = tc.critic_gp_grads(real.double(), fake.double().cpu(), alpha.double())
        rel_c = _rel(grads[0], tc.critic.flat.grad)
    assert torch.equal(grads[0], grads[1]) and torch.equal(packs[0], packs[1])
    torch.testing.assert_close(packs[0], packs[2], rtol=1e-5, atol=1e-6)
    rel = _rel(grads[0], grads[2])
    assert rel < (1e-5 if dtype == "float32" else 3e-3), f"per-t sums vs operand path rel {rel:.2e}"
    assert rel_c < TOL[dtype], f"vs fp64 rel {rel_c:.2e}"


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("B,T,F", [(37, 24, 32), (300, 40, 32), (45, 48, 36), (6000, 24, 32), (40000, 24, 32)])
def test_mlp_wgp_affine_matches_per_row_path(cuda, dtype, B, T, F):
    """Config 4, the default critic path: the affine critic's update from per-t batch sums
    (mlp_wgp_affine: column sums of real and fake-real, one-workgroup fp32 finish) and the generator
    step's broadcast dfake (mlp_critic_dx_affine) vs the per-row kernels (mlp_wgp_critic_t /
    mlp_critic_dx) on the same batch and vs the fp64 engine: gradient, loss pack, dfake and the
    generator loss; two runs bitwise identical.  fp32: summation order only; bf16: the per-row kernels
    also round h1 / h2 to bf16 (the sums path does not), so vs the fp64 engine at the bf16 tolerance."""
    ops = torch.ops.hfrep
    tg, tc = _pair(cuda, "wgan_gp", dtype, B, T, F)
    fz, dt = tg._fused, tg.dtype
    assert fz.affine and ops.mlp_affine_supported(F, T) and not ops.mlp_affine_supported(36, 7)
    real, noise, alpha = _inputs(B, T, F, seed=13)
    packs, grads = [], []
    with torch.no_grad():
        fake = ops.mlp_gen_fwd(noise.to(cuda, dt), fz.gw)
        r = real.to(cuda, dt)
        for affine in (True, True, False):
            fz.affine = affine
            tg.critic.zero_grad()
            packs.append(fz._wgp_critic_grads(r, fake).clone())
            grads.append(tg.critic.flat.grad.clone())
        pack_c = tc.critic_gp_grads(real.double(), fake.double().cpu(), alpha.double())
        gd_a, sl_a = ops.mlp_critic_dx_affine(fake, fz.cw)
        gd_b, sl_b = ops.mlp_critic_dx_affine(fake, fz.cw)
        gd_r, sl_r = ops.mlp_critic_dx(fake, fz.cw, 0, -1.0)
        la = ops.mlp_finish(sl_a, None, 1, 1.0 / B, fz.cw[5], 0.0)[0]
        lr = ops.mlp_finish(sl_r, None, 1, 1.0 / B, fz.cw[5], 0.0)[0]
        fz.affine = True
    assert torch.equal(grads[0], grads[1]) and torch.equal(packs[0], packs[1])
    assert torch.equal(gd_a, gd_b) and torch.equal(sl_a, sl_b)
    rel_c = _rel(grads[0], tc.critic.flat.grad)
    assert rel_c < TOL[dtype], f"vs fp64 rel {rel_c:.2e}"
    rel = _rel(grads[0], grads[2])
    assert rel < (2e-5 if dtype == "float32" else TOL[dtype]), f"sums vs per-row path rel {rel:.2e}"
    lt = 1e-5 if dtype == "float32" else 2e-2
    for a, b, c in zip(packs[0].cpu().tolist(), packs[2].cpu().tolist(), pack_c.tolist()):
        assert abs(a - b) <= lt * max(1.0, abs(b)) and abs(a - c) <= 10 * lt * max(1.0, abs(c)), (packs, pack_c)
    # dfake: the same per-t row for every sample; the per-row kernel's value to its rounding
    assert torch.equal(gd_a, gd_a[:1].expand_as(gd_a))
    assert _rel(gd_a, gd_r) < (1e-5 if dtype == "float32" else 2e-2)
    assert abs(la.item() - lr.item()) <= lt * max(1.0, abs(lr.item()))
