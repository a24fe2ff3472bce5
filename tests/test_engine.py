"""Explicit differentiation engine vs the autograd oracle (fp64, CPU).

The trainers never build autograd graphs: gradients come from hand-derived reverse passes and,
for the WGAN-GP critic, a reverse-over-tangent Hessian-vector product.  These tests pin every
model of the zoo against ``torch.autograd`` (double backward for the gradient penalty, the
semantics of ``K.gradients`` in GAN/MTSS_WGAN_GP.py:205).
"""
import numpy as np
import pytest
import torch

from hfrep.models import gan as zoo
from hfrep.ops import reference as R
from hfrep.train.gan_trainer import GANConfig, GANTrainer

T, F, B = 6, 5, 4
KEYS = list(zoo.ZOO.keys())


def _trainer(arch, loss, **kw):
    cfg = GANConfig(arch=arch, loss=loss, window=T, features=F, batch_size=B, hidden=7, dtype="float64", **kw)
    ds = np.random.RandomState(0).rand(20, T, F)
    tr = GANTrainer(cfg, ds, param_dtype=torch.float64)
    # perturb biases/LN params so every code path is exercised with non-trivial values
    with torch.no_grad():
        for m in (tr.generator, tr.critic):
            m.flat.add_(0.05 * torch.randn(m.flat.shape, dtype=torch.float64, generator=torch.Generator().manual_seed(5)))
    return tr


def _inputs(seed=0):
    g = torch.Generator().manual_seed(seed)
    real = torch.rand(B, T, F, dtype=torch.float64, generator=g)
    noise = torch.randn(B, T, F, dtype=torch.float64, generator=g)
    alpha = torch.rand(B, dtype=torch.float64, generator=g)
    return real, noise, alpha


@pytest.mark.parametrize("key", [k for k in KEYS if zoo.ZOO[k].loss == "wgan_gp"])
def test_gp_critic_gradient_matches_double_backward(key):
    tr = _trainer(*key)
    C, G = tr.critic, tr.generator
    real, noise, alpha = _inputs()
    with torch.no_grad():
        fake = G.predict(noise)
    C.zero_grad()
    with torch.no_grad():
        losses = tr.critic_gp_grads(real, fake, alpha)
    explicit = C.flat.grad.clone()

    C.flat.grad = None
    xh = (alpha[:, None, None] * real + (1 - alpha[:, None, None]) * fake).requires_grad_(True)
    s_r, s_f = C(real), C(fake)
    s_h = C(xh)
    g, = torch.autograd.grad(s_h.sum(), xh, create_graph=True)
    gp = R.gradient_penalty_from_grad(g)
    L = -s_r.mean() + s_f.mean() + tr.gp_weight * gp
    oracle, = torch.autograd.grad(L, C.flat)
    C.flat.grad = torch.zeros_like(C.flat)
    torch.testing.assert_close(explicit, oracle, rtol=1e-9, atol=1e-11)
    assert abs(losses[0].item() - L.item()) < 1e-10


@pytest.mark.parametrize("key", KEYS)
def test_generator_gradient_matches_autograd(key):
    tr = _trainer(*key)
    C, G = tr.critic, tr.generator
    _, noise, _ = _inputs(1)
    G.zero_grad()
    with torch.no_grad():
        loss = tr.generator_grads(noise)
    explicit = G.flat.grad.clone()
    G.flat.grad = None
    s = C(G(noise))
    L = R.binary_crossentropy(torch.ones(B, 1, dtype=torch.float64), s) if key[1] == "gan" else -s.mean()
    oracle, = torch.autograd.grad(L, G.flat)
    G.flat.grad = torch.zeros_like(G.flat)
    C.flat.grad = torch.zeros_like(C.flat)
    torch.testing.assert_close(explicit, oracle, rtol=1e-9, atol=1e-11)
    assert abs(loss.item() - L.item()) < 1e-10


@pytest.mark.parametrize("key", [k for k in KEYS if zoo.ZOO[k].loss in ("gan", "wgan")])
def test_critic_first_order_gradient(key):
    tr = _trainer(*key)
    C = tr.critic
    real, _, _ = _inputs(2)
    for label in (1.0, 0.0) if key[1] == "gan" else (-1.0, 1.0):
        C.zero_grad()
        s, tape = C.efwd(real, save=True)
        if key[1] == "gan":
            o = s.clamp(R.KERAS_EPS, 1 - R.KERAS_EPS)
            inside = ((s > R.KERAS_EPS) & (s < 1 - R.KERAS_EPS)).double()
            ds = -(label / (o + R.KERAS_EPS) - (1 - label) / (1 - o + R.KERAS_EPS)) * inside / s.numel()
        else:
            ds = torch.full_like(s, label / s.numel())
        with torch.no_grad():
            C.ebwd(tape, ds)
        explicit = C.flat.grad.clone()
        C.flat.grad = None
        s2 = C(real)
        y = torch.full((B, 1), label, dtype=torch.float64)
        L = R.binary_crossentropy(y, s2) if key[1] == "gan" else R.wasserstein_loss(y, s2)
        oracle, = torch.autograd.grad(L, C.flat)
        C.flat.grad = torch.zeros_like(C.flat)
        torch.testing.assert_close(explicit, oracle, rtol=1e-9, atol=1e-11)


def test_param_counts_match_reference():
    # SURVEY §2.2 table, T=48, F=35
    expect = {("mlp", "gan"): (17635, 13801), ("mlp", "wgan"): (17635, 14201), ("mlp", "wgan_gp"): (17635, 18501),
              ("lstm", "gan"): (138735, 134901), ("lstm", "wgan"): (138735, 135301),
              ("lstm", "wgan_gp"): (138735, 139601)}
    for key, (g, c) in expect.items():
        e = zoo.ZOO[key]
        assert e.generator(48, 35).count_params() == g, key
        assert e.critic(48, 35).count_params() == c, key
    # production generator / north-star config
    assert zoo.lstm_generator(168, 36, lrelu_after_first=True).count_params() == 139236
    assert zoo.lstm_critic_gp(168, 36).count_params() == 152001
    assert zoo.lstm_generator(24, 32).count_params() == 137232
    assert zoo.lstm_critic_gp(24, 32).count_params() == 136001


def test_keras_init_semantics():
    m = zoo.lstm_critic_gp(8, 3, hidden=5)
    U = m.view(m.layers[0], "recurrent_kernel").double()
    # orthogonal (H, 4H): rows orthonormal
    torch.testing.assert_close(U @ U.t(), torch.eye(5, dtype=torch.float64), atol=1e-6, rtol=0)
    b = m.view(m.layers[0], "bias")
    assert torch.all(b[5:10] == 1) and torch.all(b[:5] == 0) and torch.all(b[10:] == 0)
    names = [n for n, _ in m.named_weights()]
    assert names[0].endswith("/kernel:0") and "lstm_cell" in names[1]


@pytest.mark.parametrize("kind", [0, 1])
def test_gan_loss_contract_matches_keras_losses(kind):
    """R.gan_loss (the native op's contract) = the Keras losses and their autograd gradients."""
    g = torch.Generator().manual_seed(5)
    B, T = 6, 4
    p = torch.rand(2 * B, T, 1, generator=g, dtype=torch.float64)
    p[0, 0, 0], p[1, 1, 0] = 0.0, 1.0  # clipped entries: zero BCE gradient
    la, lb = (-1.0, 1.0) if kind == 0 else (1.0, 0.0)
    out, grad = R.gan_loss(p, B * T, la, lb, kind, acc=torch.float64)
    q = p.clone().requires_grad_(True)
    f = R.wasserstein_loss if kind == 0 else R.binary_crossentropy
    ya = torch.full((B, T), la, dtype=torch.float64)
    yb = torch.full((B, T), lb, dtype=torch.float64)
    la_, lb_ = f(ya, q[:B]), f(yb, q[B:])
    (la_ + lb_).backward()
    assert torch.allclose(out, torch.stack([la_, lb_]).detach(), rtol=1e-12, atol=1e-12)
    assert torch.allclose(grad, q.grad, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("loss", ["wgan_gp", "wgan"])
def test_generator_forward_reuse_is_exact(loss):
    """The generator step reuses the last critic step's G(noise) forward and tape (same noise, and the
    critic updates leave G untouched): bitwise the same training as recomputing it."""
    import numpy as np

    from hfrep.train.gan_trainer import GANConfig, GANTrainer

    ds = np.random.RandomState(0).rand(40, 6, 4)
    runs = []
    for reuse in (True, False):
        cfg = GANConfig(arch="lstm", loss=loss, window=6, features=4, batch_size=5, hidden=8, dtype="float64")
        tr = GANTrainer(cfg, ds, param_dtype=torch.float64)
        tr.reuse_gen_forward = reuse
        for _ in range(3):
            tr.train_step()
        runs.append(torch.cat([tr.generator.flat.detach(), tr.critic.flat.detach(), tr._g_acc.reshape(-1)]))
    assert torch.equal(runs[0], runs[1])


def test_head_out_false_skips_only_dead_work():
    """The gradient penalty's forward on x_hat and its tangent forward never read the linear head's
    value: with head_out=False the head is not evaluated (shape-only placeholder) and the input
    gradient and the reverse-over-tangent parameter gradient are bitwise the same."""
    import numpy as np

    from hfrep.train.gan_trainer import GANConfig, GANTrainer

    ds = np.random.RandomState(3).rand(20, 8, 4).astype(np.float32)
    tr = GANTrainer(GANConfig(arch="lstm", loss="wgan_gp", window=8, features=4, batch_size=6, hidden=8), ds)
    C = tr.critic
    x = torch.randn(6, 8, 4, generator=torch.Generator().manual_seed(1))
    s1, t1 = C.efwd(x, save=True)
    s2, t2 = C.efwd(x, save=True, head_out=False)
    assert s2.shape == s1.shape and s2.dtype == s1.dtype
    g1 = C.ebwd(t1, torch.ones_like(s1), need_dx=True, wgrad=False)
    g2 = C.ebwd(t2, torch.ones_like(s2), need_dx=True, wgrad=False)
    assert torch.equal(g1, g2)
    v = torch.randn_like(x)
    sd1, tt1 = C.etfwd(t1, v)
    sd2, tt2 = C.etfwd(t2, v, head_out=False)
    assert sd2.shape == sd1.shape
    C.zero_grad()
    C.etbwd(t1, tt1, None, torch.ones_like(sd1))
    ga = C.flat.grad.clone()
    C.zero_grad()
    C.etbwd(t2, tt2, None, torch.ones_like(sd2))
    assert torch.equal(ga, C.flat.grad)
