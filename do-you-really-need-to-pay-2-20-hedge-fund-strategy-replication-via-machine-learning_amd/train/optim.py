"""Keras 2.7-exact optimizers over flat parameter buffers.

One optimizer object may be applied to several models, sharing one ``iterations`` counter —
exactly what happens in the reference when a single Keras optimizer instance is compiled into
both the critic and the combined model (e.g. GAN/GAN.py:100,106,125): Adam's bias correction
then advances on every ``train_on_batch`` of either model.  Slots (ms / m, v) are per model.

On GPU the update is one fused kernel launch per model (``torch.ops.hfrep.{rmsprop_,adam_,nadam_}``)
with the counter kept on device, so the whole optimizer step is hipGraph-capturable.
On CPU the same formulas run in PyTorch.
"""
from __future__ import annotations

import torch

from ..ops import _native


class KerasOptimizer:
    def __init__(self, kind: str = "rmsprop", learning_rate: float = 1e-3, rho: float = 0.9, beta_1: float = 0.9,
                 beta_2: float = 0.999, epsilon: float = 1e-7, device="cpu"):
        self.kind = kind.lower()
        assert self.kind in ("rmsprop", "adam", "nadam")
        self.lr, self.rho, self.b1, self.b2, self.eps = learning_rate, rho, beta_1, beta_2, epsilon
        self.device = torch.device(device)
        self.iterations = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.m_cache = torch.ones(1, dtype=torch.float32, device=self.device)  # Nadam momentum cache
        self.slots: dict[int, tuple] = {}

    @classmethod
    def rmsprop(cls, lr=1e-3, **kw):
        return cls("rmsprop", lr, **kw)

    @classmethod
    def adam(cls, lr=1e-3, beta_1=0.9, **kw):
        return cls("adam", lr, beta_1=beta_1, **kw)

    @classmethod
    def nadam(cls, lr=1e-3, **kw):
        return cls("nadam", lr, **kw)

    def _slots(self, flat: torch.Tensor):
        key = flat.data_ptr()
        if key not in self.slots:
            z = torch.zeros_like(flat)
            self.slots[key] = (z,) if self.kind == "rmsprop" else (z, torch.zeros_like(flat))
        return self.slots[key]

    def state_dict(self):
        return {"iterations": self.iterations.detach().cpu(), "m_cache": self.m_cache.detach().cpu(),
                "slots": [tuple(s.detach().cpu() for s in v) for v in self.slots.values()]}

    def load_slots(self, flat: torch.Tensor, slots):
        self.slots[flat.data_ptr()] = tuple(s.to(flat.device) for s in slots)

    @torch.no_grad()
    def apply(self, flat: torch.Tensor, grad: torch.Tensor | None = None, clip: float = 0.0, gscale: float = 1.0):
        """One ``apply_gradients`` on a flat parameter buffer (+ optional clip to [-clip, clip])."""
        self._update(flat, flat.grad if grad is None else grad, clip, gscale)
        self._advance(flat.device)

    @torch.no_grad()
    def apply_group(self, flats, clip: float = 0.0, gscale: float = 1.0):
        """One ``apply_gradients`` over several flat buffers (one iteration tick, like one Keras model)."""
        for f in flats:
            self._update(f, f.grad, clip, gscale)
        self._advance(flats[0].device)

    def _advance(self, device):
        if device.type == "cuda" and _native.use_native_for(self.iterations):
            _native.native().step_advance_(self.iterations, self.m_cache if self.kind == "nadam" else None, self.b1)
            return
        if self.kind == "nadam":
            t = float(self.iterations.item())
            self.m_cache.mul_(self.b1 * (1 - 0.5 * 0.96 ** (0.004 * (t + 1))))
        self.iterations.add_(1)

    def _update(self, flat, grad, clip, gscale):
        slots = self._slots(flat)
        if flat.device.type == "cuda" and _native.use_native_for(flat):
            ops = _native.native()
            if self.kind == "rmsprop":
                ops.rmsprop_(flat, grad, slots[0], self.lr, self.rho, self.eps, clip, gscale)
            elif self.kind == "adam":
                ops.adam_(flat, grad, slots[0], slots[1], self.iterations, self.lr, self.b1, self.b2, self.eps, clip,
                          gscale)
            else:
                ops.nadam_(flat, grad, slots[0], slots[1], self.iterations, self.m_cache, self.lr, self.b1, self.b2,
                           self.eps, gscale)
                if clip > 0:
                    ops.clip_(flat, clip)
            return
        g = grad * gscale if gscale != 1.0 else grad
        if self.kind == "rmsprop":
            (ms,) = slots
            ms.mul_(self.rho).add_((1 - self.rho) * g * g)
            flat.sub_(self.lr * g / (ms.sqrt() + self.eps))
        elif self.kind == "adam":
            m, v = slots
            t = float(self.iterations.item()) + 1
            lr_t = self.lr * (1 - self.b2 ** t) ** 0.5 / (1 - self.b1 ** t)
            m.mul_(self.b1).add_((1 - self.b1) * g)
            v.mul_(self.b2).add_((1 - self.b2) * g * g)
            flat.sub_(lr_t * m / (v.sqrt() + self.eps))
        else:
            m, v = slots
            t = float(self.iterations.item())
            mt = self.b1 * (1 - 0.5 * 0.96 ** (0.004 * (t + 1)))
            mt1 = self.b1 * (1 - 0.5 * 0.96 ** (0.004 * (t + 2)))
            sched_new = float(self.m_cache.item()) * mt
            sched_next = sched_new * mt1
            gp = g / (1 - sched_new)
            m.mul_(self.b1).add_((1 - self.b1) * g)
            v.mul_(self.b2).add_((1 - self.b2) * g * g)
            mp = m / (1 - sched_next)
            vp = v / (1 - self.b2 ** (t + 1))
            mbar = (1 - mt) * gp + mt1 * mp
            flat.sub_(self.lr * mbar / (vp.sqrt() + self.eps))
        if clip > 0:
            flat.clamp_(-clip, clip)
