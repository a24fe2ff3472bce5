"""Random streams for training: noise, interpolation weights and batch sampling.

The reference draws everything on the host every step (``np.random.randint`` for the batch
index, ``np.random.normal`` for the noise — GAN/MTSS_WGAN_GP.py:268-271) and copies it to the
device.  Here, on GPU, a counter-based Philox4x32-10 generator runs inside the kernels that
consume the numbers (``torch.ops.hfrep.philox_normal_``, ``sample_windows``...): the stream state
is a device-resident 64-bit counter advanced by a tiny kernel, so no host sync or H2D copy is
needed and the whole training step can be captured in a hipGraph and replayed.

Data-parallel ranks use independent streams (``seed`` mixed with ``rank``).  On CPU a
``torch.Generator`` provides the same API.
"""
from __future__ import annotations

import torch

from ..ops import _native


def _mix(seed: int, stream: int) -> int:
    x = (seed * 0x9E3779B97F4A7C15 + stream * 0xBF58476D1CE4E5B9 + 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    x ^= x >> 31
    return x & 0x7FFFFFFFFFFFFFFF


class DeviceRNG:
    def __init__(self, seed: int = 123, device="cpu", stream: int = 0):
        self.device = torch.device(device)
        self.seed = _mix(seed, stream)
        self.native = self.device.type == "cuda" and _native.use_native_for(torch.empty(0, device=self.device))
        if self.native:
            self.ctr = torch.zeros(1, dtype=torch.int64, device=self.device)
        else:
            self.gen = torch.Generator(device="cpu").manual_seed(self.seed)

    def normal(self, shape, dtype=torch.float32) -> torch.Tensor:
        if self.native:
            out = torch.empty(shape, dtype=dtype, device=self.device)
            _native.native().philox_fill_(out, self.seed, self.ctr, 1)
            return out
        return torch.randn(shape, generator=self.gen, dtype=torch.float32).to(self.device, dtype)

    def uniform(self, shape, dtype=torch.float32) -> torch.Tensor:
        if self.native:
            out = torch.empty(shape, dtype=dtype, device=self.device)
            _native.native().philox_fill_(out, self.seed, self.ctr, 0)
            return out
        return torch.rand(shape, generator=self.gen, dtype=torch.float32).to(self.device, dtype)

    def sample_windows(self, dataset: torch.Tensor, batch: int, out_dtype=None, out=None) -> torch.Tensor:
        """``dataset[randint(0, N, batch)]`` (with replacement, GAN/GAN.py:178); ``out``: a contiguous
        destination (e.g. the first rows of the critic's [real; fake] input buffer)."""
        out_dtype = out_dtype or dataset.dtype
        if self.native:
            return _native.native().sample_windows(dataset, int(batch), self.seed, self.ctr, out_dtype, out)
        idx = torch.randint(0, dataset.shape[0], (batch,), generator=self.gen)
        y = dataset.index_select(0, idx.to(dataset.device)).to(out_dtype)
        return y if out is None else out.copy_(y)

    def state(self):
        return {"seed": self.seed, "ctr": (self.ctr.item() if self.native else None),
                "gen": (None if self.native else self.gen.get_state())}

    def load_state(self, st):
        if self.native and st.get("ctr") is not None:
            self.ctr.fill_(int(st["ctr"]))
        elif not self.native and st.get("gen") is not None:
            self.gen.set_state(st["gen"])
