"""The in-tree native library links and registers its ops (CPU; no GPU needed).

A symbol left unresolved at link time (e.g. a definition that ended up in an anonymous namespace of
another translation unit) makes the shared object fail to load at import.  That failure showed up only
on the GPU box before this test existed.
"""
import os

import pytest

LIB = os.path.join(os.path.dirname(__file__), "..",
                   "do-you-really-need-to-pay-2-20-hedge-fund-strategy-replication-via-machine-learning_amd",
                   "ops", "_hfrep_native.so")


@pytest.mark.skipif(not os.path.exists(LIB), reason="native library not built")
def test_native_library_loads_and_registers_ops():
    import torch

    from hfrep.ops import _native

    assert _native.available(), "in-tree _hfrep_native.so failed to load (unresolved symbol?)"
    ops = torch.ops.hfrep
    for name in ("linear_wgrad_", "mlp_gen_fwd", "mlp_wgp_affine", "mlp_critic_dx_affine", "lstm_wgrad_"):
        assert hasattr(ops, name), name
    assert ops.mlp_affine_supported(32, 24) and not ops.mlp_affine_supported(36, 7)
