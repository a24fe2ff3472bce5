"""Compatibility package mirroring the reference's ``GAN/`` scripts (one module per model)."""
