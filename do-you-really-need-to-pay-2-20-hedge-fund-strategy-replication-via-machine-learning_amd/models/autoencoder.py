"""Factor autoencoder (reference ``Autoencoder_encapsulate.Autoencoder``, :19-35).

encoder: Dense(latent, no bias) -> LeakyReLU(0.2);  decoder: Dense(22, no bias) -> LeakyReLU(0.2).
Trained with Nadam + MSE through the explicit engine (native Dense kernels on GPU).
"""
from __future__ import annotations

import torch

from .layers import Dense, LeakyReLU, Sequential


class FactorAutoencoder(torch.nn.Module):
    def __init__(self, latent_dim: int, n_assets: int = 22, seed: int = 123, dtype=torch.float32, device="cpu"):
        super().__init__()
        self.latent_dim = latent_dim
        self.n_assets = n_assets
        self.encoder = Sequential([Dense(latent_dim, use_bias=False), LeakyReLU()], (n_assets,), name="encoder",
                                  seed=seed, dtype=dtype).to(device)
        self.decoder = Sequential([Dense(n_assets, use_bias=False), LeakyReLU()], (latent_dim,), name="decoder",
                                  seed=seed + 1, dtype=dtype).to(device)

    def forward(self, x):  # autograd path (oracle)
        return self.decoder(self.encoder(x))

    def parts(self):
        return (self.encoder, self.decoder)

    def count_params(self) -> int:
        return self.encoder.count_params() + self.decoder.count_params()

    @torch.no_grad()
    def predict(self, x):
        return self.decoder.predict(self.encoder.predict(x))

    def get_weights(self):
        return self.encoder.get_weights() + self.decoder.get_weights()

    def decoder_kernel(self):
        """(latent, 22) decoder weights — ``decoder.get_weights()[0]`` in the reference."""
        return self.decoder.get_weights()[0]

    @torch.no_grad()
    def loss_and_grads(self, x: torch.Tensor) -> torch.Tensor:
        """MSE(x, AE(x)) and its gradients into the two flat grad buffers (explicit engine)."""
        z, te = self.encoder.efwd(x, save=True)
        y, td = self.decoder.efwd(z, save=True)
        diff = y - x
        loss = (diff.to(torch.float64 if x.dtype == torch.float64 else torch.float32) ** 2).mean()
        dy = (2.0 / diff.numel()) * diff
        dz = self.decoder.ebwd(td, dy, need_dx=True)
        self.encoder.ebwd(te, dz)
        return loss
