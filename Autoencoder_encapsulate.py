"""Compatibility module: ``Autoencoder`` and ``AE`` (Autoencoder_encapsulate.py:19-243) on hfrep.

``AE(x_train, y_train, x_test, y_test, latent_dim)`` with ``train / model_IS_r2 / model_IS_RMSE /
model_OOS_r2 / model_OOS_RMSE / ante / post / turnover / plot`` — see
hfrep.finance.autoencoder_replication for the implementation and the parity options.
"""
import hfrep  # noqa: F401
from hfrep.finance.autoencoder_replication import AE  # noqa: F401
from hfrep.models.autoencoder import FactorAutoencoder as Autoencoder  # noqa: F401

__all__ = ["Autoencoder", "AE"]
