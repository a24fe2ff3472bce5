"""Compatibility module: the reference's ``helper.py`` API (helper.py:10-162) on top of hfrep.

``from helper import ...`` keeps working for notebooks/scripts written against the reference.
Differences: ``dic_read`` never unpickles executable content (non-executing reader), and every
numeric routine is vectorised numpy (see hfrep.finance.replication).
"""
import hfrep  # noqa: F401  (registers the package)
from hfrep.data.io import dic_read, dic_save, read_csv  # noqa: F401
from hfrep.data.windows import random_sampling  # noqa: F401
from hfrep.finance.replication import (  # noqa: F401
    ex_post_return,
    factor_hf_split,
    normalization,
    price_impact,
    reshape_cab,
    transaction_cost,
)
from hfrep.utils.seed import set_seed  # noqa: F401

__all__ = ["normalization", "read_csv", "dic_read", "set_seed", "random_sampling", "transaction_cost",
           "price_impact", "reshape_cab", "ex_post_return", "factor_hf_split", "dic_save"]
