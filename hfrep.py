"""Import shim: exposes the framework package under the short name ``hfrep``.

The package source lives in the directory
``do-you-really-need-to-pay-2-20-hedge-fund-strategy-replication-via-machine-learning_amd/``
(the layout the build plan asks for).  A hyphenated directory is not a valid
Python identifier, so this module loads that directory as the package
``hfrep`` and replaces itself in ``sys.modules``.  ``import hfrep.models``
and friends then resolve against the real package directory.
"""
import importlib.util
import os
import sys

PACKAGE_DIR = os.path.join(
    os.path.dirname(os.path.abspath(__file__)),
    "do-you-really-need-to-pay-2-20-hedge-fund-strategy-replication-via-machine-learning_amd",
)

_spec = importlib.util.spec_from_file_location(
    "hfrep", os.path.join(PACKAGE_DIR, "__init__.py"), submodule_search_locations=[PACKAGE_DIR]
)
_mod = importlib.util.module_from_spec(_spec)
sys.modules["hfrep"] = _mod
_spec.loader.exec_module(_mod)

if __name__ == "__main__":  # python -m hfrep <command> ... / python hfrep.py <command> ...
    from hfrep.cli import main

    sys.exit(main())
