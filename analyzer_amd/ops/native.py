"""Loader for the in-tree native extension ``analyzer_amd._C``.

The extension must exist (``python -m analyzer_amd.build_ext`` or
``__graft_entry__.build()``); there is no Python re-implementation behind it.
Importing fails loudly so a GPU run can never silently fall back to eager ops.
"""
from __future__ import annotations

import importlib

_C = None


def native():
    global _C
    if _C is None:
        try:
            _C = importlib.import_module("analyzer_amd._C")
        except ImportError as e:  # pragma: no cover - exercised when the build is missing
            raise ImportError(
                "analyzer_amd native extension is not built; run "
                "`python -m analyzer_amd.build_ext` (gfx950 HIP kernels + host mirror): %s" % e
            ) from e
    return _C


def is_built() -> bool:
    try:
        native()
        return True
    except ImportError:
        return False
