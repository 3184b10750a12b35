"""Loader for the in-tree native extension ``analyzer_amd._C``.

The extension must exist (``python -m analyzer_amd.build_ext`` or
``__graft_entry__.build()``); there is no Python re-implementation behind it.
Importing fails loudly so a GPU run can never silently fall back to eager ops.
"""
from __future__ import annotations

import importlib
import importlib.util
import os

_C = None


def native():
    global _C
    if _C is None:
        try:
            lib = os.environ.get("ANA_NATIVE_LIB")  # A/B experiments: another build of the same API
            if lib:
                spec = importlib.util.spec_from_file_location("analyzer_amd._C", lib)
                _C = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(_C)
            else:
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
