"""Batched tensor operators of the rating engine (HIP kernels on MI355X)."""
from .native import native, is_built  # noqa: F401
