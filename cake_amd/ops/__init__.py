"""Compute ops: gfx950 HIP kernels (:mod:`.hip`) and the PyTorch oracle (:mod:`.reference`)."""
from . import reference  # noqa: F401
from ._lib import KernelError, available, kernels  # noqa: F401
