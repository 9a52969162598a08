"""tunebfree_amd -- MI355X-native batched render engine for tuneBfree's DSP chain.

The product is the in-tree C-ABI library ``libtbf.so`` (include/tbf.h): host-side
table builders + control plane in C++, the per-block render in a hand-written gfx950
HIP kernel.  This package is the Python host mirror of that ABI (ctypes); it has no
CPU fallback -- if the library or a GPU is missing it raises.
"""
from .engine import Engine, TbfError, load_library, LIB_PATH  # noqa: F401
from . import params  # noqa: F401

__all__ = ["Engine", "TbfError", "load_library", "LIB_PATH", "params"]
