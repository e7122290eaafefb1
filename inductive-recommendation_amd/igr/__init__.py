"""igr - MI355X-native inductive graph convolution (IGCN / LightGCN hot path).

Drop-in for the DGL-backed path of umaDosey/Inductive-Recommendation:
`igr.ops.graph` / `igr.ops.gspmm` replace `dgl.graph` / `dgl.ops.gspmm`, and
igr.model / igr.trainer keep the reference's model and trainer surface.
Device work runs in hand-written HIP kernels (libigr.so, C ABI in
include/igr.h).
"""
from . import _lib  # noqa: F401
from .graph import Graph  # noqa: F401

__version__ = '1.0.0'


def lib_path():
    return _lib.LIB_PATH
