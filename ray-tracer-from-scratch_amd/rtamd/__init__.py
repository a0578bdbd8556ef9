"""rtamd — Python host glue for the MI355X trace/shade path (C-ABI in include/rt_capi.h).

The compute path is the HIP library lib/librt_amd.so; this package only binds it
(capi), builds scenes/cameras (scenes), and runs the optional multi-GPU row tiling
(tiling).  Importing never falls back to CPU code.
"""
from . import capi, scenes  # noqa: F401

__all__ = ["capi", "scenes"]
