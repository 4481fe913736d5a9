"""netbricks_amd — MI355X-native Maglev flow-steering path for NetBricks.

The hot path (parse + MAC swap + 5-tuple FNV-1a + Maglev LUT + per-backend FIFO
grouping; optionally chained after test/lpm's DIR-24-8 gate) is hand-written HIP for gfx950 in `csrc/`, exported through the C-ABI in
`include/nbgpu.h` (`libnbgpu.so`).  This package is a thin Python surface over it.
"""
from ._lib import NBG_HOST_SLOTS, NBG_SENTINEL, NbgError, LIB_PATH  # noqa: F401  (raises ImportError if the .so is missing)
from .maglev import GroupedBatch, HostRegion, HostRing, Maglev, Ring, build_lut, make_trace  # noqa: F401
from .lpm import Lpm, LpmResult, build_lpm, chain_lpm_maglev, chain_lpm_maglev_multi  # noqa: F401

__all__ = ["Maglev", "GroupedBatch", "HostRegion", "HostRing", "build_lut", "make_trace", "NBG_SENTINEL", "NBG_HOST_SLOTS", "NbgError", "LIB_PATH",
           "Lpm", "LpmResult", "build_lpm", "chain_lpm_maglev", "chain_lpm_maglev_multi"]
