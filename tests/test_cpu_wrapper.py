"""The Python wrapper refuses output buffers the library would overrun (it writes them through raw
pointers): wrong dtype, too small, non-contiguous.  Checked before any library call, so no GPU."""
import ctypes as C

import numpy as np
import pytest

from netbricks_amd import Maglev


def _bare():
    m = Maglev.__new__(Maglev)  # no device handle: validation must fire before the library call
    m._h = C.c_void_p()
    m.n_backends = 65
    m.device = 0
    return m


@pytest.mark.parametrize("bad", [
    dict(backend=np.empty(10, np.uint32)),
    dict(backend=np.empty(9, np.uint16)),
    dict(backend=np.empty(20, np.uint16)[::2]),
    dict(perm=np.empty(10, np.int64)),
    dict(perm=np.empty(5, np.uint32)),
    dict(counts=np.empty(65, np.uint32)),
    dict(backend=[0] * 10),
])
def test_host_submit_rejects_bad_outputs(bad):
    m = _bare()
    args = dict(backend=np.empty(10, np.uint16), perm=np.empty(10, np.uint32), counts=np.empty(66, np.uint32))
    args.update(bad)
    with pytest.raises(ValueError):
        m.host_submit(np.zeros(10, np.uint64), np.zeros(10, np.uint16), **args)


def test_host_submit_rejects_length_mismatch():
    with pytest.raises(ValueError):
        _bare().host_submit(np.zeros(10, np.uint64), np.zeros(9, np.uint16), np.empty(10, np.uint16))


def test_compact_group_block_fits_beside_ring():
    """The grouping beside a running in-place ring takes the compact group kernel when the default
    block would not fit in the LDS the ring leaves (maglev_kernels.hip group_compact): the compact
    block must fit there for every bin count the group kernels take (<= 1024 bins; above 1023
    backends group_wide_kernel runs), and the default block must fit for C2's 66 bins."""
    from netbricks_amd._lib import lib

    budget = lib.nbg_debug_lds_beside_ring()
    assert 24 * 1024 <= budget < 40 * 1024
    for nbins in (2, 66, 129, 257, 1001, 1024):
        assert lib.nbg_debug_group_lds(nbins, 1) <= budget, nbins
    assert lib.nbg_debug_group_lds(66, 0) <= budget
    assert lib.nbg_debug_group_lds(1001, 0) > budget  # C3 beside a ring: the compact kernel
    assert lib.nbg_debug_set_group_compact(2) != 0
    assert lib.nbg_debug_set_group_compact(-1) == 0
