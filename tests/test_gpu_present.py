"""The context's device data environment (include/rrtmgpnn.h, rrtmgpnn_present*; csrc/present.cpp) through the C ABI:
upload on first READ, WRITE marks the device copy newer, update_host copies it back, update_device re-arms the
upload, a new size for the same address replaces the entry, per-call buffers come back from the pool, and queued
device-to-host copies (pinned staging ring) complete at rrtmgpnn_context_synchronize -- also past the ring's size."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

READ, WRITE = 1, 2


@pytest.fixture
def ctx():
    from rrtmgpnn import _lib
    L = _lib.lib()
    c = ctypes.c_void_p()
    assert L.rrtmgpnn_context_create_owned(0, ctypes.byref(c)) == 0
    yield L, c
    L.rrtmgpnn_context_destroy(c)


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def _dev_to_host(L, c, d, n):
    out = np.empty(n, np.float32)
    assert L.rrtmgpnn_copy_d2h(c, _p(out), d, out.nbytes) == 0
    assert L.rrtmgpnn_context_synchronize(c) == 0
    return out


def test_present_read_write_update(ctx):
    L, c = ctx
    h = np.arange(1000, dtype=np.float32)
    d = ctypes.c_void_p()
    assert L.rrtmgpnn_present(c, _p(h), h.nbytes, READ, ctypes.byref(d)) == 0
    np.testing.assert_array_equal(_dev_to_host(L, c, d, 1000), h)
    # a second READ of a current copy does not upload again: the host change is not seen ...
    h[:] = -1.0
    d2 = ctypes.c_void_p()
    assert L.rrtmgpnn_present(c, _p(h), h.nbytes, READ, ctypes.byref(d2)) == 0
    assert d2.value == d.value
    np.testing.assert_array_equal(_dev_to_host(L, c, d, 1000), np.arange(1000, dtype=np.float32))
    # ... until update_device announces it
    assert L.rrtmgpnn_present_update_device(c, _p(h)) == 0
    assert L.rrtmgpnn_present(c, _p(h), h.nbytes, READ, ctypes.byref(d2)) == 0
    np.testing.assert_array_equal(_dev_to_host(L, c, d2, 1000), h)
    # WRITE: the device copy is newer; update_host brings it back
    src = np.full(1000, 7.5, np.float32)
    assert L.rrtmgpnn_present(c, _p(h), h.nbytes, WRITE, ctypes.byref(d2)) == 0
    assert L.rrtmgpnn_copy_h2d(c, d2, _p(src), src.nbytes) == 0
    assert L.rrtmgpnn_present_update_host(c, _p(h)) == 0
    np.testing.assert_array_equal(h, src)
    # another size at the same address replaces the entry (uploaded again)
    d3 = ctypes.c_void_p()
    assert L.rrtmgpnn_present(c, _p(h), 400, READ, ctypes.byref(d3)) == 0
    np.testing.assert_array_equal(_dev_to_host(L, c, d3, 100), h[:100])
    assert L.rrtmgpnn_present_delete(c, _p(h)) == 0
    assert L.rrtmgpnn_present_delete(c, _p(h)) == 0  # absent: no-op
    assert L.rrtmgpnn_present(c, None, 4, READ, ctypes.byref(d3)) != 0  # null host array refused


def test_pool_reuse_and_stage(ctx):
    L, c = ctx
    a = np.random.default_rng(1).random(5000).astype(np.float32)
    d = ctypes.c_void_p()
    assert L.rrtmgpnn_stage_h2d(c, _p(a), a.nbytes, ctypes.byref(d)) == 0
    np.testing.assert_array_equal(_dev_to_host(L, c, d, 5000), a)
    assert L.rrtmgpnn_release(c, d) == 0
    e = ctypes.c_void_p()
    assert L.rrtmgpnn_scratch(c, a.nbytes - 100, ctypes.byref(e)) == 0
    assert e.value == d.value  # the released buffer serves the next request of about its size
    assert L.rrtmgpnn_memset_async(c, e, 0, a.nbytes - 100) == 0
    assert not _dev_to_host(L, c, e, 4900).any()
    assert L.rrtmgpnn_release(c, e) == 0


def test_queued_copies_complete_at_synchronize_beyond_the_ring(ctx):
    L, c = ctx
    n = 12 << 20  # 48 MiB per array: three of them exceed the 32 MiB initial ring, forcing a wrap and a regrowth
    srcs = [np.full(n, float(k + 1), np.float32) for k in range(3)]
    devs, outs = [], []
    for s in srcs:
        d = ctypes.c_void_p()
        assert L.rrtmgpnn_scratch(c, s.nbytes, ctypes.byref(d)) == 0
        assert L.rrtmgpnn_copy_h2d(c, d, _p(s), s.nbytes) == 0
        devs.append(d)
    for d in devs:
        o = np.zeros(n, np.float32)
        assert L.rrtmgpnn_copy_d2h(c, _p(o), d, o.nbytes) == 0
        outs.append(o)
    assert L.rrtmgpnn_context_synchronize(c) == 0
    for s, o in zip(srcs, outs):
        np.testing.assert_array_equal(o, s)
    for d in devs:
        assert L.rrtmgpnn_release(c, d) == 0
