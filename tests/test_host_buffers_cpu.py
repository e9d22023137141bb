"""Host-side logic of the page-locked result buffers (_native.HostBuffer): the C entry
point's failure path without a GPU (no mapping leaked, a message instead of a crash) and
the released-block cache's accounting."""
import ctypes

import pytest
import torch

from poor_man_gplvm_amd import _native as nat


@pytest.mark.skipif(torch.cuda.is_available(), reason="the failure path needs a host without a GPU")
def test_host_alloc_fails_cleanly_without_gpu():
    lib = nat.load()
    p = ctypes.c_void_p()
    rc = lib.pmg_host_alloc(1 << 20, 2, 1, ctypes.byref(p))
    assert rc != 0 and not p.value
    assert b"hipHostRegister" in lib.pmg_last_error()
    with pytest.raises(nat.NativeError):
        nat.host_array((16, 16), "float32")


def test_host_cache_accounting(monkeypatch):
    """The cache holds at most HOST_CACHE_BYTES: returning a block that does not fit
    evicts the least recently returned blocks (unmapped at once), and a block larger than
    the whole cap is released instead of cached."""
    freed = []
    fake = type("L", (), {"pmg_host_free": lambda self, p, n: freed.append((p, n))})()
    monkeypatch.setattr(nat, "load", lambda: fake)
    monkeypatch.setattr(nat, "HOST_CACHE_BYTES", 3 * 4096)
    monkeypatch.setattr(nat, "_host_cache", [])
    monkeypatch.setattr(nat, "_host_cache_total", 0)
    assert nat._host_cache_give(0x1000, 4096) and nat._host_cache_give(0x2000, 4096)
    assert nat._host_cache_give(0x3000, 8192)                   # evicts 0x1000, the oldest
    assert freed == [(0x1000, 4096)] and nat.host_cache_bytes() == 3 * 4096
    assert nat._host_cache_give(0x4000, 4 * 4096)               # larger than the cap: freed
    assert freed[-1] == (0x4000, 4 * 4096) and nat.host_cache_bytes() == 3 * 4096
    assert nat._host_cache_take(8192) == 0x3000
    assert nat._host_cache_take(8192) is None                   # no block of that size left
    assert nat.host_cache_bytes() == 4096
    nat.release_host_cache()
    assert freed[-1] == (0x2000, 4096) and nat._host_cache_total == 0 and nat._host_cache == []


def test_host_cache_default_cap():
    """Default cap: at most 2 GiB and at most 1/32 of physical memory; the environment
    variable overrides it."""
    import os
    assert 0 < nat._default_cache_bytes() <= 2 << 30
    old = os.environ.get("PMG_HOST_CACHE_BYTES")
    os.environ["PMG_HOST_CACHE_BYTES"] = "12345"
    try:
        assert nat._default_cache_bytes() == 12345
    finally:
        if old is None:
            del os.environ["PMG_HOST_CACHE_BYTES"]
        else:
            os.environ["PMG_HOST_CACHE_BYTES"] = old
