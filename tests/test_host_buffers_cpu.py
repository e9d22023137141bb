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
    monkeypatch.setattr(nat, "HOST_CACHE_BYTES", 3 * 4096)
    monkeypatch.setattr(nat, "_host_cache", {})
    monkeypatch.setattr(nat, "_host_cache_total", 0)
    assert nat._host_cache_give(0x1000, 4096) and nat._host_cache_give(0x2000, 4096)
    assert nat._host_cache_give(0x3000, 8192) is False          # over the cap: the caller frees it
    assert nat._host_cache_total == 8192
    assert nat._host_cache_take(8192) is None                   # no block of that size
    assert nat._host_cache_take(4096) in (0x1000, 0x2000)
    assert nat._host_cache_total == 4096
    freed = []
    monkeypatch.setattr(nat, "load", lambda: type("L", (), {"pmg_host_free": lambda self, p, n: freed.append((p, n))})())
    nat.release_host_cache()
    assert len(freed) == 1 and nat._host_cache_total == 0 and nat._host_cache == {}
