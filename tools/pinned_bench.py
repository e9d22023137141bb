"""Host page-locked allocation variants for the fit's returned arrays (410 MB = one
(T, 2, L) f32 array at C3): torch's pinned allocator vs pmg_host_alloc with 1..16 touch
threads, with and without huge pages, and the device->host copy rate into each.
Run on the GPU box: python tools/pinned_bench.py > gpurun_out/pinned_bench.json"""
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from poor_man_gplvm_amd import _native as nat  # noqa: E402


def main():
    lib = nat.load()
    nbytes = 100000 * 2 * 512 * 4
    g = torch.rand(nbytes // 4, device='cuda')
    torch.cuda.synchronize()
    out = {}
    t0 = time.perf_counter()
    h = torch.empty(nbytes // 4, dtype=torch.float32, pin_memory=True)
    out['torch_pinned_alloc'] = time.perf_counter() - t0
    t0 = time.perf_counter()
    h.copy_(g)
    out['torch_pinned_copy'] = time.perf_counter() - t0
    del h
    for th in (1, 4, 8, 16):
        for huge in (0, 1):
            p = ctypes.c_void_p()
            t0 = time.perf_counter()
            nat.check(lib.pmg_host_alloc(nbytes, th, huge, ctypes.byref(p)), 'alloc')
            ta = time.perf_counter() - t0
            arr = (ctypes.c_float * (nbytes // 4)).from_address(p.value)
            ht = torch.frombuffer(arr, dtype=torch.float32)
            t0 = time.perf_counter()
            ht.copy_(g)
            tc = time.perf_counter() - t0
            ok = bool(torch.equal(ht[:1000], g[:1000].cpu()))
            del ht, arr
            t0 = time.perf_counter()
            nat.check(lib.pmg_host_free(p, nbytes), 'free')
            tf = time.perf_counter() - t0
            out[f'pmg_t{th}_h{huge}'] = dict(alloc=round(ta, 5), copy=round(tc, 5), free=round(tf, 5), ok=ok)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
