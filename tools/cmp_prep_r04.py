import ctypes, sys, os, numpy as np, torch
sys.path.insert(0, '.')
import bench
res = {}
for tag, path in (('new', 'poor_man_gplvm_amd/csrc/libpmg_hip.so'), ('old', 'exp/oldprep/libpmg_hip.so')):
    lib = ctypes.CDLL(os.path.abspath(path))
    f = lib.pmg_spikes_prepare
    P, I64, I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
    f.argtypes = [P, I64, I32, P, I32, P, I32, P, P, I32, P, P]
    f.restype = I32
    for (N, T, L) in ((256, 50000, 256), (512, 100000, 512), (30, 1000, 100)):
        y, B, W0, lp0 = bench.synth(N, T, L) if T <= 100000 else None
        yt = torch.as_tensor(y, device='cuda')
        Kp = (N + 127) // 128 * 128
        Np = (N + 1 + 63) // 64 * 64
        Tp = (T + 63) // 64 * 64
        yq = torch.zeros((Tp, Kp), dtype=torch.int8, device='cuda')
        gc = torch.zeros(T, dtype=torch.float64, device='cuda')
        ye = torch.zeros((T, Np), dtype=torch.float32, device='cuda')
        fl = torch.zeros(1, dtype=torch.int32, device='cuda')
        rc = f(yt.data_ptr(), T, N, None, 0, yq.data_ptr(), Kp, gc.data_ptr(), ye.data_ptr(), Np, fl.data_ptr(), None)
        torch.cuda.synchronize()
        res[(tag, N)] = (rc, yq.cpu().numpy(), gc.cpu().numpy(), ye.cpu().numpy(), fl.cpu().numpy())
for N in (256, 512, 30):
    a, b = res[('new', N)], res[('old', N)]
    print(N, 'rc', a[0], b[0], 'yq eq', np.array_equal(a[1], b[1]), 'gconst eq', np.array_equal(a[2], b[2]),
          'max gconst diff', float(np.max(np.abs(a[2] - b[2]))), 'yext eq', np.array_equal(a[3], b[3]), 'flags', a[4], b[4])
