"""ctypes binding of ``libpmg_hip.so`` (the C ABI declared in ``include/pmg.h``).

PyTorch is imported first so that the library's ``libamdhip64.so.7`` dependency
resolves to the HIP runtime torch already loaded (one runtime per process);
device buffers are torch tensors, passed as raw pointers together with the
current torch stream.  There is no fallback: if the library is missing or fails
to load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

import torch  # noqa: F401  (loads the HIP runtime before the library)

_HERE = os.path.dirname(os.path.abspath(__file__))
# PMG_LIB_PATH: an alternative build of the same ABI (experiment variants, tools/build_variant.sh)
LIB_PATH = os.environ.get("PMG_LIB_PATH") or os.path.join(_HERE, "csrc", "libpmg_hip.so")

PMG_MAX_BAND = 32
# pmg_fwdbwd_state slots (include/pmg.h)
STATE_FWD_IN, STATE_FWD_OUT, STATE_BWD_IN, STATE_BWD_FIRST = 0, 1, 2, 3
# int32 control words at the start of a pmg_fwdbwd workspace (fb_kernels.h kCtl*):
# a forward block and a backward block, each {chunks recomputed, relaxation rounds, timeout}
CTL_WORDS, CTL_FWD, CTL_BWD = 32, 0, 16
CTL_REPAIRS, CTL_ROUNDS, CTL_ERR, CTL_WARM = 0, 1, 2, 3
# pmg_forward_filter_phase flag: alpha's d = 1 rows are not written (PMG_PHASE_NO_JUMP_ROWS)
PHASE_NO_JUMP_ROWS = 4
# both phase calls of an E-step: the device lengthens the next warm-up after a cascade (PMG_PHASE_ADAPTIVE_WARMUP)
PHASE_ADAPTIVE_WARMUP = 8
# forward, both phase calls: no alpha written at all (logc / logZ only; PMG_PHASE_NO_ALPHA)
PHASE_NO_ALPHA = 16
# backward, both phase calls: P written as three bf16 planes [3][T][ldd] (PMG_PHASE_P_BF16X3)
PHASE_P_BF16X3 = 32
# phase-1 calls: each main-pass chain on two waves where compiled (PMG_PHASE_TWO_WAVES)
PHASE_TWO_WAVES = 64
ABI_VERSION = 2


def phase_segments(S: int) -> int:
    """PMG_PHASE_SEGMENTS(S): the relaxation's segment count per sequence (0 = default)."""
    S = int(S or 0)
    if not 0 <= S <= 0xfff:
        raise ValueError(f"relax_segments must be in [0, 4095], got {S}")
    return S << 16

# every symbol the header declares (checked by tests/test_capi_symbols.py)
EXPORTED_SYMBOLS = (
    "pmg_abi_version", "pmg_last_error", "pmg_spikes_prepare", "pmg_tuning_softplus",
    "pmg_emission_workspace_size", "pmg_emission_poisson", "pmg_emission_poisson_f64",
    "pmg_emission_rowref", "pmg_loglik_materialize", "pmg_fwdbwd_workspace_size",
    "pmg_forward_filter", "pmg_backward_smoother", "pmg_fwdbwd_repair_counter_offset",
    "pmg_forward_filter_phase", "pmg_backward_smoother_phase",
    "pmg_suffstats_workspace_size", "pmg_suffstats", "pmg_exp", "pmg_log", "pmg_roll_columns",
    "pmg_emission_latent_mask", "pmg_emission_latent_mask_batched", "pmg_emission_gaussian_dt",
    "pmg_spikes_bf16t", "pmg_suffstats_bf16_workspace_size", "pmg_suffstats_bf16",
    "pmg_mstep_workspace_size", "pmg_mstep_adam_supported", "pmg_mstep_adam", "pmg_joint_workspace_size",
    "pmg_joint_accumulate", "pmg_fwdbwd_lpad", "pmg_fwdbwd_state",
    "pmg_mstep_tiled_workspace_size", "pmg_mstep_adam_tiled",
    "pmg_emission_poisson_dt", "pmg_naive_bayes_normalize",
    "pmg_tuning_linear", "pmg_emission_gaussian", "pmg_gaussian_mstep_workspace_size", "pmg_gaussian_mstep",
    "pmg_dense_workspace_size", "pmg_dense_forward", "pmg_dense_backward", "pmg_joint_log_accumulate",
    "pmg_tuning_softplus_batched", "pmg_emission_rowref_batched", "pmg_fwdbwd_batched_workspace_size",
    "pmg_forward_filter_batched", "pmg_backward_smoother_batched",
    "pmg_mstep_batched_workspace_size", "pmg_mstep_adam_batched_supported", "pmg_mstep_adam_batched",
    "pmg_emission_range_flag", "pmg_mstep_adam_status",
    "pmg_suffstats_bf16x3_workspace_size", "pmg_suffstats_bf16x3",
    "pmg_dense_lpad", "pmg_dense_state", "pmg_dense_forward_phase", "pmg_dense_backward_phase",
    "pmg_host_alloc", "pmg_host_free", "pmg_copy_d2h",
    "pmg_joint_log_workspace_size", "pmg_joint_log_accumulate_ws", "pmg_posterior_outputs",
)


class NativeError(RuntimeError):
    pass


class Transition(ctypes.Structure):
    """pmg_transition (include/pmg.h)."""
    _fields_ = [("L", ctypes.c_int32), ("band", ctypes.c_int32),
                ("g", ctypes.c_float * (PMG_MAX_BAND + 1)), ("invz", ctypes.c_void_p),
                ("A", ctypes.c_float * 4)]


class DenseTransition(ctypes.Structure):
    """pmg_dense_transition (include/pmg.h)."""
    _fields_ = [("L", ctypes.c_int32), ("logK", ctypes.c_void_p), ("logKT", ctypes.c_void_p),
                ("logK_lo", ctypes.c_void_p), ("logKT_lo", ctypes.c_void_p), ("logA", ctypes.c_float * 4)]


class AdamCfg(ctypes.Structure):
    """pmg_adam_cfg (include/pmg.h)."""
    _fields_ = [("lr", ctypes.c_double), ("b1", ctypes.c_double), ("b2", ctypes.c_double),
                ("eps", ctypes.c_double), ("eps_root", ctypes.c_double),
                ("prior_std", ctypes.c_double), ("tol", ctypes.c_double),
                ("maxiter", ctypes.c_int32)]


_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_D = ctypes.c_double
_SZ = ctypes.c_size_t

_SIGS = {
    "pmg_abi_version": ([], _I32),
    "pmg_last_error": ([], ctypes.c_char_p),
    "pmg_spikes_prepare": ([_P, _I64, _I32, _P, _I32, _P, _I32, _P, _P, _I32, _P, _P], _I32),
    "pmg_tuning_softplus": ([_P, _P, _I32, _I32, _I32, _P, _P, _P], _I32),
    "pmg_emission_workspace_size": ([_I64, _I32, _I32], _SZ),
    "pmg_emission_poisson": ([_P, _P, _P, _P, _P, _D, _I64, _I32, _I32, _I32, _P, _P, _P, _P, _SZ, _P], _I32),
    "pmg_emission_poisson_f64": ([_P, _P, _P, _P, _I32, _P, _D, _I64, _I32, _I32, _P, _P, _P, _P, _SZ, _P], _I32),
    "pmg_emission_poisson_dt": ([_P, _P, _P, _P, _I32, _P, _P, _I64, _I32, _I32, _P, _P, _P], _I32),
    "pmg_naive_bayes_normalize": ([_P, _P, _I64, _I32, _P, _P, _P], _I32),
    "pmg_emission_rowref": ([_P, _I64, _I32, _D, _P, _P, _P], _I32),
    "pmg_loglik_materialize": ([_P, _P, _I64, _I32, _P, _P], _I32),
    "pmg_fwdbwd_workspace_size": ([_I64, _I32, _I32], _SZ),
    "pmg_forward_filter": ([_P, _P, _P, _I64, ctypes.POINTER(Transition), _D, _I32, _I32, _D,
                            _P, _P, _P, _P, _SZ, _P], _I32),
    "pmg_forward_filter_phase": ([_P, _P, _P, _I64, ctypes.POINTER(Transition), _D, _I32, _I32, _D,
                                  _P, _P, _P, _P, _SZ, _P, _I32], _I32),
    "pmg_backward_smoother_phase": ([_P, _P, _P, _I64, ctypes.POINTER(Transition), _D, _I32, _I32, _D,
                                     _P, _P, _P, _P, _SZ, _P, _I32], _I32),
    "pmg_backward_smoother": ([_P, _P, _P, _I64, ctypes.POINTER(Transition), _D, _I32, _I32, _D,
                               _P, _P, _P, _P, _SZ, _P], _I32),
    "pmg_fwdbwd_repair_counter_offset": ([_I64, _I32, _I32], _SZ),
    "pmg_fwdbwd_lpad": ([_I32], _I32),
    "pmg_fwdbwd_state": ([_P, _I64, _I32, _I32, _I32, _I64], _P),
    "pmg_suffstats_workspace_size": ([_I64, _I32, _I32], _SZ),
    "pmg_suffstats": ([_P, _P, _I64, _I32, _I32, _I32, _P, _P, _P, _SZ, _P], _I32),
    "pmg_spikes_bf16t": ([_P, _I64, _I32, _P, _I64, _P], _I32),
    "pmg_suffstats_bf16_workspace_size": ([_I64, _I32, _I32], _SZ),
    "pmg_suffstats_bf16": ([_P, _P, _I64, _I64, _I32, _I32, _I32, _P, _P, _P, _SZ, _P], _I32),
    "pmg_suffstats_bf16x3_workspace_size": ([_I64, _I32, _I32], _SZ),
    "pmg_suffstats_bf16x3": ([_P, _I64, _P, _I64, _I64, _I32, _I32, _I32, _P, _P, _P, _SZ, _P], _I32),
    "pmg_exp": ([_P, _I64, _P, _P], _I32),
    "pmg_log": ([_P, _I64, _P, _P], _I32),
    "pmg_posterior_outputs": ([_P, _I64, _I32, _P, _P, _P, _P], _I32),
    "pmg_roll_columns": ([_P, _I64, _I32, _P, _P, _P], _I32),
    "pmg_emission_latent_mask": ([_P, _P, _I64, _I32, _P, _P, _P, _P], _I32),
    "pmg_emission_latent_mask_batched": ([_P, _P, _I64, _I32, _P, _I32, _P, _P, _P], _I32),
    "pmg_mstep_workspace_size": ([_I32, _I32], _SZ),
    "pmg_mstep_adam_supported": ([_I32, _I32, _I32], ctypes.c_int),
    "pmg_mstep_adam": ([_P, _P, _P, _P, _P, _P, _P, _I32, _I32, _I32, ctypes.POINTER(AdamCfg),
                        _P, _P, _P, _P, _SZ, _P], _I32),
    "pmg_mstep_adam_status": ([_P, ctypes.POINTER(_I32), _P], _I32),
    "pmg_host_alloc": ([_SZ, _I32, _I32, ctypes.POINTER(ctypes.c_void_p)], _I32),
    "pmg_host_free": ([_P, _SZ], _I32),
    "pmg_copy_d2h": ([_P, _P, _SZ, _P], _I32),
    "pmg_mstep_tiled_workspace_size": ([_I32, _I32, _I32], _SZ),
    "pmg_mstep_adam_tiled": ([_P, _P, _P, _P, _P, _P, _P, _I32, _I32, _I32, ctypes.POINTER(AdamCfg),
                              _P, _P, _P, _P, _SZ, _P], _I32),
    "pmg_tuning_linear": ([_P, _P, _I32, _I32, _I32, _P, _P, _P], _I32),
    "pmg_emission_gaussian": ([_P, _P, _P, _I32, _P, ctypes.c_double, ctypes.c_double, _I64, _I32, _I32,
                               _P, _P, _P, _P], _I32),
    "pmg_emission_gaussian_dt": ([_P, _P, _P, _I32, _P, ctypes.c_double, _P, _I64, _I32, _I32, _P, _P, _P], _I32),
    "pmg_gaussian_mstep_workspace_size": ([_I32, _I32], _SZ),
    "pmg_gaussian_mstep": ([_P, _P, _P, _I32, _I32, _I32, ctypes.c_double, ctypes.c_double, _P, _P, _P, _SZ,
                            _P], _I32),
    "pmg_joint_workspace_size": ([_I64, _I32], _SZ),
    "pmg_dense_workspace_size": ([_I64, _I32, _I32], _SZ),
    "pmg_dense_forward": ([_P, _P, _P, _P, _I64, ctypes.POINTER(DenseTransition), _D, _I32, _I32, _D,
                           _P, _P, _P, _P, _P, _SZ, _P], _I32),
    "pmg_dense_backward": ([_P, _P, _P, _P, _I64, ctypes.POINTER(DenseTransition), _D, _I32, _I32, _D,
                            _P, _P, _P, _P, _P, _P, _SZ, _P], _I32),
    "pmg_joint_log_accumulate": ([_P, _P, _I64, _I32, _P, _P], _I32),
    "pmg_joint_log_workspace_size": ([_I64, _I32], _SZ),
    "pmg_joint_log_accumulate_ws": ([_P, _P, _I64, _I32, _P, _P, _SZ, _P], _I32),
    "pmg_dense_lpad": ([_I32], _I32),
    "pmg_dense_state": ([_P, _I64, _I32, _I32, _I32, _I64], _P),
    "pmg_dense_forward_phase": ([_P, _P, _P, _P, _I64, ctypes.POINTER(DenseTransition), _D, _I32, _I32, _D,
                                 _P, _P, _P, _P, _P, _SZ, _P, _I32], _I32),
    "pmg_dense_backward_phase": ([_P, _P, _P, _P, _I64, ctypes.POINTER(DenseTransition), _D, _I32, _I32, _D,
                                  _P, _P, _P, _P, _P, _P, _SZ, _P, _I32], _I32),
    "pmg_joint_accumulate": ([_P, _P, _I64, _I32, _P, _P, _SZ, _P], _I32),
    "pmg_tuning_softplus_batched": ([_P, _P, _I32, _I32, _I32, _I32, _P, _P, _P], _I32),
    "pmg_emission_range_flag": ([_P, _I64, _I32, _I32], _P),
    "pmg_mstep_batched_workspace_size": ([_I32, _I32, _I32, _I32, _I32], _SZ),
    "pmg_mstep_adam_batched_supported": ([_I32, _I32, _I32, _I32], ctypes.c_int),
    "pmg_mstep_adam_batched": ([_P, _P, _P, _P, _P, _P, _P, _I32, _I32, _I32, _I32, ctypes.POINTER(AdamCfg),
                                _P, _P, _P, _P, _SZ, _P], _I32),
    "pmg_emission_rowref_batched": ([_P, _I64, _I32, _I32, _D, _P, _P, _P], _I32),
    "pmg_fwdbwd_batched_workspace_size": ([_I64, _I32, _I32, _I32], _SZ),
    "pmg_forward_filter_batched": ([_P, _P, _P, _I64, _I32, ctypes.POINTER(Transition), _D, _I32, _I32, _D,
                                    _P, _P, _P, _P, _SZ, _P, _I32], _I32),
    "pmg_backward_smoother_batched": ([_P, _P, _P, _I64, _I32, ctypes.POINTER(Transition), _D, _I32, _I32, _D,
                                       _P, _P, _P, _SZ, _P, _I32], _I32),
}

_lib = None


def load(path: str | None = None):
    """Load (once) and return the library with typed entry points."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise NativeError(f"libpmg_hip.so not found at {p}; run __graft_entry__.build() "
                          "(make -C poor_man_gplvm_amd/csrc)")
    lib = ctypes.CDLL(p)
    for name, (argt, rest) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = argt
        fn.restype = rest
    if lib.pmg_abi_version() != ABI_VERSION:
        raise NativeError(f"ABI mismatch: library {lib.pmg_abi_version()} != {ABI_VERSION}")
    _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = load().pmg_last_error()
        raise NativeError(f"{what} failed (rc={rc}): {msg.decode() if msg else ''}")


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise NativeError("expected a device tensor")
    if not t.is_contiguous():
        raise NativeError("expected a contiguous tensor")
    return t.data_ptr()


def stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


class HostBuffer:
    """Page-locked host memory from pmg_host_alloc (first-touched by several threads as
    huge pages, then registered with HIP), exposed through the numpy array interface.
    When the last array viewing it goes away the block returns to a process-wide cache
    (at most HOST_CACHE_BYTES, least recently returned blocks evicted first), so repeated
    fits and decodes of one shape reuse their buffers instead of re-pinning (allocation
    ~4 ms and release ~20 ms per 410 MB)."""

    THREADS = max(1, min(8, os.cpu_count() or 1))

    def __init__(self, shape, dtype):
        self.nbytes = max(int(np.prod(shape, dtype=np.int64)) * np.dtype(dtype).itemsize, 1)
        self._lib = load()
        self.ptr = _host_cache_take(self.nbytes)
        if self.ptr is None:
            p = ctypes.c_void_p()
            check(self._lib.pmg_host_alloc(self.nbytes, self.THREADS, 1, ctypes.byref(p)), "pmg_host_alloc")
            self.ptr = p.value
        self.__array_interface__ = {'shape': tuple(int(s) for s in shape), 'typestr': np.dtype(dtype).str,
                                    'data': (self.ptr, False), 'version': 3}

    def __del__(self):
        ptr, self.ptr = getattr(self, 'ptr', None), None
        if ptr:
            _host_cache_give(ptr, self.nbytes, self._lib)


def _default_cache_bytes():
    """PMG_HOST_CACHE_BYTES, else min(2 GiB, 1/32 of the host's physical memory): page-locked
    memory cannot be swapped and every rank of a node holds its own cache."""
    env = os.environ.get("PMG_HOST_CACHE_BYTES")
    if env:
        return max(0, int(env))
    try:
        phys = os.sysconf("SC_PAGE_SIZE") * os.sysconf("SC_PHYS_PAGES")
    except (ValueError, OSError, AttributeError):
        phys = 64 << 30
    return int(min(2 << 30, phys // 32))


HOST_CACHE_BYTES = _default_cache_bytes()
_host_cache = []            # [(nbytes, ptr)], least recently returned first
_host_cache_total = 0
_host_cache_lock = threading.Lock()


def _host_cache_take(nbytes):
    global _host_cache_total
    with _host_cache_lock:
        for i in range(len(_host_cache) - 1, -1, -1):
            if _host_cache[i][0] == nbytes:
                _host_cache_total -= nbytes
                return _host_cache.pop(i)[1]
    return None


def _host_cache_give(ptr, nbytes, lib=None):
    """Return a block to the cache, evicting the least recently returned blocks to stay
    within HOST_CACHE_BYTES; a block larger than the cap is released at once."""
    global _host_cache_total
    evict = []
    with _host_cache_lock:
        if nbytes > HOST_CACHE_BYTES:
            evict.append((ptr, nbytes))
        else:
            while _host_cache and _host_cache_total + nbytes > HOST_CACHE_BYTES:
                n, p = _host_cache.pop(0)
                _host_cache_total -= n
                evict.append((p, n))
            _host_cache.append((nbytes, ptr))
            _host_cache_total += nbytes
    if evict:
        lib = lib or load()
        for p, n in evict:
            lib.pmg_host_free(p, n)
    return True


def host_cache_bytes():
    """Bytes of page-locked blocks held by the cache."""
    with _host_cache_lock:
        return _host_cache_total


def release_host_cache():
    """Unregister and unmap every cached page-locked block."""
    global _host_cache_total
    with _host_cache_lock:
        items = [(p, n) for n, p in _host_cache]
        _host_cache.clear()
        _host_cache_total = 0
    lib = load()
    for p, n in items:
        lib.pmg_host_free(p, n)


def host_array(shape, dtype) -> np.ndarray:
    """A page-locked numpy array (device->host copies into it run at full PCIe rate)."""
    return np.asarray(HostBuffer(shape, dtype))
