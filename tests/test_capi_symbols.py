"""The C ABI library loads (no GPU needed) and exports every entry point that
include/pmg.h declares."""
import ctypes
import os
import re

from poor_man_gplvm_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, 'include', 'pmg.h')).read()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    return sorted(set(re.findall(r'\b(pmg_[a-z0-9_]+)\s*\(', txt)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(_native.EXPORTED_SYMBOLS)


def test_library_exports_all_declared_symbols():
    lib = ctypes.CDLL(_native.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_abi_version_and_workspace_queries():
    lib = _native.load()
    assert lib.pmg_abi_version() == _native.ABI_VERSION
    assert lib.pmg_fwdbwd_workspace_size(100000, 512, 49) > 0
    assert lib.pmg_fwdbwd_workspace_size(100, 2000, 32) == 0        # L > 1024 unsupported
    assert lib.pmg_emission_workspace_size(1000, 100, 30) > 4 * 128 * 32
    assert lib.pmg_suffstats_workspace_size(1000, 100, 64) > 0
    assert lib.pmg_joint_workspace_size(1000, 100) > 0
    assert lib.pmg_mstep_workspace_size(512, 1000) > 0
    # the log-domain joint's split partials: only where the joint splits in time
    # (the workspace was sized for 8 splits even where none runs)
    assert lib.pmg_joint_log_workspace_size(100000, 1024) == 0      # 32 x 32 tiles fill the chip
    assert lib.pmg_joint_log_workspace_size(100000, 2048) == 0
    assert lib.pmg_joint_log_workspace_size(100000, 512) == 4 * 1024 * 1024 * 16 + 256
    assert lib.pmg_joint_log_workspace_size(100000, 64) == 8 * 128 * 128 * 16 + 256
    assert lib.pmg_joint_log_workspace_size(200, 64) == 0            # too short to split


def test_invalid_arguments_are_rejected_without_gpu():
    lib = _native.load()
    rc = lib.pmg_spikes_prepare(None, 0, 0, None, 0, None, 0, None, None, 0, None, None)
    assert rc == -1
    assert b'T=0' in lib.pmg_last_error()


def test_zero_byte_copy_is_a_no_op():
    """pmg_copy_d2h of 0 bytes succeeds whatever the pointers (an empty tensor's data
    pointer is NULL) and touches no device."""
    lib = _native.load()
    assert lib.pmg_copy_d2h(None, None, 0, None) == 0
    assert lib.pmg_copy_d2h(None, None, 8, None) == -1
