"""The C ABI library (libmums_hip.so): loads, exports every symbol include/mums.h declares,
host-only helpers agree with the oracle, and it refuses to compute without a GPU
(no CPU fallback)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "mums.h")).read()
    return sorted(set(re.findall(r"\b(mums_[a-z_0-9]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol(gpu_lib):
    lib = ctypes.CDLL(gpu_lib.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(gpu_lib.EXPORTED_SYMBOLS)
    assert lib.mums_abi_version() == 6


def test_seed_helpers_match_oracle(gpu_lib, oracle_mod):
    for w in range(0, 40):
        for r in range(0, 7):
            assert gpu_lib.getSeed(w, r) == oracle_mod.get_seed(w, r), (w, r)
    for n in [0, 1, 100, 10**5, 10**6, 10**7, 10**8, 3 * 10**9]:
        assert gpu_lib.getDefaultSeedWeight(n) == oracle_mod.lib().oracle_default_seed_weight(n)


def test_no_cpu_fallback_without_device(gpu_lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    with pytest.raises(gpu_lib.MumsError) as ei:
        gpu_lib.MemHash(0)
    assert ei.value.code == -6  # MUMS_E_NODEVICE


def test_null_context_is_rejected(gpu_lib):
    lib = gpu_lib.load_library()
    assert lib.mums_find(None) == -1
    assert lib.mums_set_seed(None, 0x7AC9AF) == -1
    assert lib.mums_ctx_create(0, None) == -1


def test_every_entry_point_has_argtypes(gpu_lib):
    """ctypes passes undeclared arguments as C int: a context pointer would be truncated."""
    lib = gpu_lib.load_library()
    missing = [s for s in gpu_lib.EXPORTED_SYMBOLS if s != "mums_abi_version" and getattr(lib, s).argtypes is None]
    assert not missing, missing
