"""CPU-side checks of the C-ABI library: it loads, exports every function include/*.h
declares, its host helpers match the oracle, and it fails loudly without a GPU."""
import ctypes
import os
import subprocess

import pytest

import oracle
from cryptmpi_2022_amd import _native as N
from cryptmpi_2022_amd import aead


def _exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_library_loads_and_exports_every_declared_symbol():
    L = N.lib()
    assert L.cmpi_version().startswith(b"cmpi_aead")
    exported = _exported(N.LIB_PATH)
    declared = [f for f in N.header_functions() if f.startswith("cmpi_")]
    assert declared, "no declarations parsed"
    missing = [f for f in declared if f not in exported]
    assert not missing, missing


def test_shim_exports_evp_symbols():
    shim = os.path.join(os.path.dirname(N.LIB_PATH), "libcmpi_evp.so")
    if not os.path.exists(shim):
        pytest.skip("EVP shim not built")
    exported = _exported(shim)
    declared = [f for f in N.header_functions() if f.startswith("EVP_")]
    missing = [f for f in declared if f not in exported]
    assert not missing, missing


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", N.LIB_PATH], capture_output=True, text=True)
    assert ".hip_fatbin" in out.stdout
    with open(N.LIB_PATH, "rb") as f:
        assert b"amdgcn-amd-amdhsa--gfx950" in f.read()


@pytest.mark.parametrize("iv,cter", [
    (bytes(range(16)), 0x01020304), (b"\xff" * 16, 1), (bytes(15) + b"\x01", 0xFFFFFFFF),
    (bytes(16), (1 << 40) + 5), (bytes.fromhex("000102030405060708090a0b0c0dfeff"), 0xFFFFFF02),
])
def test_iv_count_matches_oracle(iv, cter):
    assert aead.iv_count(iv, cter) == oracle.iv_count(iv, cter)
    b = (ctypes.c_uint8 * 16)()
    N.lib().cmpi_iv_count_out(b, cter, (ctypes.c_uint8 * 16).from_buffer_copy(iv))
    assert bytes(b) == oracle.iv_count(iv, cter)


def test_no_gpu_fails_loudly():
    try:
        import torch

        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(N.CmpiError):
        aead.AeadCtx(b"\x00" * 16)
    assert "device" in N.last_error()


def test_bad_key_length_rejected():
    h = N.lib().cmpi_ctx_new(N.CMPI_AES_128_GCM, b"short", 5, 0, 0)
    assert not h and "16" in N.last_error()
