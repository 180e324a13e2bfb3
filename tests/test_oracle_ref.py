"""Oracle pin against the reference itself: IV_Count / IV_Count_out compiled from
MV/src/mpi/pt2pt/send.c:1019-1041 as they lie under /root/reference (oracle/Makefile cuts the two
function bodies into the git-ignored oracle/_ref/ and builds them unchanged).  The oracle's
restatement (oracle/ctr_ref.c) and the engine's host helper (cmpi_iv_count / _out) must agree
with it bit for bit over the carry corners CryptMPI's counters reach (702 stream offsets
send.c:1789-1808, the 32-bit truncation of `cter`)."""
import ctypes
import os
import random

import pytest

import oracle
from cryptmpi_2022_amd import _native as N

REF = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "libivcount_ref.so")
pytestmark = pytest.mark.skipif(not os.path.exists(REF), reason="oracle/_ref not built (no /root/reference here)")


def _ref():
    L = ctypes.CDLL(REF)
    L.IV_Count.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
    L.IV_Count_out.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p]
    return L


def _cases():
    rng = random.Random(1019)
    ivs = [bytes(16), b"\xff" * 16, bytes(15) + b"\xff", b"\x00" * 12 + b"\xff\xff\xff\xf0", b"\x7f" + b"\xff" * 15,
           bytes(range(16)), bytes(range(0xF0, 0x100))]
    ivs += [bytes(rng.randrange(256) for _ in range(16)) for _ in range(40)]
    cters = [0, 1, 15, 16, 255, 256, 0xFFFF, 0x10000, 0xFFFFFFFF, 0xFFFFFFF0, 1 << 32, (1 << 32) + 5, (1 << 40) + 7,
             0xFFFFFFFFFFFFFFFF, 4096, 65536 // 16, (8 << 20) // 16]
    cters += [rng.randrange(1 << 64) for _ in range(40)] + [rng.randrange(1 << 32) for _ in range(40)]
    return [(iv, c) for iv in ivs for c in cters]


def test_iv_count_reference_vs_oracle_and_engine():
    L = _ref()
    for iv, cter in _cases():
        b = (ctypes.c_uint8 * 16).from_buffer_copy(iv)
        L.IV_Count(b, cter)
        want = bytes(b)
        assert oracle.iv_count(iv, cter) == want, (iv.hex(), cter)
        e = (ctypes.c_uint8 * 16).from_buffer_copy(iv)
        N.lib().cmpi_iv_count(e, cter)
        assert bytes(e) == want, (iv.hex(), cter)


def test_iv_count_out_reference_vs_engine():
    L = _ref()
    for iv, cter in _cases()[::7]:
        src = (ctypes.c_uint8 * 16).from_buffer_copy(iv)
        dst = (ctypes.c_uint8 * 16)()
        L.IV_Count_out(dst, cter, src)
        want = bytes(dst)
        e = (ctypes.c_uint8 * 16)()
        N.lib().cmpi_iv_count_out(e, cter, (ctypes.c_uint8 * 16).from_buffer_copy(iv))
        assert bytes(e) == want
        assert want == oracle.iv_count(iv, cter)
