"""The host pipeline's copy modes (cmpi_debug_set_host_out_direct): 0 hipMemcpyAsync both ways,
1 the kernel writes the page-locked outputs, 4 the D2H on an SDMA engine through HSA, 5 both
directions through HSA with the host launching each chunk's kernel (the default).  Every mode on
page-locked inputs, outputs and nonces over many chunks (ragged last chunk, 2-4 staging slots):
ciphertext and tags bit-exact against the oracle, forged records reported per record and
zero-filled, open round trip; and the cases mode 5 hands back to the others (pageable input, a
gapped output, one chunk)."""
import ctypes

import numpy as np
import pytest

import oracle
from cryptmpi_2022_amd import aead
from cryptmpi_2022_amd.synth import random_nonces, records

pytestmark = pytest.mark.gpu
KEY = bytes(range(16))
L = aead.N.lib


def _pinned(a: np.ndarray):
    """a copy of `a` in its own page-aligned, registered buffer (numpy view, handle to free)."""
    raw = np.zeros(a.nbytes + 8192, np.uint8)
    off = (-raw.ctypes.data) % 4096
    v = raw[off: off + a.nbytes].view(a.dtype).reshape(a.shape)
    v[...] = a
    assert L().cmpi_host_register(v.ctypes.data, max(v.nbytes, 1)) == 0
    return v, raw


@pytest.fixture(autouse=True)
def _restore():
    yield
    L().cmpi_debug_set_host_out_direct(5)
    L().cmpi_debug_set_host_chunk(0)
    L().cmpi_debug_set_host_slots(3)


@pytest.mark.parametrize("slots", [2, 3, 4])
@pytest.mark.parametrize("mode", [0, 1, 4, 5])
@pytest.mark.parametrize("alg", ["aes-128-gcm", "aes-128-ocb"])
def test_copy_modes_pinned(alg, mode, slots):
    n, nrec = 1000, 1201  # chunks of 64 KiB: 19 chunks, the last one ragged
    pt = records(0x6600 + mode, nrec, n)
    nonces = random_nonces(0x6601 + slots, nrec)
    seal = oracle.gcm_seal_batch if alg == "aes-128-gcm" else oracle.ocb_seal_batch
    want = seal(KEY, nonces, pt)
    ctx = aead.AeadCtx(KEY, alg)
    lib = L()
    lib.cmpi_debug_set_host_out_direct(mode)
    lib.cmpi_debug_set_host_chunk(64 * 1024)
    lib.cmpi_debug_set_host_slots(slots)
    p_pt, _r1 = _pinned(pt)
    p_n, _r2 = _pinned(nonces)
    p_ct, _r3 = _pinned(np.zeros((nrec, n + 16), np.uint8))
    p_back, _r4 = _pinned(np.full((nrec, n), 0x77, np.uint8))
    st = (ctypes.c_int32 * nrec)()
    f_seal = lib.cmpi_gcm_seal_host if alg == "aes-128-gcm" else lib.cmpi_ocb_seal_host
    f_open = lib.cmpi_gcm_open_host if alg == "aes-128-gcm" else lib.cmpi_ocb_open_host
    try:
        for rep in range(2):  # the second call reuses the slots, signals and streams
            p_ct[...] = 0
            aead.N.check(f_seal(ctx.handle, p_ct.ctypes.data, n + 16, p_pt.ctypes.data, n, p_n.ctypes.data, 12, n, nrec))
            assert np.array_equal(p_ct, want), (mode, slots, rep)
        aead.N.check(f_open(ctx.handle, p_back.ctypes.data, n, p_ct.ctypes.data, n + 16, p_n.ctypes.data, 12, n, nrec, st))
        assert np.array_equal(p_back, pt) and all(s == 1 for s in st)
        bad = [0, 600, 1200]
        p_ct[bad, n + 15] ^= 1
        rc = f_open(ctx.handle, p_back.ctypes.data, n, p_ct.ctypes.data, n + 16, p_n.ctypes.data, 12, n, nrec, st)
        assert rc == aead.N.CMPI_EAUTH
        assert [i for i in range(nrec) if st[i] == 0] == bad
        assert (p_back[bad] == 0).all()
        good = np.setdiff1d(np.arange(nrec), bad)
        assert np.array_equal(p_back[good], pt[good])
    finally:
        for v in (p_pt, p_n, p_ct, p_back):
            lib.cmpi_host_unregister(v.ctypes.data)


@pytest.mark.parametrize("case", ["pageable_in", "gapped_out", "one_chunk", "pageable_nonces"])
def test_copy_mode5_hands_back(case):
    """Inputs mode 5 does not take (it needs page-locked records, outputs and nonces and more than
    one chunk) still seal bit-exact through the modes it hands them to."""
    n, nrec = 1000, 301
    pt = records(0x6700, nrec, n)
    nonces = random_nonces(0x6701, nrec)
    want = oracle.gcm_seal_batch(KEY, nonces, pt)
    ctx = aead.AeadCtx(KEY)
    lib = L()
    lib.cmpi_debug_set_host_out_direct(5)
    lib.cmpi_debug_set_host_chunk(0 if case == "one_chunk" else 64 * 1024)
    pad = 28 if case == "gapped_out" else 0
    ostride = n + 16 + pad
    src = pt if case == "pageable_in" else None
    regs = []
    try:
        if src is None:
            src, _r = _pinned(pt)
            regs.append(src)
        nn = nonces
        if case != "pageable_nonces":
            nn, _r2 = _pinned(nonces)
            regs.append(nn)
        out, _r3 = _pinned(np.full((nrec, ostride), 0x5A, np.uint8))
        regs.append(out)
        aead.N.check(lib.cmpi_gcm_seal_host(ctx.handle, out.ctypes.data, ostride, src.ctypes.data, n, nn.ctypes.data, 12, n, nrec))
        assert np.array_equal(out[:, : n + 16], want)
        assert (out[:, n + 16:] == 0x5A).all()
    finally:
        for v in regs:
            lib.cmpi_host_unregister(v.ctypes.data)
