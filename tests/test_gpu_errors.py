"""The C ABI reports only the HIP errors its own calls cause ("What's weak" 1).

HIP keeps a per-thread "last error".  Before round 5 every launch was checked with
hipGetLastError(), which returns (and clears) the last error of ANY earlier HIP call: a caller's
unrelated failure made the next seal fail — under the EVP shim a failed seal returns 0 with the
output zero-filled, and CryptMPI ignores the return (send.c:311), so the wire would carry zeros —
and the caller lost its own error.  BoringSSL fails a seal only for its own reasons
(aead.h:251-253).

Each test here provokes a HIP error in the calling thread first (hipSetDevice on a device that
does not exist), then calls an entry point of the library, and expects: success, output
bit-exact against the oracle, and the caller's error still pending afterwards
(hipPeekAtLastError).  Buffers are prepared before the error is provoked and read back after it
is cleared, so that torch's own launch checks never see it."""
import ctypes
import os
import subprocess

import numpy as np
import pytest
import torch

import oracle
from cryptmpi_2022_amd import aead, ctrmode
from cryptmpi_2022_amd.synth import random_nonces, splitmix64_bytes
from tests.gpu_util import dev, empty, host, status_buf

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEY = bytes.fromhex("000102030405060708090a0b0c0d0e0f")
IV32 = splitmix64_bytes(0x702E, 32).tobytes()

_hip = ctypes.CDLL("libamdhip64.so.7")  # the instance torch (and libcmpi_aead.so) bound to
for _f in ("hipSetDevice", "hipPeekAtLastError", "hipGetLastError"):
    getattr(_hip, _f).restype = ctypes.c_int


def provoke() -> int:
    """A caller-side HIP error, left pending in this thread."""
    _hip.hipGetLastError()
    code = _hip.hipSetDevice(9999)
    assert code != 0 and _hip.hipPeekAtLastError() == code
    return code


@pytest.fixture(autouse=True)
def _clear_after():
    torch.cuda.synchronize()
    yield
    _hip.hipGetLastError()
    torch.cuda.synchronize()


def still_pending(code: int) -> None:
    got = _hip.hipPeekAtLastError()
    _hip.hipGetLastError()  # clear before torch looks
    assert got == code, f"caller's HIP error {code} not preserved (now {got})"


@pytest.mark.parametrize("n,nrec", [(1024, 64), (1 << 20, 2), (1000, 3)])
def test_gcm_device_batches(n, nrec):
    """Lane kernel (1 KiB x 64), flow kernel + combine (1 MiB x 2), short-record flow (1000 B)."""
    ctx = aead.AeadCtx(KEY)
    pt = splitmix64_bytes(0xE1 + n, n * nrec).reshape(nrec, n)
    nonces = random_nonces(0xE2, nrec)
    d_pt, d_n = dev(pt), dev(nonces)
    ct = empty(nrec * (n + 16), fill=0xAA)
    back = empty(nrec * n, fill=0xAA)
    st = status_buf(nrec)
    torch.cuda.synchronize()
    code = provoke()
    ctx.seal_batch(ct, d_pt, d_n, n, nrec)
    ctx.open_batch(back, ct, d_n, n, nrec, status=st)
    still_pending(code)
    got = host(ct)[: nrec * (n + 16)].reshape(nrec, n + 16)
    for i in range(nrec):
        assert got[i].tobytes() == oracle.gcm_seal(KEY, nonces[i].tobytes(), pt[i].tobytes()), i
    assert host(back)[: nrec * n].tobytes() == pt.tobytes()
    assert (host(st)[:nrec] == 1).all()


@pytest.mark.parametrize("n", [4096, 200000])
def test_gcm_host_paths(n):
    """The *_host entry points on pageable and on page-locked (registered) buffers: the pointer
    classification (hipPointerGetAttributes fails on pageable memory) must not clear or replace
    the caller's error."""
    ctx = aead.AeadCtx(KEY)
    nrec = 3
    pt = splitmix64_bytes(0xE3 + n, n * nrec).reshape(nrec, n)
    nonces = random_nonces(0xE4, nrec)
    code = provoke()
    ct = ctx.seal_host_batch(nonces, pt)
    back, st = ctx.open_host_batch(nonces, ct)
    still_pending(code)
    for i in range(nrec):
        assert ct[i].tobytes() == oracle.gcm_seal(KEY, nonces[i].tobytes(), pt[i].tobytes()), i
    assert back.tobytes() == pt.tobytes() and (st == 1).all()
    # page-locked: register the caller's buffers, as an MPI library's registration cache does
    ptp = torch.from_numpy(pt.copy()).pin_memory().numpy()
    code = provoke()
    ct2 = ctx.seal_host_batch(nonces, ptp)
    still_pending(code)
    assert ct2.tobytes() == ct.tobytes()


def test_served_single_message():
    """The resident message service (cmpi_service_start) serving one 64 KiB host message."""
    ctx = aead.AeadCtx(KEY)
    ctx.service_start(20000)
    try:
        pt = splitmix64_bytes(0xE5, 65536).tobytes()
        nonce = random_nonces(0xE6, 1)[0].tobytes()
        code = provoke()
        ct = ctx.seal(nonce, pt)
        back = ctx.open(nonce, ct)
        still_pending(code)
        assert ct == oracle.gcm_seal(KEY, nonce, pt)
        assert back == pt
    finally:
        ctx.service_stop()


def test_ctr_and_ecb():
    """cmpi_ctr_xor (config 4's kernel) and cmpi_ecb_encrypt (the 602 sub-key, send.c:583)."""
    c = aead.CipherCtx(KEY, "aes-128-ctr")
    e = aead.CipherCtx(KEY, "aes-128-ecb")
    n = 100003
    data = splitmix64_bytes(0xE7, n)
    iv = splitmix64_bytes(0xE8, 16).tobytes()
    d_in, out = dev(data), empty(n, fill=0)
    blocks = splitmix64_bytes(0xE9, 64)
    d_b, eout = dev(blocks), empty(64, fill=0)
    torch.cuda.synchronize()
    code = provoke()
    c.ctr_xor(out, d_in, n, iv)
    e.ecb_encrypt(eout, d_b, 4)
    still_pending(code)
    assert host(out)[:n].tobytes() == oracle.ctr_xor(KEY, iv, data.tobytes())
    assert host(eout)[:64].tobytes() == b"".join(oracle.ecb_encrypt(KEY, blocks[16 * i:16 * i + 16].tobytes())
                                                  for i in range(4))


@pytest.mark.parametrize("served", [False, True])
def test_702_sender(served):
    """cmpi_702_sender_new (the round-4 failure: it reported an earlier NUMA query's error) and a
    send through it, launched and served."""
    c = aead.CipherCtx(KEY, "aes-128-ctr")
    if served:
        c.service_start(20000)
    try:
        n = 5000
        pt = splitmix64_bytes(0xEA, n)
        d_pt, out = dev(pt), empty(n, fill=0)
        torch.cuda.synchronize()
        code = provoke()
        s = ctrmode.Sender702(c, IV32, ring_bytes=1 << 20, series_threads=4)
        hdr, nseg = s.send(out, d_pt, n)
        still_pending(code)
        o = oracle.Sender702(KEY, IV32, max_bytes=1 << 20, series=4)
        ohdr, oct_ = o.send(pt.tobytes(), pending=0)
        assert hdr == ohdr
        assert host(out)[:n].tobytes() == oct_
        s.close()
    finally:
        if served:
            c.service_stop()


@pytest.mark.parametrize("service", [False, True])
def test_evp_shim_client(tmp_path, service):
    """tests/evp_client.c (CryptMPI's naive-Alltoall, 602 sub-key and CTR call sites through the
    BoringSSL-ABI drop-in) with CMPI_TEST_PROVOKE_HIP_ERROR: the client provokes a HIP error
    before its first EVP call and checks after its last one that the error is still pending."""
    shim_dir = os.path.join(ROOT, "cryptmpi_2022_amd")
    exe = tmp_path / "evp_client"
    subprocess.check_call(["gcc", "-O1", "-o", str(exe), os.path.join(ROOT, "tests", "evp_client.c"),
                           f"-L{shim_dir}", "-lcmpi_evp", f"-Wl,-rpath,{shim_dir}", "-ldl"])
    p, n = 4, 3000
    key = splitmix64_bytes(0xEB, 16).tobytes()
    nonces = random_nonces(0xEC, p)
    send = splitmix64_bytes(0xED, n * p)
    inp = tmp_path / "in.bin"
    inp.write_bytes(key + nonces.tobytes() + send.tobytes())
    outp = tmp_path / "out.bin"
    env = dict(os.environ, CMPI_TEST_PROVOKE_HIP_ERROR="1")
    env["CMPI_EVP_SERVICE_US"] = "2000" if service else "0"  # 0: a kernel launch per call
    r = subprocess.run([str(exe), str(p), str(n), str(inp), str(outp)], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 0, (r.returncode, r.stderr)
    assert "caller error preserved" in r.stderr, r.stderr
    out = outp.read_bytes()
    for i in range(p):
        rec = out[i * (n + 28):(i + 1) * (n + 28)]
        assert rec[12:] == oracle.gcm_seal(key, nonces[i].tobytes(), send[i * n:(i + 1) * n].tobytes())
