"""The BoringSSL-ABI drop-in (libcmpi_evp.so, include/cmpi_evp.h): a C program written like
CryptMPI's naive Alltoall + CTR + 602 sub-key call sites, linked against the shim instead of
libcrypto, must produce the oracle's bytes.  Also exercised directly through ctypes."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import oracle
from cryptmpi_2022_amd import _native as N
from cryptmpi_2022_amd.synth import random_nonces, splitmix64_bytes

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "cryptmpi_2022_amd", "libcmpi_evp.so")


@pytest.mark.parametrize("service", [False, True])
@pytest.mark.parametrize("p,n", [(8, 4096), (3, 1001), (2, 0)])
def test_c_client_naive_alltoall(tmp_path, p, n, service):
    """The C client of CryptMPI's call sites; with CMPI_EVP_SERVICE_US the AEAD seals and the CTR
    EncryptUpdates (the second one starting mid-block) are served by the contexts' resident kernels."""
    exe = tmp_path / "evp_client"
    subprocess.check_call(["gcc", "-O1", "-o", str(exe), os.path.join(ROOT, "tests", "evp_client.c"),
                           f"-L{os.path.dirname(SHIM)}", "-lcmpi_evp", f"-Wl,-rpath,{os.path.dirname(SHIM)}"])
    key = splitmix64_bytes(0xAB, 16).tobytes()
    nonces = random_nonces(0xAC, p)
    send = splitmix64_bytes(0xAD, n * p)
    inp = tmp_path / "in.bin"
    inp.write_bytes(key + nonces.tobytes() + send.tobytes())
    outp = tmp_path / "out.bin"
    env = dict(os.environ)
    env["CMPI_EVP_SERVICE_US"] = "2000" if service else "0"  # 0: a kernel launch per call
    r = subprocess.run([str(exe), str(p), str(n), str(inp), str(outp)], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 0, (r.returncode, r.stderr)
    out = outp.read_bytes()
    wire_len = (n + 28) * p
    wire = out[:wire_len]
    for i in range(p):
        rec = wire[i * (n + 28):(i + 1) * (n + 28)]
        assert rec[:12] == nonces[i].tobytes()
        assert rec[12:] == oracle.gcm_seal(key, nonces[i].tobytes(), send[i * n:(i + 1) * n].tobytes())
    assert out[wire_len:wire_len + n * p] == send.tobytes()
    newkey = out[wire_len + n * p: wire_len + n * p + 16]
    v = nonces[0].tobytes() + nonces[0].tobytes()[:4]
    assert newkey == oracle.ecb_encrypt(key, v)
    iv = nonces[0].tobytes() + b"\xff" * 4
    assert out[wire_len + n * p + 16:] == oracle.ctr_xor(key, iv, send.tobytes())


def test_ctypes_seal_open_semantics():
    L = ctypes.CDLL(SHIM)
    P, S = ctypes.c_void_p, ctypes.c_size_t
    L.EVP_aead_aes_128_gcm.restype = P
    L.EVP_AEAD_CTX_new.restype = P
    L.EVP_AEAD_CTX_new.argtypes = [P, P, S, S]
    for f in (L.EVP_AEAD_CTX_seal, L.EVP_AEAD_CTX_open):
        f.argtypes = [P, P, ctypes.POINTER(S), S, P, S, P, S, P, S]
    L.EVP_AEAD_CTX_free.argtypes = [P]
    key = bytes(range(16))
    ctx = L.EVP_AEAD_CTX_new(L.EVP_aead_aes_128_gcm(), key, 16, 0)
    assert ctx
    nonce, pt = bytes(range(12)), splitmix64_bytes(5, 333).tobytes()
    out = ctypes.create_string_buffer(333 + 16)
    olen = S(0)
    assert L.EVP_AEAD_CTX_seal(ctx, out, ctypes.byref(olen), 349, nonce, 12, pt, 333, None, 0) == 1
    assert olen.value == 349 and out.raw == oracle.gcm_seal(key, nonce, pt)
    # max_out_len too small -> 0, out zeroed, out_len 0
    small = ctypes.create_string_buffer(b"\x11" * 100)
    assert L.EVP_AEAD_CTX_seal(ctx, small, ctypes.byref(olen), 100, nonce, 12, pt, 333, None, 0) == 0
    assert small.raw == bytes(100) + b"\x00" and olen.value == 0
    # open ok / forged
    back = ctypes.create_string_buffer(333)
    assert L.EVP_AEAD_CTX_open(ctx, back, ctypes.byref(olen), 333, nonce, 12, out.raw, 349, None, 0) == 1
    assert back.raw[:333] == pt and olen.value == 333
    forged = bytearray(out.raw)
    forged[-1] ^= 1
    assert L.EVP_AEAD_CTX_open(ctx, back, ctypes.byref(olen), 333, nonce, 12, bytes(forged), 349, None, 0) == 0
    assert back.raw[:333] == bytes(333) and olen.value == 0
    # AAD is not supported by the drop-in (CryptMPI never passes any)
    assert L.EVP_AEAD_CTX_seal(ctx, out, ctypes.byref(olen), 349, nonce, 12, pt, 333, b"ad", 2) == 0
    # rejected inputs (aead.h:251-253, :276-278): an input shorter than the tag, a nonce of other
    # than 12 bytes, an output too small for the plaintext — 0, out zeroed, out_len 0
    back = ctypes.create_string_buffer(b"\x22" * 333)
    olen.value = 5
    assert L.EVP_AEAD_CTX_open(ctx, back, ctypes.byref(olen), 333, nonce, 12, out.raw[:15], 15, None, 0) == 0
    assert back.raw[:333] == bytes(333) and olen.value == 0
    assert L.EVP_AEAD_CTX_seal(ctx, out, ctypes.byref(olen), 349, nonce, 8, pt, 333, None, 0) == 0
    assert out.raw[:349] == bytes(349) and olen.value == 0
    assert L.EVP_AEAD_CTX_seal(ctx, out, ctypes.byref(olen), 349, nonce, 12, pt, 333, None, 0) == 1
    assert L.EVP_AEAD_CTX_open(ctx, back, ctypes.byref(olen), 332, nonce, 12, out.raw, 349, None, 0) == 0
    assert back.raw[:332] == bytes(332) and olen.value == 0
    # the empty message: tag only
    tag = ctypes.create_string_buffer(16)
    assert L.EVP_AEAD_CTX_seal(ctx, tag, ctypes.byref(olen), 16, nonce, 12, b"", 0, None, 0) == 1
    assert olen.value == 16 and tag.raw[:16] == oracle.gcm_seal(key, nonce, b"")
    assert L.EVP_AEAD_CTX_open(ctx, back, ctypes.byref(olen), 0, nonce, 12, tag.raw[:16], 16, None, 0) == 1
    assert olen.value == 0
    ftag = bytearray(tag.raw[:16])
    ftag[7] ^= 0x40
    assert L.EVP_AEAD_CTX_open(ctx, back, ctypes.byref(olen), 0, nonce, 12, bytes(ftag), 16, None, 0) == 0
    L.EVP_AEAD_CTX_free(ctx)


@pytest.mark.parametrize("threads,msgs,n,service", [(8, 16, 4096, False), (8, 4, 65536, False), (3, 5, 1001, False),
                                                    (8, 2, 0, False), (1, 24, 4096, True), (8, 4, 65536, True)])
def test_c_client_threads_share_one_ctx(tmp_path, threads, msgs, n, service):
    """An OpenMP-style team of pthreads sealing and opening on ONE shared EVP_AEAD_CTX through the
    drop-in (coalesced into batch launches), bit-exact vs the oracle; per-message 602 contexts
    (T x EVP_AEAD_CTX_new of a fresh key per message, pooled + re-keyed on the device); libcrypto's
    EVP_aes_256_ecb forwarded by the shim, not misread."""
    import json

    exe = tmp_path / "evp_mt_client"
    subprocess.check_call(["gcc", "-O1", "-o", str(exe), os.path.join(ROOT, "tests", "evp_mt_client.c"),
                           f"-L{os.path.dirname(SHIM)}", "-lcmpi_evp", "-lcrypto", "-lpthread",
                           f"-Wl,-rpath,{os.path.dirname(SHIM)}"])
    R = threads * msgs
    key = splitmix64_bytes(0xBB, 16).tobytes()
    nonces = random_nonces(0xBC, R)
    pt = splitmix64_bytes(0xBD, n * R)
    inp, outp = tmp_path / "in.bin", tmp_path / "out.bin"
    inp.write_bytes(key + nonces.tobytes() + pt.tobytes())
    env = dict(os.environ)
    # single messages served by each context's resident kernel, or a kernel launch per call
    env["CMPI_EVP_SERVICE_US"] = "2000" if service else "0"
    r = subprocess.run([str(exe), str(threads), str(msgs), str(n), str(inp), str(outp)], capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["forwarded_aes256_ok"] == 1
    out = outp.read_bytes()
    for i in range(R):
        got = out[i * (n + 16):(i + 1) * (n + 16)]
        assert got == oracle.gcm_seal(key, nonces[i].tobytes(), pt[i * n:(i + 1) * n].tobytes()), i
    assert out[R * (n + 16):] == oracle.ecb_encrypt(key, bytes((7 * i) & 0xFF for i in range(16)))
    print("evp_mt", json.dumps(rec))
