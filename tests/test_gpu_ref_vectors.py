"""The engine against known answers held by the reference itself (tests/golden/ref_bssl_vectors.json,
extracted from MVAPICH/cryptMPI-mvapich2-2.3.3/boringssl-master.tar.xz by
tests/golden/extract_ref_vectors.py; the CPU pins of the oracle are tests/test_oracle_ref_vectors.py):

* decrepit/cfb/cfb_test.cc:30-46 (SP 800-38A F.3.13, CFB128): C_i = P_i ^ AES_K(C_{i-1}), C_0 = IV —
  four AES-128 forward-cipher answers, through the ECB kernel (cmpi_ecb_encrypt) and the CTR kernel
  (counter block = C_{i-1}: ctr_xor(P_i) = C_i);
* the FIPS self-test answers of that BoringSSL build (bcm.c.o kAESCBCCiphertext, kAESGCMCiphertext)
  for the calls of fipstools/test_fips.c:70-82 and :97-117 — AES-CBC under a zero IV through the ECB
  kernel, and EVP_AEAD_CTX_seal(kAESKey, 12 zero nonce bytes, 64-byte kPlaintext, no AD) through
  every GCM path of the engine: the lane kernel at each lane width, the flow kernel, a config-2-sized
  batch of the record, the host path, the resident service, the 602 device-keyed sub-key context
  (K' = AES_K0(V) derived on the device with V chosen so that K' is the KAT key) and the BoringSSL-ABI
  drop-in libcmpi_evp.so.  Open is checked on each, and a forged tag is rejected with zero-fill."""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle
from cryptmpi_2022_amd import _native as N
from cryptmpi_2022_amd import aead
from tests.gpu_util import dev, empty, host, status_buf

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "cryptmpi_2022_amd", "libcmpi_evp.so")
DIRECT_DEFAULT = (2 << 20) + 64  # cmpi_aead.hip g_host_direct

with open(os.path.join(ROOT, "tests", "golden", "ref_bssl_vectors.json")) as _f:
    REF = json.load(_f)
CFB = REF["cfb128_f3_13"]
KAT = REF["fips_kat"]
KAT_KEY = bytes.fromhex(KAT["key"])
KAT_NONCE = bytes.fromhex(KAT["gcm_nonce"])
KAT_PT = bytes.fromhex(KAT["plaintext"])
KAT_OUT = bytes.fromhex(KAT["gcm_ct_tag"])


def _xor(a: bytes, b: bytes) -> bytes:
    return bytes(x ^ y for x, y in zip(a, b))


@pytest.fixture(autouse=True)
def _auto_plan():
    aead.force_plan(0, 0)
    aead.force_wide(0, 0)
    yield
    aead.force_plan(0, 0)
    aead.force_wide(0, 0)
    aead.set_flow_one_wg(True)
    N.lib().cmpi_debug_set_host_direct(DIRECT_DEFAULT)


# ------------------------------------------------------------------ AES forward cipher (CFB, CBC)
def test_cfb128_via_ecb_kernel():
    key, iv = bytes.fromhex(CFB["key"]), bytes.fromhex(CFB["iv"])
    pt, ct = bytes.fromhex(CFB["plaintext"]), bytes.fromhex(CFB["ciphertext"])
    inputs = iv + ct[:48]  # C_0 .. C_3
    ctx = aead.CipherCtx(key, "aes-128-ecb")
    out = empty(64, fill=0xAA)
    ctx.ecb_encrypt(out, dev(np.frombuffer(inputs, np.uint8)), 4)
    ks = host(out)[:64].tobytes()
    assert _xor(pt, ks) == ct  # C_i = P_i ^ E_K(C_{i-1})


def test_cfb128_via_ctr_kernel():
    key, iv = bytes.fromhex(CFB["key"]), bytes.fromhex(CFB["iv"])
    pt, ct = bytes.fromhex(CFB["plaintext"]), bytes.fromhex(CFB["ciphertext"])
    ctx = aead.CipherCtx(key, "aes-128-ctr")
    prev = iv
    for i in range(4):
        out = empty(16, fill=0xAA)
        ctx.ctr_xor(out, dev(np.frombuffer(pt[16 * i:16 * i + 16], np.uint8)), 16, prev)
        got = host(out)[:16].tobytes()
        assert got == ct[16 * i:16 * i + 16], i
        prev = got
    # the keystream entry point too: E_K(C_{i-1}) one block at a time
    for i, c in enumerate([iv, ct[:16], ct[16:32], ct[32:48]]):
        out = empty(16, fill=0xAA)
        ctx.keystream(out, 1, c)
        assert _xor(host(out)[:16].tobytes(), pt[16 * i:16 * i + 16]) == ct[16 * i:16 * i + 16]


def test_fips_cbc_via_ecb_kernel():
    """AES-CBC (test_fips.c:70-82, zero IV): E_K(P_i ^ C_{i-1}) = C_i for the four blocks at once."""
    key, iv = bytes.fromhex(KAT["key"]), bytes.fromhex(KAT["iv"])
    pt, ct = bytes.fromhex(KAT["plaintext"]), bytes.fromhex(KAT["cbc_ciphertext"])
    chained = b"".join(_xor(pt[16 * i:16 * i + 16], (iv + ct)[16 * i:16 * i + 16]) for i in range(4))
    ctx = aead.CipherCtx(key, "aes-128-ecb")
    out = empty(64, fill=0xAA)
    ctx.ecb_encrypt(out, dev(np.frombuffer(chained, np.uint8)), 4)
    assert host(out)[:64].tobytes() == ct


# ------------------------------------------------------------------------ AES-128-GCM (FIPS KAT)
def _seal_open_batch(ctx, nrec: int):
    n = len(KAT_PT)
    pt = np.tile(np.frombuffer(KAT_PT, np.uint8), nrec)
    nonces = np.tile(np.frombuffer(KAT_NONCE, np.uint8), nrec)
    out = empty(nrec * (n + 16), fill=0xAA)
    ctx.seal_batch(out, dev(pt), dev(nonces), n, nrec)
    ct = host(out)[: nrec * (n + 16)].reshape(nrec, n + 16)
    forged = ct.copy()
    forged[nrec // 2, -1] ^= 0x01
    back = empty(nrec * n, fill=0xAA)
    st = status_buf(nrec)
    ctx.open_batch(back, dev(forged), dev(nonces), n, nrec, status=st)
    return ct, host(back)[: nrec * n].reshape(nrec, n), host(st)[:nrec]


@pytest.mark.parametrize("plan", [(0, 0), (1, 1), (2, 1), (4, 1), (1, 2), (4, 3)])
@pytest.mark.parametrize("nrec", [1, 24])
def test_fips_gcm_kat_device_batch(plan, nrec):
    aead.force_plan(*plan)
    ctx = aead.AeadCtx(KAT_KEY)
    ct, back, st = _seal_open_batch(ctx, nrec)
    for r in range(nrec):
        assert ct[r].tobytes() == KAT_OUT, (plan, r)
    bad = nrec // 2
    assert st[bad] == 0 and not back[bad].any()  # forged: status 0, zero-filled (aead.h:276-278)
    ok = np.arange(nrec) != bad
    assert (st[ok] == 1).all() and all(back[r].tobytes() == KAT_PT for r in np.nonzero(ok)[0])


@pytest.mark.parametrize("one_wg", [True, False])
def test_fips_gcm_kat_flow_kernel(one_wg):
    """The flow kernel (wide plan forced), with the tag finished in-kernel or by the XOR combine."""
    aead.force_wide(1, 0)
    aead.set_flow_one_wg(one_wg)
    ctx = aead.AeadCtx(KAT_KEY)
    ct, back, st = _seal_open_batch(ctx, 8)
    assert all(ct[r].tobytes() == KAT_OUT for r in range(8))
    assert st[4] == 0 and (np.delete(st, 4) == 1).all()


def test_fips_gcm_kat_config2_sized_batch():
    """65 536 copies of the record in one batch (config 2's record count, automatic plan)."""
    ctx = aead.AeadCtx(KAT_KEY)
    ct, back, st = _seal_open_batch(ctx, 65536)
    want = np.frombuffer(KAT_OUT, np.uint8)
    assert (ct == want[None, :]).all()
    assert int((st == 1).sum()) == 65535 and st[32768] == 0


@pytest.mark.parametrize("direct", [True, False])
def test_fips_gcm_kat_host_path(direct):
    """cmpi_gcm_seal_host / _open_host: the kernel on page-locked bounce memory (direct) or the
    chunked H2D / kernel / D2H pipeline."""
    N.lib().cmpi_debug_set_host_direct(DIRECT_DEFAULT if direct else 0)
    ctx = aead.AeadCtx(KAT_KEY)
    assert ctx.seal(KAT_NONCE, KAT_PT) == KAT_OUT
    assert ctx.open(KAT_NONCE, KAT_OUT) == KAT_PT
    assert ctx.open(KAT_NONCE, KAT_OUT[:-1] + bytes([KAT_OUT[-1] ^ 0x80])) is None


def test_fips_gcm_kat_resident_service():
    ctx = aead.AeadCtx(KAT_KEY)
    ctx.service_start(20000)
    try:
        for _ in range(3):
            assert ctx.seal(KAT_NONCE, KAT_PT) == KAT_OUT
            assert ctx.open(KAT_NONCE, KAT_OUT) == KAT_PT
        assert ctx.service_running()
        assert ctx.open(KAT_NONCE, bytes([KAT_OUT[0] ^ 1]) + KAT_OUT[1:]) is None
    finally:
        ctx.service_stop()
        ctx.close()


def test_fips_gcm_kat_602_device_subkey():
    """The 602 sub-key context: K' = AES_K0(V) is derived on the device (send.c:572-600) and never
    reaches the host; with V = AES_K0^-1(kAESKey) the derived key is the KAT key, so the device-keyed
    seal must give BoringSSL's answer."""
    k0 = bytes(range(16))
    v = oracle.aes128_decrypt_block(k0, KAT_KEY)
    assert oracle.aes128_encrypt_block(k0, v) == KAT_KEY
    base = aead.CipherCtx(k0, "aes-128-ecb")
    sub = aead.AeadCtx.derive_subkey(base, v)
    ct, back, st = _seal_open_batch(sub, 8)
    assert all(ct[r].tobytes() == KAT_OUT for r in range(8))
    assert st[4] == 0 and not back[4].any() and (np.delete(st, 4) == 1).all()


_EVP_KAT = r"""
import ctypes, sys
L = ctypes.CDLL(sys.argv[1])
key, nonce, pt, want = (bytes.fromhex(a) for a in sys.argv[2:6])
P, S = ctypes.c_void_p, ctypes.c_size_t
L.EVP_aead_aes_128_gcm.restype = P
L.EVP_AEAD_CTX_new.restype = P
L.EVP_AEAD_CTX_new.argtypes = [P, P, S, S]
L.EVP_AEAD_CTX_free.argtypes = [P]
for f in (L.EVP_AEAD_CTX_seal, L.EVP_AEAD_CTX_open):
    f.argtypes = [P, P, ctypes.POINTER(S), S, P, S, P, S, P, S]
ctx = L.EVP_AEAD_CTX_new(L.EVP_aead_aes_128_gcm(), key, 16, 0)
assert ctx
out = ctypes.create_string_buffer(256)  # uint8_t output[256] (test_fips.c:68)
olen = S(0)
assert L.EVP_AEAD_CTX_seal(ctx, out, ctypes.byref(olen), 256, nonce, 12, pt, 64, None, 0) == 1
assert olen.value == 80 and out.raw[:80] == want, out.raw[:80].hex()
back = ctypes.create_string_buffer(256)
assert L.EVP_AEAD_CTX_open(ctx, back, ctypes.byref(olen), 256, nonce, 12, want, 80, None, 0) == 1
assert olen.value == 64 and back.raw[:64] == pt
bad = want[:79] + bytes([want[79] ^ 1])
assert L.EVP_AEAD_CTX_open(ctx, back, ctypes.byref(olen), 256, nonce, 12, bad, 80, None, 0) == 0
assert olen.value == 0 and back.raw[:64] == bytes(64)
L.EVP_AEAD_CTX_free(ctx)
print("ok")
"""


@pytest.mark.parametrize("service", [False, True])
def test_fips_gcm_kat_evp_dropin(service):
    """The BoringSSL-ABI drop-in called with test_fips.c:101-124's exact arguments, in a fresh
    process (the shim reads CMPI_EVP_SERVICE_US when it loads), with and without the service."""
    import subprocess
    import sys

    env = dict(os.environ)
    env.pop("CMPI_EVP_SERVICE_US", None)
    env["CMPI_EVP_SERVICE_US"] = "2000" if service else "0"  # 0: a kernel launch per call
    r = subprocess.run([sys.executable, "-c", _EVP_KAT, SHIM, KAT["key"], KAT["gcm_nonce"], KAT["plaintext"],
                        KAT["gcm_ct_tag"]], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", (r.returncode, r.stdout, r.stderr)
