"""AES-128-CTR, AES-128-ECB and AES-128-OCB on the MI355X vs oracle / golden vectors."""
import hashlib

import numpy as np
import pytest

import oracle
from cryptmpi_2022_amd import aead
from cryptmpi_2022_amd.synth import random_nonces, records, splitmix64_bytes
from tests.gpu_util import dev, empty, host, status_buf

pytestmark = pytest.mark.gpu

KEY = bytes.fromhex("2b7e151628aed2a6abf7158809cf4f3c")


def _check(e, out: bytes):
    if "out" in e:
        assert out.hex() == e["out"]
    else:
        assert hashlib.sha256(out).hexdigest() == e["out_sha256"]


# ------------------------------------------------------------------------- CTR
def test_ctr_kat(golden):
    kat, _ = golden
    for v in kat["ctr"]:
        ctx = aead.CipherCtx(bytes.fromhex(v["key"]), "aes-128-ctr")
        pt = np.frombuffer(bytes.fromhex(v["pt"]), np.uint8)
        out = empty(len(pt))
        ctx.ctr_xor(out, dev(pt), len(pt), bytes.fromhex(v["ctr0"]))
        assert host(out)[: len(pt)].tobytes().hex() == v["ct"]


def test_ctr_openssl_vectors(golden):
    _, ossl = golden
    ctx = aead.CipherCtx(bytes.fromhex(ossl["key"]), "aes-128-ctr")
    for e in ossl["ctr"]:
        pt = splitmix64_bytes(e["pt_seed"], e["len"])
        out = empty(len(pt))
        ctx.ctr_xor(out, dev(pt), len(pt), bytes.fromhex(e["ctr0"]))
        _check(e, host(out)[: len(pt)].tobytes())


def test_ctr_iv_count_stream():
    """702-style: base counter = IV_Count(common IV, ctr) (send.c:1789-1808), 8 MiB + tail."""
    iv = splitmix64_bytes(0x1F, 16).tobytes()
    base = aead.iv_count(iv, 0xFFFFFFF0)  # forces the carry path of IV_Count
    assert base == oracle.iv_count(iv, 0xFFFFFFF0)
    n = (8 << 20) + 13
    pt = splitmix64_bytes(0x20, n)
    ctx = aead.CipherCtx(KEY, "aes-128-ctr")
    out = empty(n)
    ctx.ctr_xor(out, dev(pt), n, base)
    assert np.array_equal(host(out)[:n], oracle.ctr_xor_mt(KEY, base, pt))
    # inverse: XOR again restores the plaintext (in place)
    ctx.ctr_xor(out, out, n, base)
    assert np.array_equal(host(out)[:n], pt)


@pytest.mark.parametrize("ctr_lo", [0, 2**32 - 8])
def test_ctr_config4_full_stream(ctr_lo):
    """BASELINE config 4: one 1 GiB stream + XOR, counter low word starting at 0 and at 2^32 - 8
    (the 32-bit carry after 8 blocks), every byte against the oracle."""
    import torch

    n = 1 << 30
    g = torch.Generator(device="cuda").manual_seed(11)
    pt = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    iv = splitmix64_bytes(0x44, 12).tobytes() + ctr_lo.to_bytes(4, "big")
    ctx = aead.CipherCtx(KEY, "aes-128-ctr")
    out = empty(n)
    ctx.ctr_xor(out, pt, n, iv)
    assert np.array_equal(host(out), oracle.ctr_xor_mt(KEY, iv, pt.cpu().numpy()))


@pytest.mark.parametrize("cb_hex", ["fffffffffffffffffffffffffffff000", "000102030405060708090a0bfffff7f0",
                                    "f0f1f2f3f4f5f6f7f8f9fafbfcfdfeff"])
def test_ctr_carry_corners_chunks(cb_hex):
    """Counters carrying across 32 / 64 / 128 bits inside a 2 048-block chunk: every byte vs the
    oracle, XOR, in place and keystream-only (the bitsliced share this test also covered in round 5
    left the product library in round 6)."""
    cb = bytes.fromhex(cb_hex)
    ctx = aead.CipherCtx(KEY, "aes-128-ctr")
    n = 5 * 2048 * 16 + 13  # five whole 2 048-block chunks and a ragged tail
    pt = splitmix64_bytes(0x51, n)
    want = oracle.ctr_xor_mt(KEY, cb, pt)
    out = empty(n)
    ctx.ctr_xor(out, dev(pt), n, cb)
    assert np.array_equal(host(out)[:n], want)
    ctx.ctr_xor(out, out, n, cb)  # in place: back to the plaintext
    assert np.array_equal(host(out)[:n], pt)
    nb = n // 16
    ks = empty(nb * 16)
    ctx.keystream(ks, nb, cb)
    assert host(ks)[: nb * 16].tobytes() == oracle.ctr_xor(KEY, cb, bytes(nb * 16))


def test_ctr_keystream_equals_xor_of_zeros():
    ctx = aead.CipherCtx(KEY, "aes-128-ctr")
    cb = bytes.fromhex("fffffffffffffffffffffffffffffff0")
    nb = 4096
    ks = empty(nb * 16)
    ctx.keystream(ks, nb, cb)
    z = np.zeros(nb * 16, np.uint8)
    assert host(ks)[: nb * 16].tobytes() == oracle.ctr_xor(KEY, cb, z.tobytes())


# ------------------------------------------------------------------------- ECB
def test_ecb_kat(golden):
    kat, ossl = golden
    for v in kat["ecb"]:
        ctx = aead.CipherCtx(bytes.fromhex(v["key"]), "aes-128-ecb")
        pt = np.frombuffer(bytes.fromhex(v["pt"]), np.uint8)
        out = empty(len(pt))
        ctx.ecb_encrypt(out, dev(pt), len(pt) // 16)
        assert host(out)[: len(pt)].tobytes().hex() == v["ct"]
    ctx = aead.CipherCtx(bytes.fromhex(ossl["key"]), "aes-128-ecb")
    for e in ossl["ecb"]:
        out = empty(16)
        ctx.ecb_encrypt(out, dev(np.frombuffer(bytes.fromhex(e["v"]), np.uint8)), 1)
        assert host(out)[:16].tobytes().hex() == e["out"]


def test_ecb_random():
    ctx = aead.CipherCtx(KEY, "aes-128-ecb")
    data = splitmix64_bytes(0xECB, 16 * 10000)
    out = empty(len(data))
    ctx.ecb_encrypt(out, dev(data), 10000)
    assert host(out).tobytes() == oracle.ecb_encrypt(KEY, data.tobytes())


# ------------------------------------------------------------------------- OCB
def gpu_ocb_seal(ctx, nonces, pt):
    nrec, n = pt.shape
    out = empty(nrec * (n + 16), fill=0x55)
    ctx.seal_batch(out, dev(pt), dev(nonces), n, nrec)
    return host(out)[: nrec * (n + 16)].reshape(nrec, n + 16)


def gpu_ocb_open(ctx, nonces, ct):
    nrec, m = ct.shape
    out = empty(nrec * (m - 16), fill=0x55)
    st = status_buf(nrec)
    ctx.open_batch(out, dev(ct), dev(nonces), m - 16, nrec, status=st)
    return host(out)[: nrec * (m - 16)].reshape(nrec, m - 16), host(st)[:nrec]


def test_ocb_rfc7253(golden):
    kat, _ = golden
    for v in kat["ocb"]:
        if v["aad"]:
            continue
        ctx = aead.AeadCtx(bytes.fromhex(v["key"]), "aes-128-ocb")
        pt = np.frombuffer(bytes.fromhex(v["pt"]), np.uint8)[None, :].copy()
        nonce = np.frombuffer(bytes.fromhex(v["nonce"]), np.uint8)[None, :].copy()
        out = gpu_ocb_seal(ctx, nonce, pt)
        assert out[0].tobytes().hex() == v["out"], v["src"]
        back, st = gpu_ocb_open(ctx, nonce, out)
        assert st[0] == 1 and back[0].tobytes() == pt[0].tobytes()


def test_ocb_openssl_vectors(golden):
    _, ossl = golden
    ctx = aead.AeadCtx(bytes.fromhex(ossl["key"]), "aes-128-ocb")
    for e in ossl["ocb"]:
        pt = splitmix64_bytes(e["pt_seed"], e["len"])[None, :]
        nonce = np.frombuffer(bytes.fromhex(e["nonce"]), np.uint8)[None, :].copy()
        out = gpu_ocb_seal(ctx, nonce, pt)
        _check(e, out[0].tobytes())
        back, st = gpu_ocb_open(ctx, nonce, out)
        assert st[0] == 1 and np.array_equal(back[0], pt[0])


@pytest.mark.parametrize("n", [0, 1, 16, 17, 100, 1008, 1024, 1040, 4096 + 5, 65536, 200000])
def test_ocb_batch_parity(n):
    nrec = 16 if n <= 65536 else 3
    pt = records(0x0CB + n, nrec, n)
    nonces = random_nonces(0x0CC + n, nrec)
    ctx = aead.AeadCtx(KEY, "aes-128-ocb")
    want = oracle.ocb_seal_batch(KEY, nonces, pt)
    assert np.array_equal(gpu_ocb_seal(ctx, nonces, pt), want)
    bad = want.copy()
    bad[1, -1] ^= 1
    back, st = gpu_ocb_open(ctx, nonces, bad)
    assert st[1] == 0 and not back[1].any()
    assert (np.delete(st, 1) == 1).all() and np.array_equal(np.delete(back, 1, axis=0), np.delete(pt, 1, axis=0))


def test_ocb_config3_sample():
    """BASELINE config 3 (4 096 records of 1 MiB): the whole batch round trip on the GPU, and 256
    seeded records (256 MiB) bit-exact against the oracle."""
    import torch

    n, nrec = 1 << 20, 4096
    g = torch.Generator(device="cuda").manual_seed(7)
    pt = torch.randint(0, 256, (nrec * n,), dtype=torch.uint8, device="cuda", generator=g)
    nonces = torch.randint(0, 256, (nrec * 12,), dtype=torch.uint8, device="cuda", generator=g)
    ctx = aead.AeadCtx(KEY, "aes-128-ocb")
    ct = empty(nrec * (n + 16))
    ctx.seal_batch(ct, pt, nonces, n, nrec)
    back = empty(nrec * n)
    st = status_buf(nrec)
    ctx.open_batch(back, ct, nonces, n, nrec, status=st)
    torch.cuda.synchronize()
    assert bool((st == 1).all()) and torch.equal(back, pt)
    idx = torch.from_numpy(np.random.default_rng(3).choice(nrec, 256, replace=False)).cuda()
    want = oracle.ocb_seal_batch(KEY, nonces.view(nrec, 12)[idx].cpu().numpy(), pt.view(nrec, n)[idx].cpu().numpy())
    assert np.array_equal(ct.view(nrec, n + 16)[idx].cpu().numpy(), want)


# ------------------------------------------------------------ the bench's copy kernel
@pytest.mark.parametrize("n", [16, 4096, (1 << 20) + 48, 64 << 20])
def test_debug_copy_kernel(n):
    """cmpi_debug_copy (bench.py's measured HBM peak) copies every byte, grid-stride tail included."""
    import torch

    from cryptmpi_2022_amd import _native as N

    src = dev(splitmix64_bytes(n, n))
    dst = empty(n, fill=0)
    N.check(N.lib().cmpi_debug_copy(dst.data_ptr(), src.data_ptr(), n, torch.cuda.current_stream().cuda_stream))
    assert np.array_equal(host(dst)[:n], host(src)[:n])
    assert N.lib().cmpi_debug_copy(dst.data_ptr(), src.data_ptr(), 8, None) != 0  # n % 16 refused
