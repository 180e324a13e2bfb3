"""Oracle pin against known answers held by the reference itself: tests/golden/ref_bssl_vectors.json,
extracted from MVAPICH/cryptMPI-mvapich2-2.3.3/boringssl-master.tar.xz (the BoringSSL snapshot
CryptMPI links) by tests/golden/extract_ref_vectors.py.  The JSON is committed, so these run
without /root/reference.  What they pin: the AES-128 forward and inverse cipher (CFB128 F.3.13 of
decrepit/cfb/cfb_test.cc:30-46, the FIPS self-test CBC answer) and the AES-128-GCM seal / open of
EVP_AEAD_CTX_seal (the FIPS self-test GCM answer for test_fips.c:97-117's call), i.e. GHASH and
the GCM composition.  tests/test_gpu_ref_vectors.py runs the same answers through the engine."""
import json
import os

import oracle


def ref_vectors():
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_bssl_vectors.json")
    with open(p) as f:
        return json.load(f)


def _xor(a: bytes, b: bytes) -> bytes:
    return bytes(x ^ y for x, y in zip(a, b))


def test_oracle_aes_vs_reference_cfb128():
    """BoringSSL decrepit/cfb/cfb_test.cc:30-46 (SP 800-38A F.3.13): C_i = P_i ^ AES_K(C_{i-1})."""
    v = ref_vectors()["cfb128_f3_13"]
    key, prev = bytes.fromhex(v["key"]), bytes.fromhex(v["iv"])
    pt, ct = bytes.fromhex(v["plaintext"]), bytes.fromhex(v["ciphertext"])
    out = b""
    for i in range(4):
        blk = _xor(pt[16 * i:16 * i + 16], oracle.aes128_encrypt_block(key, prev))
        out += blk
        prev = blk
    assert out == ct
    # and decryption (CFB decrypt uses the forward cipher too)
    prev, back = bytes.fromhex(v["iv"]), b""
    for i in range(4):
        back += _xor(ct[16 * i:16 * i + 16], oracle.aes128_encrypt_block(key, prev))
        prev = ct[16 * i:16 * i + 16]
    assert back == pt


def test_oracle_gcm_vs_reference_fips_kat():
    """BoringSSL's own AES-128-GCM answer (kAESGCMCiphertext of its FIPS self-test, read from the
    shipped bcm.c.o) for EVP_AEAD_CTX_seal(kAESKey, 12 zero nonce bytes, kPlaintext, no AD) —
    test_fips.c:97-117: pins GHASH, J0 / inc32, the length block and the tag composition."""
    v = ref_vectors()["fips_kat"]
    key, nonce, pt = bytes.fromhex(v["key"]), bytes.fromhex(v["gcm_nonce"]), bytes.fromhex(v["plaintext"])
    want = bytes.fromhex(v["gcm_ct_tag"])
    assert len(want) == len(pt) + 16
    assert oracle.gcm_seal(key, nonce, pt) == want
    assert oracle.gcm_open(key, nonce, want) == pt
    forged = bytearray(want)
    forged[-1] ^= 1
    assert oracle.gcm_open(key, nonce, bytes(forged)) is None


def test_oracle_aes_vs_reference_fips_cbc():
    """kAESCBCCiphertext (AES-CBC, zero IV, test_fips.c:70-82): C_i = AES_K(P_i ^ C_{i-1}), and the
    inverse cipher (OCB open's) gives P_i = AES_K^-1(C_i) ^ C_{i-1}."""
    v = ref_vectors()["fips_kat"]
    key, prev = bytes.fromhex(v["key"]), bytes.fromhex(v["iv"])
    pt, ct = bytes.fromhex(v["plaintext"]), bytes.fromhex(v["cbc_ciphertext"])
    for i in range(4):
        c = oracle.aes128_encrypt_block(key, _xor(pt[16 * i:16 * i + 16], prev))
        assert c == ct[16 * i:16 * i + 16]
        assert _xor(oracle.aes128_decrypt_block(key, c), prev) == pt[16 * i:16 * i + 16]
        prev = c
