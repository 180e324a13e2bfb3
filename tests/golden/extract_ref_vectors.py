#!/usr/bin/env python3
"""Extract the reference's own AES / AES-GCM known answers into tests/golden/ref_bssl_vectors.json.

Run where /root/reference exists (this container); the GPU box only reads the committed JSON.
Nothing from the reference is executed, linked or loaded: the tarball is opened with `tarfile`,
the test source is read as text and the object file is read as bytes by the small ELF64 reader
below (section headers + symbol table), exactly like a hex dump.

Vectors, all shipped inside MVAPICH/cryptMPI-mvapich2-2.3.3/boringssl-master.tar.xz (the
BoringSSL snapshot CryptMPI links):

1. `decrepit/cfb/cfb_test.cc:30-46` `kCFBTestCases` — SP 800-38A F.3.13, CFB128-AES128.
   C_i = P_i ^ E_K(C_{i-1}), C_0 = IV, so the vector pins the AES-128 forward cipher on four
   blocks: E_K(IV), E_K(C_1), E_K(C_2), E_K(C_3).
2. The FIPS power-on self-test known answers of that BoringSSL build, as compiled into
   `build/crypto/fipsmodule/CMakeFiles/fipsmodule.dir/bcm.c.o` (the self-test source,
   crypto/fipsmodule/self_check/self_check.c, is not in the tarball; its constant tables are in the
   object's read-only data under their own symbol names): `kAESKey`, `kAESIV`, `kPlaintext`,
   `kAESCBCCiphertext` and `kAESGCMCiphertext` (64 ciphertext bytes then the 16-byte tag).
   `fipstools/test_fips.c:48-50, :97-117` gives the call they answer, in the reference's own
   text: `EVP_AEAD_CTX_init(EVP_aead_aes_128_gcm(), kAESKey)` then
   `EVP_AEAD_CTX_seal(..., nonce = 12 zero bytes, kPlaintext (64 B), ad = NULL, 0)` — the same
   EVP call CryptMPI makes (send.c:311) — and AES-CBC with a zero IV (test_fips.c:70-82).
   The script checks the object's key and plaintext bytes against test_fips.c's literals.
   So this pins GHASH and the GCM composition (J0, inc32, the length block, the tag) as well.
"""
from __future__ import annotations

import json
import os
import re
import struct
import sys
import tarfile

TARBALL = "/root/reference/MVAPICH/cryptMPI-mvapich2-2.3.3/boringssl-master.tar.xz"
CFB_TEST = "boringssl-master/decrepit/cfb/cfb_test.cc"
TEST_FIPS = "boringssl-master/fipstools/test_fips.c"
BCM_OBJ = "boringssl-master/build/crypto/fipsmodule/CMakeFiles/fipsmodule.dir/bcm.c.o"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_bssl_vectors.json")


def parse_cfb(text: str) -> dict:
    """kCFBTestCases[0]: four brace groups of 0x.. bytes (key, iv, plaintext, ciphertext)."""
    body = text[text.index("kCFBTestCases[]"):]
    body = body[: body.index("};")]
    groups = re.findall(r"\{([^{}]*)\}", body)
    vals = [bytes(int(h, 16) for h in re.findall(r"0x([0-9a-fA-F]{2})", g)) for g in groups]
    vals = [v for v in vals if v]
    key, iv, pt, ct = vals[:4]
    assert (len(key), len(iv), len(pt), len(ct)) == (16, 16, 64, 64), [len(v) for v in vals]
    start = text[: text.index("kCFBTestCases[]")].count("\n") + 1
    return {"key": key.hex(), "iv": iv.hex(), "plaintext": pt.hex(), "ciphertext": ct.hex(),
            "source": f"{CFB_TEST}:{start}-{start + 16} (kCFBTestCases, SP 800-38A F.3.13)"}


def elf_symbols(obj: bytes) -> dict[str, bytes]:
    """Bytes of every sized data symbol of an ELF64 little-endian relocatable object."""
    assert obj[:4] == b"\x7fELF" and obj[4] == 2 and obj[5] == 1, "not ELF64 LE"
    e_shoff, = struct.unpack_from("<Q", obj, 0x28)
    e_shentsize, e_shnum, e_shstrndx = struct.unpack_from("<HHH", obj, 0x3A)
    secs = []
    for i in range(e_shnum):
        sh = struct.unpack_from("<IIQQQQIIQQ", obj, e_shoff + i * e_shentsize)
        secs.append(dict(name=sh[0], type=sh[1], offset=sh[4], size=sh[5], link=sh[6], entsize=sh[9]))
    out = {}
    for s in secs:
        if s["type"] != 2:  # SHT_SYMTAB
            continue
        strtab = secs[s["link"]]
        for j in range(s["size"] // s["entsize"]):
            st_name, st_info, _o, st_shndx, st_value, st_size = struct.unpack_from(
                "<IBBHQQ", obj, s["offset"] + j * s["entsize"])
            if (st_info & 0xF) != 1 or st_size == 0 or st_shndx == 0 or st_shndx >= 0xFF00:  # STT_OBJECT
                continue
            nm = obj[strtab["offset"] + st_name: obj.index(b"\0", strtab["offset"] + st_name)].decode()
            sec = secs[st_shndx]
            if sec["type"] == 8:  # SHT_NOBITS (.bss): no stored bytes
                continue
            nm = nm.split(".")[0]  # function-scope statics carry a ".<id>" suffix
            out.setdefault(nm, obj[sec["offset"] + st_value: sec["offset"] + st_value + st_size])
    return out


def main() -> None:
    if not os.path.exists(TARBALL):
        sys.exit(f"{TARBALL} not found: run in the container that holds the reference")
    t = tarfile.open(TARBALL)
    cfb_text = t.extractfile(CFB_TEST).read().decode()
    fips_text = t.extractfile(TEST_FIPS).read().decode()
    syms = elf_symbols(t.extractfile(BCM_OBJ).read())
    want = ["kAESKey", "kAESIV", "kPlaintext", "kAESCBCCiphertext", "kAESGCMCiphertext"]
    missing = [k for k in want if k not in syms]
    assert not missing, f"symbols not found in {BCM_OBJ}: {missing}"
    key, iv, pt = syms["kAESKey"], syms["kAESIV"], syms["kPlaintext"]
    cbc, gcm = syms["kAESCBCCiphertext"], syms["kAESGCMCiphertext"]
    assert (len(key), len(iv), len(pt), len(cbc), len(gcm)) == (16, 16, 64, 64, 80)
    # the object's inputs are the literals of the reference's own driver of the same calls
    lit_key = re.search(r'kAESKey\[16\] = "([^"]*)"', fips_text).group(1).encode()
    lit_pt = re.search(r'kPlaintext\[64\] =\s*"([^"]*)"', fips_text).group(1).encode()
    assert key == lit_key and pt == lit_pt, "bcm.c.o inputs differ from test_fips.c literals"
    seal_line = fips_text[: fips_text.index("EVP_AEAD_CTX_seal(")].count("\n") + 1
    doc = {
        "provenance": (f"{TARBALL} read with tarfile by tests/golden/extract_ref_vectors.py; "
                       "text parsed from the test source, constants read as bytes from the object's "
                       "ELF symbol table (nothing executed, linked or loaded)"),
        "cfb128_f3_13": parse_cfb(cfb_text),
        "fips_kat": {
            "key": key.hex(), "iv": iv.hex(), "plaintext": pt.hex(),
            "gcm_nonce": bytes(12).hex(), "gcm_ad": "",
            "gcm_ct_tag": gcm.hex(), "cbc_ciphertext": cbc.hex(),
            "source": (f"{BCM_OBJ} symbols kAESKey/kAESIV/kPlaintext/kAESCBCCiphertext/kAESGCMCiphertext "
                       f"(BoringSSL FIPS self-test KATs); call shape {TEST_FIPS}:48-50, :{seal_line} "
                       "(EVP_AEAD_CTX_seal, 12 zero nonce bytes, no AD) and :70-82 (AES-CBC, zero IV)"),
        },
    }
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
