"""ctypes wrapper over oracle/liboracle.so — the CPU restatement used as the parity checker.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package (cryptmpi_2022_amd/).  See oracle/oracle.h for
what each function restates and the reference file:line it follows.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build() -> None:
    import subprocess

    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        sig = {
            "orc_aes128_expand": [P, P],
            "orc_aes128_encrypt": [P, P, P],
            "orc_aes128_decrypt": [P, P, P],
            "orc_aes128_ecb": [P, P, P, S],
            "orc_gf128_mul": [P, P, P],
            "orc_ghash": [P, P, S, P, S, P],
            "orc_gcm_seal": [P, P, S, P, S, P, S, P],
            "orc_gcm_open": [P, P, S, P, S, P, S, P],
            "orc_gcm_seal_batch": [P, P, S, P, S, P, S, S, S, I],
            "orc_gcm_open_batch": [P, P, S, P, S, P, S, S, S, P, I],
            "orc_ctr128_xor": [P, P, P, P, S],
            "orc_ctr128_xor_mt": [P, P, P, P, S, I],
            "orc_iv_count": [P, ctypes.c_ulong],
            "orc_iv_count_out": [P, ctypes.c_ulong, P],
            "orc_ocb_seal": [P, P, S, P, S, P, S, P],
            "orc_ocb_open": [P, P, S, P, S, P, S, P],
            "orc_ocb_seal_batch": [P, P, S, P, S, P, S, S, S, I],
            "orc_nonce602": [P, ctypes.c_uint8, ctypes.c_uint32],
            "orc_header600": [P, ctypes.c_uint32, ctypes.c_uint8, ctypes.c_uint32],
            "orc_700_send": [P, P, P, P, I, P, P],
            "orc_700_recv": [P, P, P, P, P],
            "orc_702_init": [P, P, P, P, I, I],
            "orc_702_send": [P, I, P, I, P, P],
            "orc_702_precompute": [P, I, I],
            "orc_702_recv": [P, P, P, P, P, I],
        }
        for name, args in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int if name in ("orc_gcm_seal", "orc_gcm_open", "orc_ocb_seal", "orc_ocb_open",
                                                  "orc_702_send", "orc_702_precompute", "orc_702_recv") else None
        _lib = L
    return _lib


def _buf(b) -> ctypes.Array:
    return (ctypes.c_uint8 * max(1, len(b))).from_buffer_copy(bytes(b) or b"\0")


def _ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


# ---------------------------------------------------------------- single-message API
def aes128_encrypt_block(key: bytes, block: bytes) -> bytes:
    rk = (ctypes.c_uint8 * 176)()
    out = (ctypes.c_uint8 * 16)()
    lib().orc_aes128_expand(_buf(key), rk)
    lib().orc_aes128_encrypt(rk, _buf(block), out)
    return bytes(out)


def aes128_decrypt_block(key: bytes, block: bytes) -> bytes:
    rk = (ctypes.c_uint8 * 176)()
    out = (ctypes.c_uint8 * 16)()
    lib().orc_aes128_expand(_buf(key), rk)
    lib().orc_aes128_decrypt(rk, _buf(block), out)
    return bytes(out)


def ecb_encrypt(key: bytes, data: bytes) -> bytes:
    assert len(data) % 16 == 0
    out = (ctypes.c_uint8 * max(1, len(data)))()
    lib().orc_aes128_ecb(_buf(key), _buf(data), out, len(data) // 16)
    return bytes(out)[: len(data)]


def gf128_mul(x: bytes, y: bytes) -> bytes:
    out = (ctypes.c_uint8 * 16)()
    lib().orc_gf128_mul(_buf(x), _buf(y), out)
    return bytes(out)


def gcm_seal(key: bytes, nonce: bytes, pt: bytes, aad: bytes = b"") -> bytes:
    out = (ctypes.c_uint8 * (len(pt) + 16))()
    ok = lib().orc_gcm_seal(_buf(key), _buf(nonce), len(nonce), _buf(aad), len(aad), _buf(pt), len(pt), out)
    assert ok == 1
    return bytes(out)


def gcm_open(key: bytes, nonce: bytes, ct_tag: bytes, aad: bytes = b""):
    """Returns plaintext bytes, or None on authentication failure."""
    out = (ctypes.c_uint8 * max(1, len(ct_tag) - 16))()
    ok = lib().orc_gcm_open(_buf(key), _buf(nonce), len(nonce), _buf(aad), len(aad), _buf(ct_tag), len(ct_tag), out)
    return bytes(out)[: len(ct_tag) - 16] if ok else None


def ctr_xor(key: bytes, ctr0: bytes, data: bytes) -> bytes:
    out = (ctypes.c_uint8 * max(1, len(data)))()
    lib().orc_ctr128_xor(_buf(key), _buf(ctr0), _buf(data), out, len(data))
    return bytes(out)[: len(data)]


def iv_count(iv: bytes, cter: int) -> bytes:
    b = _buf(iv)
    lib().orc_iv_count(b, cter & 0xFFFFFFFFFFFFFFFF)
    return bytes(b)


def ocb_seal(key: bytes, nonce: bytes, pt: bytes, aad: bytes = b"") -> bytes:
    out = (ctypes.c_uint8 * (len(pt) + 16))()
    ok = lib().orc_ocb_seal(_buf(key), _buf(nonce), len(nonce), _buf(aad), len(aad), _buf(pt), len(pt), out)
    assert ok == 1
    return bytes(out)


def ocb_open(key: bytes, nonce: bytes, ct_tag: bytes, aad: bytes = b""):
    out = (ctypes.c_uint8 * max(1, len(ct_tag) - 16))()
    ok = lib().orc_ocb_open(_buf(key), _buf(nonce), len(nonce), _buf(aad), len(aad), _buf(ct_tag), len(ct_tag), out)
    return bytes(out)[: len(ct_tag) - 16] if ok else None


def nonce602(flag: bytes, seg: int) -> bytes:
    b = (ctypes.c_uint8 * 12)()
    lib().orc_nonce602(b, flag[0], seg)
    return bytes(b)


# ---------------------------------------------------------------- batch API (numpy, host memory)
def gcm_seal_batch(key: bytes, nonces: np.ndarray, pt: np.ndarray, nthreads: int = 0) -> np.ndarray:
    """nonces: (N,12) u8; pt: (N,n) u8 → (N, n+16) u8 (ct || tag)."""
    N, n = pt.shape
    out = np.empty((N, n + 16), dtype=np.uint8)
    lib().orc_gcm_seal_batch(_buf(key), _ptr(nonces), nonces.strides[0], _ptr(pt), pt.strides[0], _ptr(out), out.strides[0], n, N, nthreads)
    return out


def gcm_open_batch(key: bytes, nonces: np.ndarray, ct_tag: np.ndarray, nthreads: int = 0):
    N, m = ct_tag.shape
    n = m - 16
    out = np.empty((N, n), dtype=np.uint8)
    status = np.empty(N, dtype=np.int32)
    lib().orc_gcm_open_batch(_buf(key), _ptr(nonces), nonces.strides[0], _ptr(ct_tag), ct_tag.strides[0], _ptr(out), max(1, out.strides[0]), n, N, _ptr(status), nthreads)
    return out, status


def ocb_seal_batch(key: bytes, nonces: np.ndarray, pt: np.ndarray, nthreads: int = 0) -> np.ndarray:
    N, n = pt.shape
    out = np.empty((N, n + 16), dtype=np.uint8)
    lib().orc_ocb_seal_batch(_buf(key), _ptr(nonces), nonces.strides[0], _ptr(pt), pt.strides[0], _ptr(out), out.strides[0], n, N, nthreads)
    return out


def ctr_xor_mt(key: bytes, ctr0: bytes, data: np.ndarray, nthreads: int = 0) -> np.ndarray:
    out = np.empty_like(data)
    lib().orc_ctr128_xor_mt(_buf(key), _buf(ctr0), _ptr(data), _ptr(out), data.nbytes, nthreads)
    return out


# ---------------------------------------------------------------- 602 framing (send.c:339-884)
class _Plan602(ctypes.Structure):
    _fields_ = [("total", ctypes.c_uint32), ("chop", ctypes.c_uint32), ("outer", ctypes.c_uint32),
                ("nseg", ctypes.c_uint32), ("mode", ctypes.c_uint8), ("subkey", ctypes.c_uint8),
                ("wire_bytes", ctypes.c_uint64)]


def plan602(n: int, series_threads: int = 8, pending: int = 0) -> dict:
    p = _Plan602()
    lib().orc_602_plan(ctypes.c_uint32(n), series_threads, pending, ctypes.byref(p))
    return {"total": p.total, "chop": p.chop, "outer": p.outer, "nseg": p.nseg, "mode": chr(p.mode),
            "subkey": bool(p.subkey), "wire_bytes": p.wire_bytes}


def seal602(key: bytes, small_key: bytes, pt: bytes, rand16: bytes, series_threads: int = 8, pending: int = 0,
            wire_fill: int = 0):
    """(header[25], wire[wire_bytes]) of one 602 message exactly as send.c builds them."""
    p = _Plan602()
    lib().orc_602_plan(ctypes.c_uint32(len(pt)), series_threads, pending, ctypes.byref(p))
    hdr = (ctypes.c_uint8 * 25)()
    wire = (ctypes.c_uint8 * max(1, p.wire_bytes))(*([wire_fill] * max(1, p.wire_bytes)))
    lib().orc_602_seal(_buf(key), _buf(small_key), ctypes.byref(p), _buf(rand16), _buf(pt) if pt else None, hdr, wire)
    return bytes(hdr), bytes(wire)[: p.wire_bytes]


# ---------------------------------------------------------------- CTR mask ring (send.c:1162-1465)
class _Ring(ctypes.Structure):
    _fields_ = [("key", ctypes.c_uint8 * 16), ("iv", ctypes.c_uint8 * 16), ("buf", ctypes.c_void_p),
                ("max", ctypes.c_int), ("start", ctypes.c_int), ("end", ctypes.c_int), ("compute_size", ctypes.c_int),
                ("counter", ctypes.c_ulong), ("counter_needto_send", ctypes.c_ulong)]


class Ring:
    """The reference's enc_common_buffer state machine (generateCommonEncMask /
    encryption_common_counter) over a ring of `max_bytes`."""

    def __init__(self, key: bytes, iv: bytes, max_bytes: int = 8 << 20):
        self._mem = (ctypes.c_uint8 * max_bytes)()
        self._r = _Ring()
        lib().orc_ring_init(ctypes.byref(self._r), _buf(key), _buf(iv), self._mem, max_bytes)

    def generate(self, nbytes: int) -> int:
        return lib().orc_ring_generate(ctypes.byref(self._r), nbytes)

    def encrypt(self, data: bytes) -> bytes:
        out = (ctypes.c_uint8 * max(1, len(data)))()
        lib().orc_ring_encrypt(ctypes.byref(self._r), _buf(data) if data else None, len(data), out)
        return bytes(out)[: len(data)]

    def state(self) -> dict:
        r = self._r
        return {"start": r.start, "end": r.end, "compute_size": r.compute_size, "counter": r.counter,
                "counter_needto_send": r.counter_needto_send}


def mask_decrypt(key: bytes, iv: bytes, counter: int, mask: bytes, data: bytes) -> bytes:
    """recv.c:954-1023 decryption_common_counter_ivflag."""
    out = (ctypes.c_uint8 * max(1, len(data)))()
    lib().orc_mask_decrypt(_buf(key), _buf(iv), ctypes.c_ulong(counter), _buf(mask) if mask else None, len(mask),
                           _buf(data) if data else None, len(data), out)
    return bytes(out)[: len(data)]


# ---------------------------------------------------------------- counter-mode messages (700 / 702)
def send700(key: bytes, send_iv: bytes, counter: int, pt: bytes):
    """MPI_SEC_BaseCounter_Pipeline_Send (send.c:886-1017): (header[26], ct, next counter)."""
    c = ctypes.c_ulong(counter)
    hdr = (ctypes.c_uint8 * 26)()
    out = (ctypes.c_uint8 * max(1, len(pt)))()
    lib().orc_700_send(_buf(key), _buf(send_iv), ctypes.byref(c), _buf(pt) if pt else None, len(pt), hdr, out)
    return bytes(hdr), bytes(out)[: len(pt)], c.value


def recv700(key: bytes, recv_iv: bytes, hdr: bytes, ct: bytes) -> bytes:
    out = (ctypes.c_uint8 * max(1, len(ct)))()
    lib().orc_700_recv(_buf(key), _buf(recv_iv), _buf(hdr), _buf(ct) if ct else None, out)
    return bytes(out)[: len(ct)]


class _Sender702(ctypes.Structure):
    _fields_ = [("ring", _Ring), ("ivb", ctypes.c_uint8 * 16), ("enc_common_counter_long_msg", ctypes.c_ulong),
                ("counter_needto_send_large_msg", ctypes.c_ulong), ("series", ctypes.c_int)]


class Sender702:
    """One rank's 702 sender state (init.c:766-792 + send.c:1502-1987) over a ring of max_bytes."""

    def __init__(self, key: bytes, send_iv: bytes, max_bytes: int = 8 << 20, series: int = 16):
        self._mem = (ctypes.c_uint8 * max_bytes)()
        self._s = _Sender702()
        lib().orc_702_init(ctypes.byref(self._s), _buf(key), _buf(send_iv), self._mem, max_bytes, series)

    def send(self, pt: bytes, pending: int = 0):
        """-> (header[26], ciphertext)"""
        hdr = (ctypes.c_uint8 * 26)()
        out = (ctypes.c_uint8 * max(1, len(pt)))()
        lib().orc_702_send(ctypes.byref(self._s), pending, _buf(pt) if pt else None, len(pt), hdr, out)
        return bytes(hdr), bytes(out)[: len(pt)]

    def precompute(self, n: int, rounds: int) -> int:
        return lib().orc_702_precompute(ctypes.byref(self._s), n, rounds)

    def state(self) -> dict:
        s = self._s
        r = s.ring
        return {"start": r.start, "end": r.end, "compute_size": r.compute_size, "counter": r.counter,
                "counter_needto_send": r.counter_needto_send,
                "enc_common_counter_long_msg": s.enc_common_counter_long_msg,
                "counter_needto_send_large_msg": s.counter_needto_send_large_msg}


def recv702(key: bytes, recv_iv: bytes, hdr: bytes, ct: bytes, premask: bool = True) -> bytes:
    """MPI_SEC_PreComputeCounter_Recv_v4 (recv.c:1025-1403); premask: mask generated while the
    payload was in flight (recv.c:1107-1196), else the direct path."""
    out = (ctypes.c_uint8 * max(1, len(ct)))()
    lib().orc_702_recv(_buf(key), _buf(recv_iv), _buf(hdr), _buf(ct) if ct else None, out, 1 if premask else 0)
    return bytes(out)[: len(ct)]
