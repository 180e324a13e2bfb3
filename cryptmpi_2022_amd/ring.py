"""CTR precompute mask ring (include/cmpi_ring.h) — the enc_common_buffer path of CryptMPI
(MV/src/mpi/pt2pt/send.c:1162-1465, recv.c:954-1023) with the ring in HBM."""
from __future__ import annotations

import ctypes

from . import _native as N
from .aead import _dptr, _stream_ptr


class CtrRing:
    def __init__(self, ctx, iv: bytes, ring_bytes: int = 8 << 20):
        self._ctx = ctx  # keep the key context alive
        h = N.lib().cmpi_ctr_ring_new(ctx.handle, (ctypes.c_uint8 * 16).from_buffer_copy(iv), ring_bytes)
        if not h:
            raise N.CmpiError(N.CMPI_EINVAL, N.last_error())
        self._h = h

    def close(self):
        if getattr(self, "_h", None) and N is not None and N.lib is not None:
            N.lib().cmpi_ctr_ring_free(self._h)
        self._h = None

    __del__ = close

    def generate(self, nbytes: int, stream=None) -> int:
        rc = N.lib().cmpi_ctr_ring_generate(self._h, nbytes, _stream_ptr(stream))
        if rc < 0:
            N.check(rc)
        return rc

    def encrypt(self, out, inp, n: int, stream=None) -> None:
        N.check(N.lib().cmpi_ctr_ring_encrypt(self._h, _dptr(out), _dptr(inp), n, _stream_ptr(stream)))

    def state(self) -> dict:
        st = (ctypes.c_uint64 * 5)()
        N.check(N.lib().cmpi_ctr_ring_state(self._h, st))
        return dict(zip(("start", "end", "compute_size", "counter", "counter_needto_send"), list(st)))


def mask_decrypt(ctx, out, inp, n: int, mask, mask_len: int, iv: bytes, counter: int, stream=None) -> None:
    N.check(N.lib().cmpi_ctr_mask_decrypt(ctx.handle, _dptr(out), _dptr(inp), n, _dptr(mask), mask_len,
                                          (ctypes.c_uint8 * 16).from_buffer_copy(iv), counter, _stream_ptr(stream)))


def xor_bytes(out, a, b, n: int, stream=None) -> None:
    N.check(N.lib().cmpi_xor_bytes(_dptr(out), _dptr(a), _dptr(b), n, _stream_ptr(stream)))
