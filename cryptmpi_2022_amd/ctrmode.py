"""CryptMPI's counter-mode messages on the engine (include/cmpi_ctrmode.h): 700 base counter
(MV/src/mpi/pt2pt/send.c:886-1017, recv.c:812-940) and 702 pre-computed counter
(send.c:1502-1987, recv.c:1025-1403).  Device tensors in and out; 26-byte headers and the
per-rank IVs (Send_common_IV / Recv_common_IV, init.c:766-792) are host bytes."""
from __future__ import annotations

import ctypes

from . import _native as N
from .aead import _dptr, _stream_ptr

HEADER = 26


def _b(data: bytes, n: int):
    return (ctypes.c_uint8 * n).from_buffer_copy(bytes(data))


def send700(ctx, send_iv: bytes, counter: int, out, inp, n: int, stream=None):
    """-> (header bytes, next counter); out = ct (device, n bytes)."""
    c = ctypes.c_uint64(counter)
    hdr = (ctypes.c_uint8 * HEADER)()
    N.check(N.lib().cmpi_700_send(ctx.handle, _b(send_iv, 16), ctypes.byref(c), _dptr(inp), n, hdr, _dptr(out),
                                  _stream_ptr(stream)))
    return bytes(hdr), c.value


def recv700(ctx, recv_iv: bytes, header: bytes, out, inp, stream=None) -> None:
    N.check(N.lib().cmpi_700_recv(ctx.handle, _b(recv_iv, 16), _b(header, HEADER), _dptr(out),
                                  out.numel() if out is not None else 0, _dptr(inp), _stream_ptr(stream)))


class Sender702:
    """One rank's 702 sender: mask ring of stream A in HBM + stream-B long-message counter."""

    def __init__(self, ctx, send_iv: bytes, ring_bytes: int = 8 << 20, series_threads: int = 16, stream=None):
        self.ctx = ctx
        self._h = N.lib().cmpi_702_sender_new(ctx.handle, _b(send_iv, 32), ring_bytes, series_threads,
                                              _stream_ptr(stream))
        if not self._h:
            raise N.CmpiError(N.CMPI_EINVAL, N.last_error())

    def close(self):
        if getattr(self, "_h", None) and N is not None and N.lib is not None:
            N.lib().cmpi_702_sender_free(self._h)
        self._h = None

    __del__ = close

    def send(self, out, inp, n: int, pending_isends: int = 0, stream=None) -> tuple[bytes, int]:
        """-> (header, number of MPI_Isend segments)"""
        hdr = (ctypes.c_uint8 * HEADER)()
        rc = N.lib().cmpi_702_send(self._h, pending_isends, _dptr(inp), n, hdr, _dptr(out), _stream_ptr(stream))
        if rc < 0:
            N.check(rc)
        return bytes(hdr), rc

    def precompute(self, n: int, rounds: int, stream=None) -> int:
        rc = N.lib().cmpi_702_precompute(self._h, n, rounds, _stream_ptr(stream))
        if rc < 0:
            N.check(rc)
        return rc

    def state(self) -> dict:
        st = (ctypes.c_uint64 * 7)()
        N.check(N.lib().cmpi_702_sender_state(self._h, st))
        keys = ("start", "end", "compute_size", "counter", "counter_needto_send", "enc_common_counter_long_msg",
                "counter_needto_send_large_msg")
        return dict(zip(keys, (int(x) for x in st)))


def recv702_premask(ctx, recv_iv: bytes, header: bytes, mask, stream=None) -> int:
    """Decryption mask while the payload is in flight (n < 64 KiB); returns the mask bytes made."""
    ml = ctypes.c_size_t(0)
    N.check(N.lib().cmpi_702_recv_premask(ctx.handle, _b(recv_iv, 32), _b(header, HEADER), _dptr(mask),
                                          mask.numel() if mask is not None else 0, ctypes.byref(ml),
                                          _stream_ptr(stream)))
    return ml.value


def recv702(ctx, recv_iv: bytes, header: bytes, out, inp, mask=None, mask_len: int = 0, stream=None) -> None:
    N.check(N.lib().cmpi_702_recv(ctx.handle, _b(recv_iv, 32), _b(header, HEADER), _dptr(out),
                                  out.numel() if out is not None else 0, _dptr(inp), _dptr(mask), mask_len,
                                  _stream_ptr(stream)))


# ---- host-memory forms (numpy buffers; include/cmpi_ctrmode.h *_host)
def _np(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def send700_host(ctx, send_iv: bytes, counter: int, out, inp, n: int):
    """-> (header, next counter); out = ct (host, n bytes)."""
    c = ctypes.c_uint64(counter)
    hdr = (ctypes.c_uint8 * HEADER)()
    N.check(N.lib().cmpi_700_send_host(ctx.handle, _b(send_iv, 16), ctypes.byref(c), _np(inp), n, hdr, _np(out)))
    return bytes(hdr), c.value


def recv700_host(ctx, recv_iv: bytes, header: bytes, out, inp) -> None:
    N.check(N.lib().cmpi_700_recv_host(ctx.handle, _b(recv_iv, 16), _b(header, HEADER), _np(out), out.size, _np(inp)))


def send702_host(sender: "Sender702", out, inp, n: int, pending_isends: int = 0) -> tuple[bytes, int]:
    hdr = (ctypes.c_uint8 * HEADER)()
    rc = N.lib().cmpi_702_send_host(sender._h, pending_isends, _np(inp), n, hdr, _np(out))
    if rc < 0:
        N.check(rc)
    return bytes(hdr), rc


def recv702_host(ctx, recv_iv: bytes, header: bytes, out, inp, mask=None, mask_len: int = 0, mask_stream=None) -> None:
    """mask: device tensor from recv702_premask (made on mask_stream, default the current stream)."""
    N.check(N.lib().cmpi_702_recv_host(ctx.handle, _b(recv_iv, 32), _b(header, HEADER), _np(out), out.size, _np(inp),
                                       _dptr(mask), mask_len, _stream_ptr(mask_stream)))
