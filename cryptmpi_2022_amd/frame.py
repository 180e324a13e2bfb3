"""CryptMPI 600/602 framings on the device (include/cmpi_frame.h) — Python mirror used by the
tests and the bench.  The reference senders/receivers are MV/src/mpi/pt2pt/send.c:221-884 and
recv.c:219-809; see include/cmpi_frame.h for the byte layouts."""
from __future__ import annotations

import ctypes

from . import _native as N
from .aead import _dptr, _stream_ptr


class Plan602(ctypes.Structure):
    _fields_ = [("total", ctypes.c_uint32), ("chop", ctypes.c_uint32), ("outer", ctypes.c_uint32),
                ("nseg", ctypes.c_uint32), ("mode", ctypes.c_uint8), ("subkey", ctypes.c_uint8),
                ("pad_", ctypes.c_uint8 * 2), ("wire_bytes", ctypes.c_uint64)]

    def as_dict(self) -> dict:
        return {"total": self.total, "chop": self.chop, "outer": self.outer, "nseg": self.nseg,
                "mode": chr(self.mode), "subkey": bool(self.subkey), "wire_bytes": self.wire_bytes}


def plan602(n: int, series_threads: int = 8, pending: int = 0) -> Plan602:
    p = Plan602()
    N.check(N.lib().cmpi_602_plan_make(n, series_threads, pending, ctypes.byref(p)))
    return p


def plan602_from_header(header: bytes) -> Plan602:
    p = Plan602()
    N.check(N.lib().cmpi_602_plan_from_header(_hdr(header), ctypes.byref(p)))
    return p


def header602(plan: Plan602, rand16: bytes) -> bytes:
    h = (ctypes.c_uint8 * 25)()
    N.check(N.lib().cmpi_602_header(ctypes.byref(plan), (ctypes.c_uint8 * 16).from_buffer_copy(rand16), h))
    return bytes(h)


def outer_span(plan: Plan602, o: int):
    v = [ctypes.c_uint64() for _ in range(4)]
    N.check(N.lib().cmpi_602_outer_span(ctypes.byref(plan), o, *[ctypes.byref(x) for x in v]))
    return tuple(x.value for x in v)  # wire_off, wire_len, pt_off, pt_len


def _hdr(header: bytes):
    if len(header) != 25:
        raise ValueError("602/600 header is 25 bytes")
    return (ctypes.c_uint8 * 25).from_buffer_copy(header)


def seal602(ctx, plan: Plan602, header: bytes, wire, inp, stream=None, first: int = 0, count: int | None = None):
    """Seal outer messages [first, first+count) of a 602 message into `wire` (device)."""
    count = plan.outer - first if count is None else count
    N.check(N.lib().cmpi_602_seal_outer(ctx.handle, ctypes.byref(plan), _hdr(header), _dptr(wire), _dptr(inp),
                                        first, count, _stream_ptr(stream)))


def open602(ctx, header: bytes, out, wire, status=None, stream=None):
    N.check(N.lib().cmpi_602_open(ctx.handle, _hdr(header), _dptr(out), _dptr(wire), _dptr(status),
                                  _stream_ptr(stream)))


def header600(n: int, kind: bytes = b"1") -> bytes:
    h = (ctypes.c_uint8 * 25)()
    N.check(N.lib().cmpi_600_header(n, kind[0], h))
    return bytes(h)


def seal600(ctx, nonce: bytes, payload, inp, n: int, stream=None):
    N.check(N.lib().cmpi_600_seal(ctx.handle, (ctypes.c_uint8 * 12).from_buffer_copy(nonce), _dptr(payload),
                                  _dptr(inp), n, _stream_ptr(stream)))


def open600(ctx, out, payload, n: int, status=None, stream=None):
    N.check(N.lib().cmpi_600_open(ctx.handle, _dptr(out), _dptr(payload), n, _dptr(status), _stream_ptr(stream)))


# ---- host-memory forms (numpy buffers; include/cmpi_frame.h *_host*): the 602 pipelined sender is
# one seal602_host_begin per outer message, waited in order (send.c:729-850)
def _np(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def seal602_host_begin(ctx, plan: Plan602, header: bytes, wire, inp, first: int, count: int = 1):
    from .aead import Request

    r = ctypes.c_void_p()
    N.check(N.lib().cmpi_602_seal_host_begin(ctx.handle, ctypes.byref(plan), _hdr(header), _np(wire), _np(inp),
                                             first, count, ctypes.byref(r)))
    return Request(r, keep=(wire, inp))


def seal602_host(ctx, plan: Plan602, header: bytes, wire, inp) -> None:
    N.check(N.lib().cmpi_602_seal_host(ctx.handle, ctypes.byref(plan), _hdr(header), _np(wire), _np(inp)))


def open602_host_begin(ctx, header: bytes, out, wire, first: int, count: int = 1, status=None):
    from .aead import Request

    r = ctypes.c_void_p()
    N.check(N.lib().cmpi_602_open_host_begin(ctx.handle, _hdr(header), _np(out), _np(wire), first, count, _np(status),
                                             ctypes.byref(r)))
    return Request(r, keep=(out, wire, status))


def open602_host(ctx, header: bytes, out, wire, status=None) -> int:
    """-> CMPI_OK, or CMPI_EAUTH when a segment failed (status says which; zero-filled)."""
    rc = N.lib().cmpi_602_open_host(ctx.handle, _hdr(header), _np(out), _np(wire), _np(status))
    if rc not in (N.CMPI_OK, N.CMPI_EAUTH):
        N.check(rc)
    return rc
