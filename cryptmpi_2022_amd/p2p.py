"""Secure point-to-point messages over a host transport — the 600 pair of BASELINE config 1:
MPI_SEC_Multi_Thread_Send_OpenMP (MV/src/mpi/pt2pt/send.c:221-337) and
MPI_SEC_Multi_Thread_Recv_OpenMP (recv.c:219-341).  A message of n bytes travels as two MPI
messages: the 25-byte header ([0..3] BE32 n, [20] '1', [21..24] BE32 n) and the payload
nonce(12, RAND_bytes) || ct || tag(16).  The buffers start and end in host memory (MPI user
buffers); the seal/open run on the GPU through the engine's host-memory batch calls, and the
transport is torch.distributed on CPU tensors (gloo: the host path an MPI over TCP/shm takes).
The reference prints "Decryption error" and continues on a bad tag (recv.c:328); here open
raises CmpiError(CMPI_EAUTH)."""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _native as N

HEADER = 25
OVERHEAD = 28


class Endpoint:
    """Pinned staging reused across messages (MPI's static large_send_buffer / large_recv_buffer,
    mpiimpl.h:265) and the context of the rank's key (global_openmp_ctx, init.c:587-612)."""

    def __init__(self, ctx, max_bytes: int = 1 << 20):
        import torch

        self.ctx = ctx
        self.cap = max_bytes
        self.send_buf = torch.empty(max_bytes + OVERHEAD, dtype=torch.uint8).pin_memory()
        self.recv_buf = torch.empty(max_bytes + OVERHEAD, dtype=torch.uint8).pin_memory()
        self.hdr_out = torch.zeros(HEADER, dtype=torch.uint8)
        self.hdr_in = torch.zeros(HEADER, dtype=torch.uint8)

    def send(self, msg: np.ndarray, dst: int, group=None, nonce: bytes | None = None) -> None:
        """send.c:221-337: the header goes out first (MPI_Isend_original, :288) and travels while
        the message is sealed into pinned staging, then nonce || ct || tag (:330), both waited
        (:333-334)."""
        import torch
        import torch.distributed as dist

        n = int(msg.size)
        if n > self.cap:  # an explicit check: a bare assert vanishes under python -O
            raise N.CmpiError(N.CMPI_EINVAL, f"message of {n} B exceeds the endpoint's {self.cap} B staging")
        L = N.lib()
        hb = (ctypes.c_uint8 * HEADER)()
        N.check(L.cmpi_600_header(n, ord("1"), hb))
        self.hdr_out.numpy()[:] = np.frombuffer(bytes(hb), np.uint8)
        w_hdr = dist.isend(self.hdr_out, dst, group=group)
        sb = self.send_buf.numpy()
        sb[:12] = np.frombuffer(nonce if nonce is not None else os.urandom(12), np.uint8)  # RAND_bytes
        src = np.ascontiguousarray(msg).reshape(-1).view(np.uint8)  # sealed where it lies (MPI user buffer)
        base = self.send_buf.data_ptr()
        try:
            N.check(L.cmpi_gcm_seal_host(self.ctx.handle, ctypes.c_void_p(base + 12), n + 16,
                                         ctypes.c_void_p(src.ctypes.data if n else base), max(n, 1),
                                         ctypes.c_void_p(base), 12, n, 1))
        finally:
            w_hdr.wait()  # the header buffer is reused by the next message
        dist.send(self.send_buf[: n + OVERHEAD], dst, group=group)

    def recv(self, src: int, group=None, out: np.ndarray | None = None) -> np.ndarray:
        """recv.c:219-341: header, payload, open; returns the plaintext (host), opened straight
        into `out` (a uint8 array of at least the message's size, the MPI receive buffer) when
        given, else into a new array."""
        import torch.distributed as dist

        dist.recv(self.hdr_in, src, group=group)
        h = bytes(self.hdr_in.numpy())
        n = int.from_bytes(h[0:4], "big")
        if n > self.cap:  # the header is untrusted peer input: never size a copy from it unchecked
            raise N.CmpiError(N.CMPI_EINVAL, f"peer header announces {n} B, endpoint staging holds {self.cap} B")
        dist.recv(self.recv_buf[: n + OVERHEAD], src, group=group)
        if out is None:
            out = np.empty(max(n, 1), np.uint8)
        elif out.dtype != np.uint8 or not out.flags.c_contiguous or out.size < n:
            raise N.CmpiError(N.CMPI_EINVAL, f"receive buffer must be a contiguous uint8 array of >= {n} bytes")
        st = ctypes.c_int32(0)
        base = self.recv_buf.data_ptr()
        rc = N.lib().cmpi_gcm_open_host(self.ctx.handle, ctypes.c_void_p(out.ctypes.data), max(n, 1),
                                        ctypes.c_void_p(base + 12), n + 16, ctypes.c_void_p(base), 12, n, 1,
                                        ctypes.byref(st))
        if rc == N.CMPI_EAUTH or st.value != 1:
            raise N.CmpiError(N.CMPI_EAUTH, "Decryption error")
        N.check(rc)
        return out[:n]

    def last_payload(self, n: int) -> bytes:
        return bytes(self.send_buf.numpy()[: n + OVERHEAD])
