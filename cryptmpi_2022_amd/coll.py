"""Naive secure collectives (include/cmpi_coll.h): one batched seal / open per side.
Reference: MPIR_Naive_Sec_Alltoall (MV/src/mpi/coll/alltoall.c:764-836), MPIR_Naive_Sec_Allgather
(allgather.c:839-899), gather 301 (gather.c:1508-1606), MPIR_Naive_Sec_Scatter (scatter.c:659-730),
MPI_Naive_Sec_Bcast (bcast.c:1510-1580).  Wire block = nonce(12) || ct(n) || tag(16)."""
from __future__ import annotations

from . import _native as N
from .aead import _dptr, _stream_ptr

BLOCK_OVERHEAD = 28


def seal_blocks(ctx, wire, inp, n: int, nblk: int, workspace=None, stream=None) -> None:
    """inp[i*n : (i+1)*n] -> wire[i*(n+28) ...] with a fresh nonce per block."""
    N.check(N.lib().cmpi_naive_seal_blocks(ctx.handle, _dptr(wire), _dptr(inp), n, nblk, _dptr(workspace),
                                           _stream_ptr(stream)))


def open_blocks(ctx, out, wire, n: int, nblk: int, status=None, workspace=None, stream=None) -> None:
    N.check(N.lib().cmpi_naive_open_blocks(ctx.handle, _dptr(out), _dptr(wire), n, nblk, _dptr(status),
                                           _dptr(workspace), _stream_ptr(stream)))


def alltoall(ctx, sendbuf, recvbuf, n: int, group=None, stream=None) -> None:
    """MPIR_Naive_Sec_Alltoall on torch.distributed: seal p blocks, all_to_all the ciphertext
    (RCCL over xGMI on ROCm), open p blocks.  sendbuf/recvbuf: p*n bytes (device)."""
    import torch
    import torch.distributed as dist

    p = dist.get_world_size(group)
    wire = torch.empty(p * (n + BLOCK_OVERHEAD), dtype=torch.uint8, device=sendbuf.device)
    wire_in = torch.empty_like(wire)
    seal_blocks(ctx, wire, sendbuf, n, p, stream=stream)
    dist.all_to_all_single(wire_in, wire, group=group)
    status = torch.empty(p, dtype=torch.int32, device=sendbuf.device)
    open_blocks(ctx, recvbuf, wire_in, n, p, status=status, stream=stream)
    if not bool((status == 1).all()):
        raise N.CmpiError(N.CMPI_EAUTH, "Decryption error: alltoall")  # alltoall.c:831 prints
