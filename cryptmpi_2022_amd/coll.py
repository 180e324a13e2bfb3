"""Naive secure collectives (include/cmpi_coll.h): one batched seal / open per side.
Reference: MPIR_Naive_Sec_Alltoall (MV/src/mpi/coll/alltoall.c:764-836), MPIR_Naive_Sec_Allgather
(allgather.c:839-899), gather 301 (gather.c:1508-1606), MPIR_Naive_Sec_Scatter (scatter.c:659-730),
MPI_Naive_Sec_Bcast (bcast.c:1510-1580).  Wire block = nonce(12) || ct(n) || tag(16); every block
is sealed under a fresh nonce (the reference's RAND_bytes; here made by the seal kernel itself:
cmpi_coll.h, a random 4-byte field and a 64-bit counter with a random start per context).

The stock collective in between runs on the ciphertext through torch.distributed: RCCL over
xGMI for device buffers (backend "nccl"), or the host transport (backend "gloo": wire blocks are
staged through host memory, as a host MPI would carry them).  A block that fails to open is
zero-filled and raises CmpiError(CMPI_EAUTH, "Decryption error: <collective>") — the
reference prints that message and continues (alltoall.c:831)."""
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


def _host_transport(group) -> bool:
    import torch.distributed as dist

    return dist.get_backend(group) == "gloo"


def _wire(p: int, n: int, device):
    import torch

    return torch.empty(max(p * (n + BLOCK_OVERHEAD), 1), dtype=torch.uint8, device=device)


def _open_checked(ctx, out, wire, n: int, p: int, what: str) -> None:
    import torch

    status = torch.zeros(p, dtype=torch.int32, device=wire.device)
    open_blocks(ctx, out, wire, n, p, status=status)
    if not bool((status == 1).all()):
        raise N.CmpiError(N.CMPI_EAUTH, f"Decryption error: {what}")


def _on_stream(stream):
    """Run a whole collective on `stream` (None: the current stream): seal, transport and open
    then share one stream, so the collective reads the wire only after the seal wrote it."""
    import contextlib

    import torch

    return contextlib.nullcontext() if stream is None else torch.cuda.stream(stream)


def _root_global(root: int, group) -> int:
    """torch.distributed's src=/dst= take a GLOBAL rank; `root` is the rank within `group`
    (the communicator's rank, as MPI's root argument)."""
    import torch.distributed as dist

    return root if group is None else dist.get_global_rank(group, root)


def alltoall(ctx, sendbuf, recvbuf, n: int, group=None, stream=None) -> None:
    """MPIR_Naive_Sec_Alltoall: seal p blocks, all_to_all the ciphertext, open p blocks.
    sendbuf/recvbuf: p*n bytes (device).  Everything runs on `stream` (default: current)."""
    import torch.distributed as dist

    p = dist.get_world_size(group)
    with _on_stream(stream):
        wire, wire_in = _wire(p, n, sendbuf.device), _wire(p, n, sendbuf.device)
        seal_blocks(ctx, wire, sendbuf, n, p)
        if _host_transport(group):
            h_in = wire_in.cpu()
            dist.all_to_all_single(h_in, wire.cpu(), group=group)
            wire_in.copy_(h_in)
        else:
            dist.all_to_all_single(wire_in, wire, group=group)
        _open_checked(ctx, recvbuf, wire_in, n, p, "alltoall")


def allgather(ctx, sendbuf, recvbuf, n: int, group=None) -> None:
    """MPIR_Naive_Sec_Allgather (allgather.c:839-899): seal the rank's block, allgather the wire
    blocks, open all p.  sendbuf n bytes, recvbuf p*n bytes (device)."""
    import torch.distributed as dist

    p = dist.get_world_size(group)
    wire, wire_in = _wire(1, n, sendbuf.device), _wire(p, n, sendbuf.device)
    seal_blocks(ctx, wire, sendbuf, n, 1)
    if _host_transport(group):
        parts = [wire.new_empty(n + BLOCK_OVERHEAD, device="cpu") for _ in range(p)]
        dist.all_gather(parts, wire.cpu(), group=group)
        for i, t in enumerate(parts):
            wire_in[i * (n + BLOCK_OVERHEAD):(i + 1) * (n + BLOCK_OVERHEAD)].copy_(t)
    else:
        dist.all_gather_into_tensor(wire_in, wire, group=group)
    _open_checked(ctx, recvbuf, wire_in, n, p, "allgather")


def gather(ctx, sendbuf, recvbuf, n: int, root: int = 0, group=None) -> None:
    """Gather approach 301 (gather.c:1508-1606): every rank seals its block; the root gathers the
    wire blocks and opens all p into recvbuf (p*n bytes, root only)."""
    import torch.distributed as dist

    p, rank = dist.get_world_size(group), dist.get_rank(group)
    wire = _wire(1, n, sendbuf.device)
    seal_blocks(ctx, wire, sendbuf, n, 1)
    host = _host_transport(group)
    src = wire.cpu() if host else wire
    if rank == root:
        parts = [src.new_empty(n + BLOCK_OVERHEAD) for _ in range(p)]
        dist.gather(src, parts, dst=_root_global(root, group), group=group)
        wire_in = _wire(p, n, sendbuf.device)
        for i, t in enumerate(parts):
            wire_in[i * (n + BLOCK_OVERHEAD):(i + 1) * (n + BLOCK_OVERHEAD)].copy_(t)
        _open_checked(ctx, recvbuf, wire_in, n, p, "gather")
    else:
        dist.gather(src, None, dst=_root_global(root, group), group=group)


def scatter(ctx, sendbuf, recvbuf, n: int, root: int = 0, group=None) -> None:
    """MPIR_Naive_Sec_Scatter (scatter.c:659-730): the root seals its p blocks (one batch), the
    wire blocks are scattered, every rank opens its one block into recvbuf (n bytes)."""
    import torch.distributed as dist

    p, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = recvbuf.device
    host = _host_transport(group)
    mine = _wire(1, n, dev)
    dst = mine.cpu() if host else mine
    if rank == root:
        wire = _wire(p, n, dev)
        seal_blocks(ctx, wire, sendbuf, n, p)
        src = wire.cpu() if host else wire
        parts = list(src.split(n + BLOCK_OVERHEAD))
        dist.scatter(dst, parts, src=_root_global(root, group), group=group)
    else:
        dist.scatter(dst, None, src=_root_global(root, group), group=group)
    if host:
        mine.copy_(dst)
    _open_checked(ctx, recvbuf, mine, n, 1, "scatter")


def bcast(ctx, buf, n: int, root: int = 0, group=None) -> None:
    """MPI_Naive_Sec_Bcast (bcast.c:1510-1580): the root seals buf, the wire block is broadcast,
    every other rank opens it into buf (n bytes, device)."""
    import torch.distributed as dist

    rank = dist.get_rank(group)
    wire = _wire(1, n, buf.device)
    if rank == root:
        seal_blocks(ctx, wire, buf, n, 1)
    host = _host_transport(group)
    t = wire.cpu() if host else wire
    dist.broadcast(t, src=_root_global(root, group), group=group)
    if rank != root:
        if host:
            wire.copy_(t)
        _open_checked(ctx, buf, wire, n, 1, "bcast")
