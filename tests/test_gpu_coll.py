"""Naive secure collectives as batch calls (alltoall.c:764-836 and siblings): fresh nonces,
wire blocks bit-exact vs the oracle for the nonces they carry, round trip, forgery, and an
in-process two-rank Alltoall exchange."""
import numpy as np
import pytest

import oracle
from cryptmpi_2022_amd import aead, coll
from cryptmpi_2022_amd.synth import records

from tests.gpu_util import dev, empty, host, status_buf

pytestmark = pytest.mark.gpu
KEY = bytes(range(16))


@pytest.mark.parametrize("n,p", [(0, 3), (1, 8), (1000, 8), (4096, 5), (1 << 20, 8)])
def test_seal_blocks_wire_and_round_trip(n, p):
    ctx = aead.AeadCtx(KEY)
    pt = records(0xA2A + n, p, n)
    wire = empty(p * (n + 28), fill=0)
    coll.seal_blocks(ctx, wire, dev(pt) if n else empty(1), n, p)
    w = host(wire)[: p * (n + 28)].reshape(p, n + 28)
    nonces = np.ascontiguousarray(w[:, :12])
    assert len({bytes(x) for x in nonces}) == p  # fresh nonce per block
    assert np.array_equal(w[:, 12:], oracle.gcm_seal_batch(KEY, nonces, pt))
    out, st = empty(max(p * n, 1), fill=0xEE), status_buf(p)
    coll.open_blocks(ctx, out, wire, n, p, status=st)
    assert (host(st)[:p] == 1).all() and host(out)[: p * n].tobytes() == pt.tobytes()
    w2 = w.copy()
    w2[p // 2, -1] ^= 0x80
    out2, st2 = empty(max(p * n, 1), fill=0xEE), status_buf(p)
    coll.open_blocks(ctx, out2, dev(w2), n, p, status=st2)
    s = host(st2)[:p]
    assert s[p // 2] == 0 and s.sum() == p - 1
    assert (host(out2)[(p // 2) * n: (p // 2 + 1) * n] == 0).all()


def test_nonces_never_repeat_across_calls():
    ctx = aead.AeadCtx(KEY)
    seen = set()
    for _ in range(4):
        wire = empty(64 * 28)
        coll.seal_blocks(ctx, wire, empty(1), 0, 64)
        w = host(wire)[: 64 * 28].reshape(64, 28)
        seen |= {bytes(x[:12]) for x in w}
    assert len(seen) == 256


def test_fresh_nonce_construction():
    """cmpi_coll.h: nonce = P || BE64(c + r) — one random field per context, a counter that
    advances by the block count per call (both flow-kernel and lane-kernel seals), and two
    contexts under one key draw different random fields."""
    ctx, other = aead.AeadCtx(KEY), aead.AeadCtx(KEY)
    ctrs = []
    for n, p in [(1 << 20, 8), (1000, 3), (64, 70)]:
        pt = records(0xF0 + n, p, n)
        wire = empty(p * (n + 28), fill=0)
        coll.seal_blocks(ctx, wire, dev(pt), n, p)
        w = host(wire)[: p * (n + 28)].reshape(p, n + 28)
        assert np.array_equal(w[:, 12:], oracle.gcm_seal_batch(KEY, np.ascontiguousarray(w[:, :12]), pt))
        assert len({bytes(x[:4]) for x in w}) == 1
        c = [int.from_bytes(bytes(x[4:12]), "big") for x in w]
        assert c == [(c[0] + i) % (1 << 64) for i in range(p)]
        ctrs.append((bytes(w[0, :4]), c[0], p))
    for (pa, ca, na), (pb, cb, _) in zip(ctrs, ctrs[1:]):
        assert pa == pb and cb == (ca + na) % (1 << 64)
    wire = empty(28, fill=0)
    coll.seal_blocks(other, wire, empty(1), 0, 1)
    assert bytes(host(wire)[:4]) != ctrs[0][0]


def test_fresh_nonces_disjoint_across_contexts():
    """Sixteen contexts under one key (ranks sharing CryptMPI's global key) seal 64 blocks each
    twice: all 2 048 nonces are distinct, each context keeps one random field (the bound
    across contexts is probabilistic, include/cmpi_coll.h)."""
    ctxs = [aead.AeadCtx(KEY) for _ in range(16)]
    seen, fields = set(), set()
    for rnd in range(2):
        for k, c in enumerate(ctxs):
            wire = empty(64 * 28, fill=0)
            coll.seal_blocks(c, wire, empty(1), 0, 64)
            w = host(wire)[: 64 * 28].reshape(64, 28)
            nonces = {bytes(x[:12]) for x in w}
            assert len(nonces) == 64 and not (nonces & seen), (rnd, k)
            seen |= nonces
            fields.add(bytes(w[0, :4]))
    assert len(seen) == 2 * 16 * 64 and len(fields) == 16


def test_two_rank_alltoall_in_process():
    """Rank r seals p blocks for its peers, block (r -> q) travels to rank q, q opens it."""
    p, n = 2, 4096
    ctxs = [aead.AeadCtx(KEY), aead.AeadCtx(KEY)]  # every rank holds the same symmetric key
    send = [records(0x2A2A + r, p, n) for r in range(p)]
    wires = []
    for r in range(p):
        w = empty(p * (n + 28))
        coll.seal_blocks(ctxs[r], w, dev(send[r]), n, p)
        wires.append(host(w)[: p * (n + 28)].reshape(p, n + 28))
    for q in range(p):
        recv_wire = np.stack([wires[r][q] for r in range(p)])  # MPIR_Alltoall_impl on ciphertext
        out, st = empty(p * n), status_buf(p)
        coll.open_blocks(ctxs[q], out, dev(recv_wire), n, p, status=st)
        assert (host(st)[:p] == 1).all()
        got = host(out)[: p * n].reshape(p, n)
        for r in range(p):
            assert got[r].tobytes() == send[r][q].tobytes()


@pytest.mark.parametrize("n", [4096, 1 << 20])
def test_bench_alltoall_e2e_one_rank(n):
    """bench.py's BASELINE config-5 timing path (seal -> exchange -> open) on one rank: runs,
    every block authenticates and the rank gets its own plaintext back."""
    import bench

    res = bench.alltoall_e2e(0, None, lambda: None, n=n, steps=2, warmup=1, warmup_s=0.05)
    assert res["ranks"] == 1 and res["all_blocks_authenticated"] and res["recv_matches_peers"] and res["ms_per_call"] > 0


def _coll_rank(rank: int, ws: int, port: int, q, n: int = 3000):
    import os
    import traceback

    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    try:
        # RCCL between GPUs when every rank has one; otherwise (one GPU box) every rank shares
        # cuda:0 and the ciphertext moves over gloo through host memory
        rccl = torch.cuda.device_count() >= ws
        torch.cuda.set_device(rank if rccl else 0)
        dist.init_process_group("nccl" if rccl else "gloo", rank=rank, world_size=ws)
        ctx = aead.AeadCtx(KEY, device=torch.cuda.current_device())
        plain = lambda r, i: records(0xC011 + 16 * r + i, 1, n)[0]  # noqa: E731  block (rank r, index i)
        dv = lambda a: torch.from_numpy(np.ascontiguousarray(a).reshape(-1)).cuda()  # noqa: E731
        res = {}
        # alltoall: rank r sends block (r, i) to rank i — on a side stream (everything ordered on it)
        recv = torch.empty(ws * n, dtype=torch.uint8, device="cuda")
        side = torch.cuda.Stream()
        send = dv(np.stack([plain(rank, i) for i in range(ws)]))
        side.wait_stream(torch.cuda.current_stream())
        coll.alltoall(ctx, send, recv, n, stream=side)
        torch.cuda.current_stream().wait_stream(side)
        res["alltoall"] = np.array_equal(recv.cpu().numpy().reshape(ws, n), np.stack([plain(r, rank) for r in range(ws)]))
        # allgather
        recv = torch.empty(ws * n, dtype=torch.uint8, device="cuda")
        coll.allgather(ctx, dv(plain(rank, 0)), recv, n)
        res["allgather"] = np.array_equal(recv.cpu().numpy().reshape(ws, n), np.stack([plain(r, 0) for r in range(ws)]))
        # gather to root 1
        recv = torch.empty(ws * n, dtype=torch.uint8, device="cuda")
        coll.gather(ctx, dv(plain(rank, 1)), recv, n, root=1)
        res["gather"] = rank != 1 or np.array_equal(recv.cpu().numpy().reshape(ws, n), np.stack([plain(r, 1) for r in range(ws)]))
        # scatter from root 0: rank i gets block (0, i)
        recv = torch.empty(n, dtype=torch.uint8, device="cuda")
        coll.scatter(ctx, dv(np.stack([plain(0, i) for i in range(ws)])) if rank == 0 else None, recv, n, root=0)
        res["scatter"] = np.array_equal(recv.cpu().numpy(), plain(0, rank))
        # bcast from root 1
        buf = dv(plain(1, 7)) if rank == 1 else torch.zeros(n, dtype=torch.uint8, device="cuda")
        coll.bcast(ctx, buf, n, root=1)
        res["bcast"] = np.array_equal(buf.cpu().numpy(), plain(1, 7))
        if ws >= 3:
            # a sub-communicator {1, 2}: root 0 of the group is global rank 1 (MPI semantics)
            sub = dist.new_group([1, 2])
            if rank in (1, 2):
                g = rank - 1
                recv = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
                coll.gather(ctx, dv(plain(rank, 3)), recv, n, root=0, group=sub)
                res["sub_gather"] = g != 0 or np.array_equal(recv.cpu().numpy().reshape(2, n), np.stack([plain(1, 3), plain(2, 3)]))
                recv = torch.empty(n, dtype=torch.uint8, device="cuda")
                coll.scatter(ctx, dv(np.stack([plain(1, 4), plain(1, 5)])) if g == 0 else None, recv, n, root=0, group=sub)
                res["sub_scatter"] = np.array_equal(recv.cpu().numpy(), plain(1, 4 + g))
                buf = dv(plain(2, 6)) if g == 1 else torch.zeros(n, dtype=torch.uint8, device="cuda")
                coll.bcast(ctx, buf, n, root=1, group=sub)
                res["sub_bcast"] = np.array_equal(buf.cpu().numpy(), plain(2, 6))
            dist.barrier()
        torch.cuda.synchronize()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception:
        q.put((rank, traceback.format_exc()))


def _run_ranks(ws: int, n: int):
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    procs = [ctxm.Process(target=_coll_rank, args=(r, ws, port, q, n)) for r in range(ws)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=150) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
    for r in range(ws):
        assert isinstance(out[r], dict), out[r]
        assert all(out[r].values()), (r, out[r])


@pytest.mark.parametrize("n", [3000, 1 << 20])
def test_naive_collectives_two_processes(n):
    """The five naive secure collectives end to end across two processes (RCCL when each rank has
    a GPU, else gloo host transport with one GPU shared by both ranks), 3000-byte and config-5
    1 MiB blocks, alltoall on a non-current stream: every rank gets the reference semantics'
    plaintext back, every block authenticated."""
    _run_ranks(2, n)


def test_naive_collectives_subgroup_three_processes():
    """Three ranks; gather / scatter / bcast on the sub-communicator {1, 2} with group roots
    (root 0 of the group = global rank 1)."""
    _run_ranks(3, 4096)
