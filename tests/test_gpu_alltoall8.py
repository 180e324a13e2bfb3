"""BASELINE config 5 at its own rank count: 8 ranks x 8 peer blocks of 1 MiB through
MPIR_Naive_Sec_Alltoall (MV/src/mpi/coll/alltoall.c:764-836; MPICH twin alltoall_intra_brucks.c).

Eight processes share cuda:0 (the test box has one GPU) and exchange the wire blocks over gloo
through host memory.  Every rank:
  * runs coll.alltoall with 1 MiB blocks and gets exactly block `rank` of every peer back;
  * seals its 8 peer blocks into the wire layout nonce(12)||ct||tag(16) and compares every wire
    block with the oracle (oracle/gcm_ref.c) under the nonce the block carries; the 64 nonces
    of the 8 ranks are pairwise distinct (fresh nonce per block, the reference's RAND_bytes);
  * exchanges those wire blocks; rank FORGE_RANK flips one ciphertext bit of the block from
    FORGE_SRC before opening: that block alone fails (status 0, plaintext zero-filled) and
    coll's checked open raises "Decryption error: alltoall" (alltoall.c:831);
  * runs bench.alltoall_e2e with p = 8 (one block per peer, the bench's config-5 path): every
    block authenticated, every rank received its peers' plaintext, wire parity vs OpenSSL.
Timing from this run means nothing (eight ranks on one GPU); correctness at 8 ranks is the point."""
import numpy as np
import pytest

import oracle
from cryptmpi_2022_amd import _native as NT
from cryptmpi_2022_amd import aead, coll
from cryptmpi_2022_amd.synth import records

pytestmark = pytest.mark.gpu
KEY = bytes.fromhex("000102030405060708090a0b0c0d0e0f")  # bench.KEY: alltoall_e2e's key
WS, N = 8, 1 << 20
FORGE_RANK, FORGE_SRC = 5, 2


def _plain(r: int, i: int) -> np.ndarray:  # block (rank r -> peer i)
    return records(0xA2A8 + 16 * r + i, 1, N)[0]


def _rank_main(rank: int, port: int, q) -> None:
    import os
    import traceback

    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WS))
    res = {}
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=WS)
        ctx = aead.AeadCtx(KEY, device=0)
        dv = lambda a: torch.from_numpy(np.ascontiguousarray(a).reshape(-1)).cuda()  # noqa: E731
        mine = np.stack([_plain(rank, i) for i in range(WS)])
        expect = np.stack([_plain(r, rank) for r in range(WS)])

        # (1) the collective as a caller uses it
        recv = torch.empty(WS * N, dtype=torch.uint8, device="cuda")
        coll.alltoall(ctx, dv(mine), recv, N)
        res["coll_alltoall"] = bool(np.array_equal(recv.cpu().numpy().reshape(WS, N), expect))

        # (2) this rank's wire blocks vs the oracle under the nonces they carry
        wire = torch.empty(WS * (N + 28), dtype=torch.uint8, device="cuda")
        coll.seal_blocks(ctx, wire, dv(mine), N, WS)
        w = wire.cpu()
        wn = w.numpy().reshape(WS, N + 28)
        nonces = np.ascontiguousarray(wn[:, :12])
        res["wire_vs_oracle"] = bool(np.array_equal(wn[:, 12:], oracle.gcm_seal_batch(KEY, nonces, mine)))
        allnon = [None] * WS
        dist.all_gather_object(allnon, [bytes(x) for x in nonces])
        res["nonces_unique_64"] = len({x for lst in allnon for x in lst}) == WS * WS

        # (3) exchange; one forged block on one rank
        h_in = torch.empty_like(w)
        dist.all_to_all_single(h_in, w)
        if rank == FORGE_RANK:
            h_in[FORGE_SRC * (N + 28) + 12 + 777] ^= 0x10
        out = torch.full((WS * N,), 0xEE, dtype=torch.uint8, device="cuda")
        st = torch.full((WS,), 7, dtype=torch.int32, device="cuda")
        coll.open_blocks(ctx, out, h_in.cuda(), N, WS, status=st)
        s, got = st.cpu().numpy(), out.cpu().numpy().reshape(WS, N)
        if rank == FORGE_RANK:
            good = [i for i in range(WS) if i != FORGE_SRC]
            res["forged_rejected"] = bool(s[FORGE_SRC] == 0 and (s[good] == 1).all() and not got[FORGE_SRC].any()
                                          and np.array_equal(got[good], expect[good]))
            try:
                coll._open_checked(ctx, out, h_in.cuda(), N, WS, "alltoall")
                res["forged_raises"] = False
            except NT.CmpiError as e:
                res["forged_raises"] = e.code == NT.CMPI_EAUTH and "Decryption error: alltoall" in str(e)
        else:
            res["opened"] = bool((s == 1).all() and np.array_equal(got, expect))

        # (4) the bench's config-5 path at p = 8
        import bench

        r = bench.alltoall_e2e(0, dist, dist.barrier, n=N, steps=2, warmup=1, warmup_s=0.05)
        res["bench_e2e"] = (r["ranks"] == WS and r["blocks_per_rank"] == WS and r["all_blocks_authenticated"]
                            and r["recv_matches_peers"] and r["parity_cpu"] and "gloo" in r["transport"])
        if not res["bench_e2e"]:
            res["bench_e2e_detail"] = str(r)
            res["bench_e2e"] = False
        ctx.close()
        torch.cuda.synchronize()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception:
        q.put((rank, traceback.format_exc()))


def test_config5_alltoall_eight_ranks():
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    procs = [ctxm.Process(target=_rank_main, args=(r, port, q)) for r in range(WS)]
    for p in procs:
        p.start()
    try:
        out = dict(q.get(timeout=110) for _ in range(WS))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(WS):
        assert isinstance(out[r], dict), out[r]
        assert all(v for k, v in out[r].items() if not k.endswith("_detail")), (r, out[r])
    assert "forged_rejected" in out[FORGE_RANK] and out[FORGE_RANK]["forged_raises"]
