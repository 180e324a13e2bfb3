"""The N>1 path of bench.py on CPU: two gloo ranks, each with its own timed wall clock; the
job rate must use the MAX over ranks and count every rank's bytes (weak scaling)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank: int, ws: int, port: int, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    import bench

    wall = 1.0 + rank  # rank 1 is the slow one
    wall_max, value = bench.aggregate(wall, per_rank_bytes=1 << 30, steps=4, pg=dist, device="cpu")
    q.put((rank, wall_max, value))
    dist.destroy_process_group()


def test_aggregate_max_over_ranks_two_gloo_ranks():
    ws, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, wall_max, value in res:
        assert wall_max == 2.0                          # slowest rank's clock
        assert abs(value - 2 * 4 * 1.0 / 2.0) < 1e-12  # 2 ranks x 4 steps x 1 GiB / 2 s


def test_aggregate_single_rank():
    import bench

    wall_max, value = bench.aggregate(0.5, per_rank_bytes=1 << 30, steps=2, pg=None, device="cpu")
    assert wall_max == 0.5 and abs(value - 4.0) < 1e-12
