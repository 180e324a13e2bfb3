"""BASELINE config 1's counterpart on this engine: a 2-process 64 KiB secure MPI_Send/MPI_Recv
ping-pong with 600 framing (send.c:221-337, recv.c:219-341) — host buffers, GPU seal/open through
the host-memory batch calls, torch.distributed (gloo) as the host transport — next to the same
ping-pong in plaintext over the same transport (what the reference's config 1 measures: SURVEY.md
§0.3, 401 never encrypts).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29555 tools/config1_exchange.py [--msg-bytes 65536] [--iters 200]

Rank 0 prints one JSON line: one-way latency per message (round trip / 2), secure and plaintext.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--msg-bytes", type=int, default=64 << 10)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--no-service", action="store_true", help="skip the resident-service leg")
    args = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist

    from cryptmpi_2022_amd import aead, p2p
    from cryptmpi_2022_amd.synth import splitmix64_bytes

    rank = int(os.environ["RANK"])
    ngpu = torch.cuda.device_count()
    dev = rank % max(ngpu, 1)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    ctx = aead.AeadCtx(bytes(range(16)), device=dev)
    ep = p2p.Endpoint(ctx, max_bytes=args.msg_bytes)
    # the MPI user buffers: page-locked, so the engine reads and writes them in place
    msg = torch.from_numpy(splitmix64_bytes(0xC1 + rank, args.msg_bytes)).pin_memory().numpy()
    rbuf = torch.empty(max(args.msg_bytes, 1), dtype=torch.uint8).pin_memory().numpy()
    peer = 1 - rank

    def secure_round():
        if rank == 0:
            ep.send(msg, peer)
            got = ep.recv(peer, out=rbuf)
        else:
            got = ep.recv(peer, out=rbuf)
            ep.send(got, peer)
        return got

    plain_t = torch.from_numpy(msg.copy())
    plain_r = torch.empty_like(plain_t)

    def plain_round():
        if rank == 0:
            dist.send(plain_t, peer)
            dist.recv(plain_r, peer)
        else:
            dist.recv(plain_r, peer)
            dist.send(plain_r, peer)

    ok = True

    def timed(fn) -> float:
        nonlocal ok
        for _ in range(args.warmup):
            got = fn()
            ok = ok and (fn is not secure_round or rank != 0 or np.array_equal(got, msg))
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            fn()
        dist.barrier()
        return (time.perf_counter() - t0) / args.iters / 2

    t_pl = timed(plain_round)
    t_sec = timed(secure_round)
    res = {"message_bytes": args.msg_bytes, "ranks": 2, "transport": "gloo (host memory)",
           "gpus": min(ngpu, 2), "framing": "600: header(25) + nonce||ct||tag",
           "secure_one_way_us": round(t_sec * 1e6, 2), "plaintext_one_way_us": round(t_pl * 1e6, 2),
           "crypto_added_us": round((t_sec - t_pl) * 1e6, 2)}
    if not args.no_service:  # the same exchange with each rank's messages served by its resident kernel
        ctx.service_start(0)
        t_svc = timed(secure_round)
        ok = ok and ctx.service_running()
        ctx.service_stop()
        res.update({"secure_service_one_way_us": round(t_svc * 1e6, 2),
                    "crypto_added_service_us": round((t_svc - t_pl) * 1e6, 2),
                    "service": "cmpi_service_start per rank (include/cmpi_service.h)"})
    res["round_trips_verified"] = ok
    if rank == 0:
        print(json.dumps(res))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
