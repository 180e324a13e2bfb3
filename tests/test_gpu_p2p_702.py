"""Two processes exchanging 702 pre-computed-counter messages (MPI_SEC_PreComputeCounter_Send_v4 /
_Recv_v4, send.c:1502-1987 / recv.c:1025-1403): rank 0 runs the sender (mask ring of stream A,
stream B for long messages, the precompute while its sends are pending), rank 1 the receiver
(the mask made from the header while the payload is in flight, then the XOR), both on the GPU
with device buffers and gloo carrying header and payload through host memory.  Each rank runs
launched and served (its CTR context's resident kernel, cmpi_service_start): every plaintext
arrives intact, and the sender's headers equal the oracle's."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
KEY = bytes(range(16))
SIZES = [1, 16, 1000, 4096, 30000, 65535, 65536, 200000, 1 << 20, 4096, 17, 70000]


def _rank(rank: int, port: int, served: bool, q):
    import os
    import traceback

    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2")
    try:
        import oracle
        from cryptmpi_2022_amd import aead, ctrmode
        from cryptmpi_2022_amd.synth import splitmix64_bytes

        torch.cuda.set_device(rank % max(torch.cuda.device_count(), 1))
        dev = f"cuda:{torch.cuda.current_device()}"
        dist.init_process_group("gloo", rank=rank, world_size=2)
        iv = splitmix64_bytes(0x702702, 32).tobytes()  # Send_common_IV of rank 0 = Recv_common_IV at rank 1
        ctx = aead.CipherCtx(KEY, "aes-128-ctr", device=torch.cuda.current_device())
        if served:
            ctx.service_start(20000)
        res = {}
        if rank == 0:
            s = ctrmode.Sender702(ctx, iv, ring_bytes=1 << 20, series_threads=8)
            o = oracle.Sender702(KEY, iv, max_bytes=1 << 20, series=8)
            for i, n in enumerate(SIZES):
                pt = splitmix64_bytes(0x7020 + i, n)
                ct = torch.empty(n, dtype=torch.uint8, device=dev)
                hdr, _ = s.send(ct, torch.from_numpy(pt).to(dev), n, pending_isends=i % 3)
                ohdr, _ = o.send(pt.tobytes(), pending=i % 3)
                res[f"hdr_{i}"] = hdr == ohdr
                dist.send(torch.tensor(list(hdr), dtype=torch.uint8), 1)
                s.precompute(n, 2)  # the reference's pre-computation while its Isends are pending
                o.precompute(n, 2)
                torch.cuda.synchronize()
                dist.send(ct.cpu(), 1)
            s.close()
        else:
            for i, n in enumerate(SIZES):
                h = torch.empty(26, dtype=torch.uint8)
                dist.recv(h, 0)
                hdr = bytes(h.tolist())
                mask = torch.empty(n + 1024, dtype=torch.uint8, device=dev)
                ml = ctrmode.recv702_premask(ctx, iv, hdr, mask)  # while the payload is in flight
                buf = torch.empty(n, dtype=torch.uint8)
                dist.recv(buf, 0)
                out = torch.empty(n, dtype=torch.uint8, device=dev)
                ctrmode.recv702(ctx, iv, hdr, out, buf.to(dev), mask=mask if ml else None, mask_len=ml)
                res[f"pt_{i}"] = np.array_equal(out.cpu().numpy(), splitmix64_bytes(0x7020 + i, n))
        if served:
            ctx.service_stop()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception:
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("served", [False, True])
def test_two_process_702_exchange(served):
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    procs = [ctxm.Process(target=_rank, args=(r, port, served, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=150) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        assert isinstance(out[r], dict), out[r]
        assert out[r] and all(out[r].values()), (r, out[r])
