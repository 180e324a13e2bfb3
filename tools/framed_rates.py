#!/usr/bin/env python3
"""602 message rates: an 8 MiB message (mode '1', 16 outer messages of 512 KiB,
send.c:729-850) with its per-message sub-key K' = AES_K(V) derived on the device.

  device   : re-key (cmpi_ctx_rekey_subkey) + cmpi_602_seal / + cmpi_602_open, device buffers,
             HIP events on the stream, back to back;
  host     : from host memory (pageable / page-locked), one request per outer message:
             'stepwise' = begin(o), wait(o) in turn (each outer sealed, then sent); 'pipelined' =
             every outer begun before outer 0 is waited (the reference's overlap of the seal of outer
             k+1 with MPI_Isend of k); the receiver likewise with open.
Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cryptmpi_2022_amd import _native as N  # noqa: E402
from cryptmpi_2022_amd import aead, frame  # noqa: E402

KEY = bytes(range(16))


def main(n=8 << 20, iters=40):
    res = {"message_bytes": n}
    plan = frame.plan602(n, 8, 0)
    res["plan"] = plan.as_dict()
    rand16 = bytes(range(16, 32))
    header = frame.header602(plan, rand16)
    master = aead.AeadCtx(KEY)
    seg = aead.AeadCtx(bytes(16))
    st = torch.cuda.current_stream()
    seg.rekey_subkey(master, header[4:20], stream=st)
    pt = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    wire = torch.empty(plan.wire_bytes, dtype=torch.uint8, device="cuda")
    back = torch.empty(n, dtype=torch.uint8, device="cuda")
    L = N.lib()
    ev = [L.cmpi_debug_event_new() for _ in range(3)]
    s_ = st.cuda_stream

    def dev_round(open_too: bool):
        seg.rekey_subkey(master, header[4:20], stream=st)
        frame.seal602(seg, plan, header, wire, pt, stream=st)
        if open_too:
            frame.open602(seg, header, back, wire, stream=st)

    for _ in range(10):
        dev_round(True)
    torch.cuda.synchronize()
    for key, open_too in (("rekey_seal_us", False), ("rekey_seal_open_us", True)):
        L.cmpi_debug_event_record(ev[0], s_)
        for _ in range(iters):
            dev_round(open_too)
        L.cmpi_debug_event_record(ev[1], s_)
        torch.cuda.synchronize()
        res.setdefault("device", {})[key] = round(L.cmpi_debug_event_ms(ev[0], ev[1]) * 1e3 / iters, 2)
    assert torch.equal(back, pt)
    res["device"]["seal_GiBps"] = round(n / (res["device"]["rekey_seal_us"] * 1e-6) / (1 << 30), 2)

    h_pt = pt.cpu().numpy()
    for kind in ("pageable", "pinned"):
        if kind == "pinned":
            t1 = torch.from_numpy(h_pt.copy()).pin_memory()
            t2 = torch.empty(plan.wire_bytes, dtype=torch.uint8).pin_memory()
            t3 = torch.empty(n, dtype=torch.uint8).pin_memory()
            src, hw, out = t1.numpy(), t2.numpy(), t3.numpy()
        else:
            src, hw, out = h_pt.copy(), np.empty(plan.wire_bytes, np.uint8), np.empty(n, np.uint8)
        r = {}

        def stepwise_seal():
            for o in range(plan.outer):
                frame.seal602_host_begin(seg, plan, header, hw, src, o).wait()

        def pipelined_seal():
            reqs = [frame.seal602_host_begin(seg, plan, header, hw, src, o) for o in range(plan.outer)]
            for q in reqs:
                q.wait()

        def stepwise_open():
            for o in range(plan.outer):
                frame.open602_host_begin(seg, header, out, hw, o).wait()

        def pipelined_open():
            reqs = [frame.open602_host_begin(seg, header, out, hw, o) for o in range(plan.outer)]
            for q in reqs:
                q.wait()

        for name, fn in (("seal_stepwise", stepwise_seal), ("seal_pipelined", pipelined_seal),
                         ("open_stepwise", stepwise_open), ("open_pipelined", pipelined_open)):
            for _ in range(3):
                fn()
            best = float("inf")
            for _ in range(8):
                t0 = time.perf_counter()
                fn()
                best = min(best, time.perf_counter() - t0)
            r[name + "_us"] = round(best * 1e6, 1)
            r[name + "_GiBps"] = round(n / best / (1 << 30), 2)
        assert out.tobytes() == h_pt.tobytes()
        res["host_" + kind] = r
    for e in ev:
        L.cmpi_debug_event_free(e)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
