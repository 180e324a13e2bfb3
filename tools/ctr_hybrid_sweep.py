#!/usr/bin/env python3
"""Config 4 (1 GiB CTR XOR) rate vs the bitsliced share of the stream (cmpi_debug_set_ctr_hybrid):
per share, 3 s of back-to-back calls (sustained clocks), then 50 timed calls between two events;
the output of every share is compared with the T-table-only output.
usage: python tools/ctr_hybrid_sweep.py [permille ...]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cryptmpi_2022_amd import _native as N  # noqa: E402
from cryptmpi_2022_amd import aead  # noqa: E402


def main() -> None:
    shares = [int(x) for x in sys.argv[1:]] or [0, 100, 150, 200, 250, 0]
    n = 1 << 30
    L = N.lib()
    g = torch.Generator(device="cuda").manual_seed(5)
    pt = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.empty_like(pt)
    ref = None
    ctx = aead.CipherCtx(bytes(range(16)), "aes-128-ctr")
    cb = bytes.fromhex("f0f1f2f3f4f5f6f7f8f9fafbfcfdfeff")
    for pm in shares:
        L.cmpi_debug_set_ctr_hybrid(64 << 20, pm)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 3.0:
            for _ in range(8):
                ctx.ctr_xor(out, pt, n, cb)
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            ctx.ctr_xor(out, pt, n, cb)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 50
        if ref is None:
            ref = out.clone()
        same = bool(torch.equal(out, ref))
        print(json.dumps({"permille": pm, "ms": round(ms, 4), "GiBps": round(n / (ms * 1e-3) / 2**30, 1), "same_as_ttable": same}),
              flush=True)
    L.cmpi_debug_set_ctr_hybrid(64 << 20, 0)


if __name__ == "__main__":
    main()
