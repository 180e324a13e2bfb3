#!/usr/bin/env python3
"""Per-message cost of the 602 path on the device (send.c:339-884): re-key the segment context
to K' = AES_K(V) (key-setup kernel) + seal all segments with in-kernel 602 nonces/prefixes;
and the receiver's open.  HIP-event medians per message, device-resident buffers."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cryptmpi_2022_amd import aead, frame  # noqa: E402

KEY = bytes(range(16))
master = aead.AeadCtx(KEY)
seg = aead.AeadCtx(bytes(16))
res = {}


def med(fn, reps=9):
    ts = []
    for _ in range(reps):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(4):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 4)
    return sorted(ts)[len(ts) // 2]


steps = [int(x) for x in os.environ.get("AB602_STEPS", "0").split(",")]
for n, S in [(n, S) for n in (1 << 16, 1 << 20, 8 << 20) for S in steps]:
    aead.force_wide(1 if S else 0, S)
    plan = frame.plan602(n, series_threads=8)
    rand16 = bytes(range(100, 116))
    hdr = frame.header602(plan, rand16)
    pt = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    wire = torch.empty(plan.wire_bytes, dtype=torch.uint8, device="cuda")
    back = torch.empty(n, dtype=torch.uint8, device="cuda")
    st = torch.zeros(plan.nseg, dtype=torch.int32, device="cuda")

    def rekey():
        seg.rekey_subkey(master, rand16[:16])

    def seal():
        frame.seal602(seg, plan, hdr, wire, pt)

    def both():
        rekey()
        seal()

    def opn():
        frame.open602(seg, hdr, back, wire, status=st)

    both()
    opn()
    torch.cuda.synchronize()
    ok = bool((st == 1).all()) and torch.equal(back, pt)
    t_rk, t_seal, t_both, t_open = med(rekey), med(seal), med(both), med(opn)
    key = f"602_{n >> 10}KiB" + (f"_S{S}" if S else "")
    res[key] = {"plan": plan.as_dict(), "gcm_plan": aead.gcm_plan(seg, plan.chop, plan.nseg), "rekey_us": round(t_rk * 1e3, 1),
                                "seal_us": round(t_seal * 1e3, 1), "rekey_seal_us": round(t_both * 1e3, 1),
                                "open_us": round(t_open * 1e3, 1),
                                "seal_GiBps": round(n / (t_both * 1e-3) / 2**30, 1), "round_trip_ok": ok}
    print(key, {k: v for k, v in res[key].items() if k != "plan"}, flush=True)
aead.force_wide(0, 0)
print(json.dumps(res))
