#!/usr/bin/env python3
"""Pipelined host path sweep (cmpi_gcm_seal_host / _open_host, 65 536 x 1 KiB from page-locked
memory): staging slots (SWEEP_SLOTS) (cmpi_debug_set_host_slots) x chunk MiB (SWEEP_CHUNKS_MIB; cmpi_debug_set_host_chunk) x
output modes (SWEEP_OUT_DIRECT: cmpi_debug_set_host_out_direct's 0, 1, 4, 5, and 9 = the whole batch
on the direct path, the kernel reading and writing host memory), on
THP-backed registered buffers and on torch pin_memory buffers.  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
GIB = float(1 << 30)
SLOTS = tuple(int(x) for x in os.environ.get("SWEEP_SLOTS", "2,3,4").split(","))
CHUNKS = tuple(int(x) for x in os.environ.get("SWEEP_CHUNKS_MIB", "4,8,16").split(","))
DIRECT_DEFAULT = (2 << 20) + 64  # cmpi_aead.hip g_host_direct
OUTD = tuple(int(x) for x in os.environ.get("SWEEP_OUT_DIRECT", "0").split(","))


def main() -> None:
    import torch

    from cryptmpi_2022_amd import _native as N
    from cryptmpi_2022_amd import aead
    from tools.host_regress_probe import thp_buffer

    L = N.lib()
    n, nrec = 1024, 65536
    bufs = {"thp": (thp_buffer(nrec * n), thp_buffer(nrec * (n + 16)), thp_buffer(nrec * 12), thp_buffer(nrec * n)),
            "torch_pin": tuple(torch.randint(0, 256, (sz,), dtype=torch.uint8).pin_memory().numpy()
                               for sz in (nrec * n, nrec * (n + 16), nrec * 12, nrec * n))}
    ctx = aead.AeadCtx(bytes(range(16)))
    st = (ctypes.c_int32 * nrec)()
    P = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    res = {}
    for kind, (pt, ct, nn, back) in bufs.items():
        pt[:] = np.random.default_rng(5).integers(0, 256, pt.size, dtype=np.uint8)
        nn[:] = np.random.default_rng(6).integers(0, 256, nn.size, dtype=np.uint8)
        ref_ct = None
        for slots, chunk, od in [(a, b, c) for c in OUTD for a in SLOTS for b in CHUNKS]:
            L.cmpi_debug_set_host_out_direct(od if od < 9 else 0)
            L.cmpi_debug_set_host_direct(1 << 30 if od == 9 else DIRECT_DEFAULT)  # 9: the kernel reads and writes host memory
            L.cmpi_debug_set_host_slots(slots)
            L.cmpi_debug_set_host_chunk(chunk << 20)

            def seal():
                N.check(L.cmpi_gcm_seal_host(ctx.handle, P(ct), n + 16, P(pt), n, P(nn), 12, n, nrec))

            def opn():
                N.check(L.cmpi_gcm_open_host(ctx.handle, P(back), n, P(ct), n + 16, P(nn), 12, n, nrec, st))

            r = {}
            for name, fn in (("seal", seal), ("open", opn)):
                for _ in range(3):
                    fn()
                t0 = time.perf_counter()
                for _ in range(8):
                    fn()
                r[name] = round(nrec * n * 8 / (time.perf_counter() - t0) / GIB, 2)
            res[f"{kind}_slots{slots}_chunk{chunk}M" + (f"_outdirect{od}" if len(OUTD) > 1 else "")] = r
            assert back.tobytes() == pt.tobytes()
            if ref_ct is None:
                ref_ct = ct.tobytes()
            assert ct.tobytes() == ref_ct  # same nonces: every setting seals the same bytes
            back[:] = 0
    L.cmpi_debug_set_host_slots(0)
    L.cmpi_debug_set_host_chunk(0)
    L.cmpi_debug_set_host_out_direct(0)
    L.cmpi_debug_set_host_direct(DIRECT_DEFAULT)
    ctx.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
