#!/usr/bin/env python3
"""Pipelined host path sweep (cmpi_gcm_seal_host / _open_host, 65 536 x 1 KiB from page-locked
memory): staging slots (cmpi_debug_set_host_slots) x chunk bytes (cmpi_debug_set_host_chunk), on
THP-backed registered buffers and on torch pin_memory buffers.  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
GIB = float(1 << 30)


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
        pt[:] = 7
        for slots in (2, 3, 4):
            for chunk in (4, 8, 16):
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
                res[f"{kind}_slots{slots}_chunk{chunk}M"] = r
        assert back.tobytes() == pt.tobytes()
    L.cmpi_debug_set_host_slots(0)
    L.cmpi_debug_set_host_chunk(0)
    ctx.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
