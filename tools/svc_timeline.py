#!/usr/bin/env python3
"""Where a served single message's time goes: the resident service kernel's
phase stamps (diagnostics build, service_kernels.hpp SVC_STAMP, 100 MHz wall clock) for single
GCM seals / opens from page-locked host memory, next to the host's time per call.

Phases (us, medians over the messages; per-workgroup phases take the slowest workgroup):
  publish     leader sees the seq -> descriptor in LDS (and published to the other workgroups)
  wg_start    -> the last workgroup starts the message
  compute     workgroup start -> its waves' record stores performed (input read over PCIe, AES,
              lane tree, chunk weight, output written over PCIe)
  post        -> its completion slot issued (system-scope release of its record bytes + two
              16-byte system-scope stores)
  gpu_span    leader sees the seq -> the last workgroup's completion issued
  host_call   the host's time per call (post, wait for the completion word, tag copy)
Run with the diagnostics library (make -C tools diag):  python tools/svc_timeline.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("CMPI_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcmpi_aead_tools.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cryptmpi_2022_amd import _native as N  # noqa: E402
from cryptmpi_2022_amd import aead  # noqa: E402


def main():
    msgs = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    probe = torch.zeros(8 * 32, dtype=torch.int64, device="cuda")
    side = torch.cuda.Stream()  # probe zeroing / reads: never a device-wide sync (the service is resident)
    hostbuf = torch.zeros(8 * 32, dtype=torch.int64).pin_memory()
    N.lib().cmpi_debug_set_svc_probe(probe.data_ptr())
    ctx = aead.AeadCtx(bytes(range(16)))
    ctx.service_start(20000)
    res = {}
    try:
        for n in (1024, 4096, 65536):
            pt = torch.randint(0, 256, (n,), dtype=torch.uint8).pin_memory().numpy()
            nonce = bytes(range(12))
            for op in ("seal", "open"):
                rows, host = [], []
                ct = ctx.seal(nonce, pt.tobytes())
                ctp = torch.from_numpy(np.frombuffer(ct, np.uint8).copy()).pin_memory().numpy()
                for i in range(msgs + 20):
                    with torch.cuda.stream(side):
                        probe.zero_()
                    side.synchronize()
                    t0 = time.perf_counter()
                    if op == "seal":
                        ctx.seal_host_batch(np.frombuffer(nonce, np.uint8)[None, :], pt[None, :])
                    else:
                        ctx.open_host_batch(np.frombuffer(nonce, np.uint8)[None, :], ctp[None, :])
                    t1 = time.perf_counter()
                    with torch.cuda.stream(side):
                        hostbuf.copy_(probe, non_blocking=True)
                    side.synchronize()
                    b = hostbuf.view(8, 32).numpy().copy()
                    b = b[b[:, 0] > 0]
                    if i >= 20 and len(b) == 1:
                        rows.append(b[0])
                        host.append((t1 - t0) * 1e6)
                if not rows:
                    res[f"{op}_{n}"] = {"error": "no stamps"}
                    continue
                r = np.array(rows, dtype=np.float64) / 100.0  # 100 MHz ticks -> us
                t0 = r[:, 0:1]
                r = r - t0
                start = r[:, 2:10]
                act = start > -t0  # workgroups that took part (stamp non-zero)
                ngrp = int(act[0].sum())
                wg_start = np.where(act, start, -np.inf).max(axis=1)
                comp = np.where(act, r[:, 10:18] - start, -np.inf).max(axis=1)
                done = np.where(act, r[:, 18:26], -np.inf).max(axis=1)
                med = lambda x: round(float(np.median(x)), 2)  # noqa: E731
                res[f"{op}_{n}"] = {
                    "workgroups": ngrp, "messages": len(rows),
                    "publish": med(r[:, 1]), "wg_start": med(wg_start), "compute": med(comp),
                    "post": med(np.where(act, r[:, 18:26] - r[:, 10:18], -np.inf).max(axis=1)),
                    "gpu_span": med(done), "host_call": med(host),
                    # workgroup 0's first unit (chunk 0 on the single-workgroup shapes), from its start
                    "u_first_keystream": med(r[:, 28] - r[:, 2]), "u_first_step": med(r[:, 29] - r[:, 2]),
                    "u_steps_done": med(r[:, 30] - r[:, 2]), "u_tree_weight": med(r[:, 31] - r[:, 2]),
                }
                print(json.dumps({f"{op}_{n}": res[f"{op}_{n}"]}), flush=True)
    finally:
        ctx.service_stop()
        N.lib().cmpi_debug_set_svc_probe(None)


if __name__ == "__main__":
    main()
