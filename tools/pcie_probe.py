#!/usr/bin/env python3
"""PCIe probe on the GPU box: pinned H2D alone, D2H alone, and both at once on two streams
(full duplex?), 64 MiB, plus chunked versions (8 x 8 MiB) — the ceiling of the host path."""
import json
import time

import torch

MB = 1 << 20
n = 64 * MB
h_src = torch.empty(n, dtype=torch.uint8).pin_memory()
h_dst = torch.empty(n, dtype=torch.uint8).pin_memory()
d_a = torch.empty(n, dtype=torch.uint8, device="cuda")
d_b = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def rate(fn, nbytes, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return round(nbytes * reps / (time.perf_counter() - t0) / 1e9, 2)


def h2d():
    with torch.cuda.stream(s1):
        d_a.copy_(h_src, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        h_dst.copy_(d_b, non_blocking=True)


def both():
    h2d()
    d2h()


def chunked(k=8):
    c = n // k
    for i in range(k):
        with torch.cuda.stream(s1):
            d_a[i * c:(i + 1) * c].copy_(h_src[i * c:(i + 1) * c], non_blocking=True)
        with torch.cuda.stream(s2):
            h_dst[i * c:(i + 1) * c].copy_(d_b[i * c:(i + 1) * c], non_blocking=True)


s3, s4 = torch.cuda.Stream(), torch.cuda.Stream()


def split2(h2d_on=True, d2h_on=True):  # each direction as two concurrent copies on two streams
    c = n // 2
    for i, (sa, sb) in enumerate(((s1, s2), (s3, s4))):
        if h2d_on:
            with torch.cuda.stream(sa):
                d_a[i * c:(i + 1) * c].copy_(h_src[i * c:(i + 1) * c], non_blocking=True)
        if d2h_on:
            with torch.cuda.stream(sb):
                h_dst[i * c:(i + 1) * c].copy_(d_b[i * c:(i + 1) * c], non_blocking=True)


res = {"h2d_GBps": rate(h2d, n), "d2h_GBps": rate(d2h, n), "both_GBps_each_dir": rate(both, n),
       "chunked8_both_GBps_each_dir": rate(chunked, n),
       "h2d_2streams_GBps": rate(lambda: split2(True, False), n),
       "d2h_2streams_GBps": rate(lambda: split2(False, True), n),
       "both_2streams_each_GBps_each_dir": rate(split2, n)}
print(json.dumps(res))
