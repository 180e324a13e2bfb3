"""The kernel-timing hook bench.py's roofline uses (cmpi_debug_time_next_launch: the call's kernels
through hipExtLaunchKernel with start / stop events, first kernel's start to last kernel's end):
the time it reports lies inside the stream bracket of the same call (fence-free events recorded
around it on the stream), covers both launches of a two-launch seal (flow kernel + XOR combine),
and leaves the output bit-exact."""
import numpy as np
import pytest

import oracle
from cryptmpi_2022_amd import _native as N
from cryptmpi_2022_amd import aead
from cryptmpi_2022_amd.synth import random_nonces, records
from tests.gpu_util import dev, empty, host

pytestmark = pytest.mark.gpu
KEY = bytes(range(16))


def _time_seal(ctx, n, nrec, reps=5):
    import torch

    L = N.lib()
    pt = records(0x71 + n, nrec, n)
    nonces = random_nonces(0x72 + n, nrec)
    d_pt, d_n = dev(pt), dev(nonces)
    out = empty(nrec * (n + 16))
    st = torch.cuda.current_stream().cuda_stream
    ev = [L.cmpi_debug_event_new() for _ in range(4)]
    kern, br = [], []
    try:
        for _ in range(reps):
            L.cmpi_debug_event_record(ev[0], st)
            L.cmpi_debug_time_next_launch(ev[2], ev[3])
            ctx.seal_batch(out, d_pt, d_n, n, nrec)
            L.cmpi_debug_time_next_launch(None, None)
            L.cmpi_debug_event_record(ev[1], st)
            torch.cuda.synchronize()
            kern.append(L.cmpi_debug_event_ms(ev[2], ev[3]))
            br.append(L.cmpi_debug_event_ms(ev[0], ev[1]))
    finally:
        for e in ev:
            L.cmpi_debug_event_free(e)
    got = host(out)[: nrec * (n + 16)].reshape(nrec, n + 16)
    return kern, br, got, pt, nonces


@pytest.mark.parametrize("n,nrec,launches", [(1024, 65536, 1), (1 << 20, 8, 2), (1000, 2048, 2)])
def test_kernel_timing_hook(n, nrec, launches):
    ctx = aead.AeadCtx(KEY)
    kern, br, got, pt, nonces = _time_seal(ctx, n, nrec)
    assert all(k > 0.0 for k in kern), kern
    assert all(k <= b * 1.02 + 1e-3 for k, b in zip(kern, br)), (kern, br)  # inside the bracket
    want = oracle.gcm_seal_batch(KEY, nonces, pt)
    assert np.array_equal(got, want)
    if launches == 2:  # these shapes take the flow plan (L = 64): flow kernel + XOR combine, both timed
        assert aead.gcm_plan(ctx, n, nrec)[0] == 64
