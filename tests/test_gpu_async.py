"""Asynchronous host batches (include/cmpi_async.h) — the MPI_Isend / MPI_Wait split of
isend.c:187-1260 / wait.c:244-1780: 64 outstanding requests of mixed sizes, pinned and pageable
buffers, seal and open (with forged records), completed in a different order than begun, every
byte against the oracle."""
import random

import numpy as np
import pytest
import torch

import oracle
from cryptmpi_2022_amd import _native as N
from cryptmpi_2022_amd import aead
from cryptmpi_2022_amd.synth import random_nonces, records

pytestmark = pytest.mark.gpu
KEY = bytes(range(16))


DIRECT_DEFAULT = (2 << 20) + 64  # cmpi_aead.hip g_host_direct


@pytest.fixture(params=[DIRECT_DEFAULT, 0], ids=["direct", "dma"])
def path(request):
    """Requests up to the threshold run the direct path (kernel on page-locked host memory);
    threshold 0 sends every request through H2D / kernel / D2H DMA."""
    N.lib().cmpi_debug_set_host_direct(request.param)
    yield request.param
    N.lib().cmpi_debug_set_host_direct(DIRECT_DEFAULT)


def _buf(shape, pinned: bool):
    if pinned:
        return torch.empty(shape, dtype=torch.uint8, pin_memory=True).numpy()
    return np.empty(shape, np.uint8)


def test_64_outstanding_seal_then_open(path):
    ctx = aead.AeadCtx(KEY)
    rng = random.Random(64)
    jobs = []
    for i in range(64):
        n = rng.choice([0, 1, 17, 1000, 1024, 4096, 65536, 100000])
        nrec = rng.choice([1, 3, 16])
        pinned = i % 2 == 0
        pt = records(0xA5 + i, nrec, n)
        if pinned:
            p = _buf(pt.shape, True)
            p[...] = pt
            pt = p
        nn = random_nonces(0xB5 + i, nrec)
        out = _buf((nrec, n + 16), pinned)
        jobs.append((pt.copy(), nn, out, ctx.seal_host_begin(nn, pt, out)))
    order = list(range(64))
    rng.shuffle(order)
    for i in order:
        pt, nn, out, req = jobs[i]
        if i % 3 == 0:  # MPI_Test polling
            while not req.test():
                pass
        else:
            assert req.wait() == N.CMPI_OK
        assert np.array_equal(out, oracle.gcm_seal_batch(KEY, nn, pt)), i
    # open them all back, forging one record in every 4th request
    opens = []
    for i, (pt, nn, out, _) in enumerate(jobs):
        ct = out.copy()
        forged = i % 4 == 1 and ct.shape[0] > 0
        if forged:
            ct[ct.shape[0] // 2, -1] ^= 1
        back = _buf(pt.shape, i % 2 == 1)
        st = np.full(ct.shape[0], -1, np.int32)
        opens.append((pt, back, st, forged, ctx.open_host_begin(nn, ct, back, st)))
    for i in reversed(range(64)):
        pt, back, st, forged, req = opens[i]
        rc = req.wait()
        if forged:
            k = pt.shape[0] // 2
            assert rc == N.CMPI_EAUTH and st[k] == 0 and (st[np.arange(len(st)) != k] == 1).all()
            assert not back[k].any()  # zero-filled (aead.h:276-278)
            mask = np.arange(len(st)) != k
            assert np.array_equal(back[mask], pt[mask])
        else:
            assert rc == N.CMPI_OK and (st == 1).all() and np.array_equal(back, pt), i


def test_async_ocb_and_overlap_with_device_work(path):
    ctx = aead.AeadCtx(KEY, "aes-128-ocb")
    reqs = []
    for i in range(8):
        pt = records(0xC0 + i, 4, 1 << 16)
        nn = random_nonces(0xD0 + i, 4)
        out = np.empty((4, (1 << 16) + 16), np.uint8)
        reqs.append((pt, nn, out, ctx.seal_host_begin(nn, pt, out)))
    # unrelated device work on the default stream meanwhile
    x = torch.randint(0, 255, (1 << 24,), dtype=torch.uint8, device="cuda")
    y = (x ^ 0x5A).sum()
    for pt, nn, out, r in reqs:
        assert r.wait() == N.CMPI_OK
        assert np.array_equal(out, oracle.ocb_seal_batch(KEY, nn, pt))
    torch.cuda.synchronize()
    assert int(y) >= 0
