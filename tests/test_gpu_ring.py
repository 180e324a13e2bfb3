"""CTR precompute mask ring on the device vs the oracle's restatement of send.c:1162-1465 /
recv.c:954-1023: identical ciphertext and identical bookkeeping (start, end, compute_size,
counter, counter_needto_send) over random generate/encrypt sequences, with small rings so the
wrap-around branches run, and at the reference's 8 MiB."""
import random

import numpy as np
import pytest

import oracle
from cryptmpi_2022_amd import aead, ring
from cryptmpi_2022_amd.synth import splitmix64_bytes

from tests.gpu_util import dev, empty, host

pytestmark = pytest.mark.gpu
KEY = bytes(range(16))


@pytest.fixture(params=[False, True], ids=["launch", "served"])
def ctx(request):
    """CTR context; served: its message service started (ring XORs / keystreams up to 64 KiB
    run on the resident kernel, ring_host.hpp Served)."""
    c = aead.CipherCtx(KEY, "aes-128-ctr")
    if request.param:
        c.service_start()
    yield c
    if request.param:
        c.service_stop()


@pytest.mark.parametrize("ring_bytes,seed", [(4096, 1), (8192, 2), (65536, 3), (8 << 20, 4)])
def test_ring_matches_oracle(ring_bytes, seed, ctx):
    iv = splitmix64_bytes(0x1A + seed, 16).tobytes()
    if seed == 2:
        iv = bytes(12) + b"\xff\xff\xff\xf0"  # counter blocks carry through the 32-bit tail
    g = ring.CtrRing(ctx, iv, ring_bytes)
    o = oracle.Ring(KEY, iv, ring_bytes)
    rnd = random.Random(seed)
    big = ring_bytes >= (1 << 20)
    import torch

    for step in range(60):
        before = g.state()
        if rnd.random() < 0.5:
            gen = rnd.choice([1, 16, 100, 1000, 1024, 3000]) if not big else rnd.choice([4096, 1 << 20, 3 << 20])
            op = ("generate", gen)
            assert g.generate(gen) == o.generate(gen), step
        else:
            n = rnd.choice([0, 1, 15, 16, 17, 100, 999, 2048, 5000]) if not big else rnd.choice([17, 65536, 2 << 20])
            op = ("encrypt", n)
            pt = splitmix64_bytes(seed * 1000 + step, n)
            out = empty(max(n, 1), fill=0)
            inp = dev(pt) if n else empty(1)
            g.encrypt(out, inp, n)
        try:  # each step's launches complete before the next: a device fault names its step and op
            torch.cuda.synchronize()
        except Exception as e:
            raise AssertionError(f"device fault at step {step} {op}, ring state before {before}") from e
        if op[0] == "encrypt":
            want = o.encrypt(pt.tobytes())
            assert host(out)[:n].tobytes() == want, step
            del inp
        assert g.state() == o.state(), step


@pytest.mark.parametrize("n,mask_len,counter", [(100, 40, 0), (5000, 4096, 7), (4096, 8192, 3), (33, 0, 2**32 - 1)])
def test_mask_decrypt_matches_oracle(n, mask_len, counter, ctx):
    iv = splitmix64_bytes(0x77 + n, 16).tobytes()
    mask = splitmix64_bytes(0x78 + n, mask_len)
    ct = splitmix64_bytes(0x79 + n, n)
    out = empty(n)
    ring.mask_decrypt(ctx, out, dev(ct), n, dev(mask) if mask_len else None, mask_len, iv, counter)
    assert host(out)[:n].tobytes() == oracle.mask_decrypt(KEY, iv, counter, mask.tobytes(), ct.tobytes())


def test_sender_ring_receiver_mask_round_trip(ctx):
    """A sender encrypting through its ring and a receiver holding the same keystream as its
    precomputed dec mask recover the plaintext (the 702 pairing of send.c / recv.c)."""
    iv = bytes(range(32, 48))
    g = ring.CtrRing(ctx, iv, 1 << 16)
    assert g.generate(10000) == 1
    n = 30000
    pt = splitmix64_bytes(0xABC, n)
    ct = empty(n)
    g.encrypt(ct, dev(pt), n)
    # receiver: mask = keystream of counters 0.. for the first 10000 bytes (rounded), CTR after
    mask = empty(10016)
    ctx.keystream(mask, 10016 // 16, oracle.iv_count(iv, 0))
    out = empty(n)
    ring.mask_decrypt(ctx, out, ct, n, mask, 10016, iv, 626)  # 10016/16 blocks from the ring
    assert host(out)[:n].tobytes() == pt.tobytes()
    assert g.state()["counter_needto_send"] == (n + 15) // 16


@pytest.mark.parametrize("rounds", [1, 3])
def test_ring_fill_and_encrypt_on_two_streams(rounds, ctx):
    """the ring is filled on stream B behind ~10 ms of queued GPU work and the
    XOR that consumes it runs on stream A; the XOR must wait for the fill (RingOrder is built in
    place, so the cross-stream wait is not skipped) and the bytes must match the oracle."""
    import torch

    iv = splitmix64_bytes(0x2B, 16).tobytes()
    g = ring.CtrRing(ctx, iv, 65536)
    o = oracle.Ring(KEY, iv, 65536)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for r in range(rounds):
        n = 4096 + 16 * r
        pt = splitmix64_bytes(0x2C + r, n)
        inp, out = dev(pt), empty(n, fill=0)
        torch.cuda.synchronize()
        with torch.cuda.stream(sb):
            torch.cuda._sleep(20_000_000)  # long work ahead of the fill on stream B
        assert g.generate(n, stream=sb) == o.generate(n)
        g.encrypt(out, inp, n, stream=sa)
        torch.cuda.synchronize()
        assert host(out)[:n].tobytes() == o.encrypt(pt.tobytes()), r
        assert g.state() == o.state(), r
