"""Counter-mode messages on the GPU vs the oracle's statement-by-statement restatement
(oracle/ctrmode_ref.c): the 700 base counter (send.c:886-1017 / recv.c:812-940) and the 702
pre-computed counter (send.c:1502-1987 / recv.c:1025-1403) — 26-byte headers, ciphertext, the
sender's ring / counter state after every call, the receiver's in-flight mask and its direct
path, over message sequences that cross every branch (ring hit '0', stream B '1', mode '4',
pipelined '1' > 1 MiB, ring wrap with small rings, multithreaded generation, empty messages).
Every test runs twice: with a launch per op, and with the context's message service started
(`served`: the ring XORs and keystreams of messages up to 64 KiB run on the resident kernel,
ring_host.hpp Served)."""
import random

import numpy as np

import pytest
import torch

import oracle
from cryptmpi_2022_amd import aead, ctrmode
from cryptmpi_2022_amd.synth import splitmix64_bytes

from tests.gpu_util import dev, empty, host

pytestmark = pytest.mark.gpu
KEY = bytes(range(16))
IV32 = splitmix64_bytes(0x702, 32).tobytes()


@pytest.fixture(params=[False, True], ids=["launch", "served"])
def ctx(request):
    c = aead.CipherCtx(KEY, "aes-128-ctr")
    if request.param:
        c.service_start()
    yield c
    if request.param:
        c.service_stop()


def _seq(seed: int):
    rng = random.Random(seed)
    sizes = [0, 1, 15, 16, 17, 1000, 1024, 1025, 3000, 4095, 4096, 65535, 65536, 65537, 300000, 1048575,
             1048576, (1 << 21) + 7]
    sizes += [rng.randrange(1, 70000) for _ in range(25)] + [rng.randrange(65536, 3 << 20) for _ in range(4)]
    rng.shuffle(sizes)
    return [(n, rng.randrange(0, 5), rng.choice([0, 0, 70])) for n in sizes]


@pytest.mark.parametrize("ring_bytes,series,seed", [(8 << 20, 16, 1), (65536, 4, 2), (20480, 1, 3)])
def test_702_sender_sequence_vs_oracle(ring_bytes, series, seed, ctx):
    s = ctrmode.Sender702(ctx, IV32, ring_bytes=ring_bytes, series_threads=series)
    o = oracle.Sender702(KEY, IV32, max_bytes=ring_bytes, series=series)
    assert s.state() == o.state()
    for n, rounds, pending in _seq(seed):
        pt = splitmix64_bytes(n * 7 + seed, n)
        out = empty(max(n, 1), fill=0xEE)
        hdr, nseg = s.send(out, dev(pt) if n else empty(1), n, pending_isends=pending)
        ohdr, oct_ = o.send(pt.tobytes(), pending=pending)
        assert hdr == ohdr, (n, hdr.hex(), ohdr.hex())
        assert host(out)[:n].tobytes() == oct_, n
        assert nseg >= 1
        assert s.state() == o.state(), n
        assert s.precompute(n, rounds) == o.precompute(n, rounds)
        assert s.state() == o.state(), ("precompute", n, rounds)
    s.close()


@pytest.mark.parametrize("n", [0, 1, 16, 17, 1000, 1024, 1025, 4096, 5000, 65535, 65536, 100001, 1048576, (1 << 21) + 7])
def test_702_receiver_premask_and_direct(n, ctx):
    """recv.c:1107-1220: the mask made while the payload is in flight, then XOR; or the direct
    path when the payload arrived first — both equal the oracle and round-trip the sender."""
    s = ctrmode.Sender702(ctx, IV32)
    o = oracle.Sender702(KEY, IV32)
    # push the sender into stream B for some sizes: a message bigger than the ring holds
    for warm in (5000, 70000):
        w = splitmix64_bytes(warm, warm)
        s.send(empty(warm), dev(w), warm)
        o.send(w.tobytes())
    pt = splitmix64_bytes(n + 3, n)
    ct = empty(max(n, 1))
    hdr, _ = s.send(ct, dev(pt) if n else empty(1), n)
    ohdr, oct_ = o.send(pt.tobytes())
    assert hdr == ohdr and host(ct)[:n].tobytes() == oct_
    mask = empty(n + 1024)
    ml = ctrmode.recv702_premask(ctx, IV32, hdr, mask)
    assert ml == (0 if n >= 65536 or n == 0 else ((n + 511) // 512 * 512 if n > 1024 else n))
    for use_mask in (True, False):
        out = empty(max(n, 1), fill=0x55)
        ctrmode.recv702(ctx, IV32, hdr, out, ct, mask=mask if use_mask else None, mask_len=ml if use_mask else 0)
        got = host(out)[:n].tobytes()
        assert got == pt.tobytes(), (n, use_mask)
        assert got == oracle.recv702(KEY, IV32, hdr, oct_, premask=use_mask)


@pytest.mark.parametrize("n", [1, 17, 100, 1000])
def test_702_premask_writes_only_its_bytes(n, ctx):
    """A <= 1 KiB mask of a length that is not a multiple of 16 (recv.c:1187-1194): the keystream
    kernel stores the last block's bytes only — nothing past mask_len changes."""
    s = ctrmode.Sender702(ctx, IV32)
    pt = splitmix64_bytes(n + 11, n)
    ct = empty(n)
    hdr = s.send(ct, dev(pt), n)[0]
    mask = empty(n + 64, fill=0xA5)
    ml = ctrmode.recv702_premask(ctx, IV32, hdr, mask)
    assert ml == n
    m = host(mask)
    assert (m[n:] == 0xA5).all()
    out = empty(n)
    ctrmode.recv702(ctx, IV32, hdr, out, ct, mask=mask, mask_len=ml)
    assert host(out)[:n].tobytes() == pt.tobytes()


@pytest.mark.parametrize("n,mode", [(200000, b"4"), (3000, b"0"), (40000, b"1"), (3 << 20, b"1")])
def test_702_iv_count_carry_breaks_runs(n, mode, ctx):
    """Header counters near 2^32 and IVs ending in 0xff: IV_Count's 32-bit accumulator
    (send.c:1021) truncates the counter and drops a carry between the reference's slices / mask
    chunks, so they are NOT one CTR stream — the engine must split its launches exactly there."""
    iv = IV32[:15] + b"\xff" + IV32[16:31] + b"\xff"
    hdr = bytearray(26)
    hdr[0:4] = n.to_bytes(4, "big")
    hdr[4:5] = mode if n < 65536 else b"\0"
    hdr[5:9] = (0xFFFFFFFF - 300).to_bytes(4, "big")
    hdr[20:21] = b"4" if n <= 1048575 else b"1"
    chop = ((n - 1) // 12 + 1 + 15) // 16 * 16 if n <= 1048575 else ((524288 - 1) // 12 + 1 + 15) // 16 * 16
    hdr[21:25] = chop.to_bytes(4, "big")
    hdr = bytes(hdr)
    ct = splitmix64_bytes(n ^ 0x55, n)
    mask = empty(n + 1024)
    ml = ctrmode.recv702_premask(ctx, iv, hdr, mask)
    for use_mask in (True, False):
        out = empty(n)
        ctrmode.recv702(ctx, iv, hdr, out, dev(ct), mask=mask if use_mask else None, mask_len=ml if use_mask else 0)
        assert host(out)[:n].tobytes() == oracle.recv702(KEY, iv, hdr, ct.tobytes(), premask=use_mask), use_mask


def test_700_sequence_vs_oracle(ctx):
    iv = IV32[:16]
    c = oc = 5
    for n in [1, 15, 16, 17, 4096, 65536, 100000, 1 << 20, (1 << 21) + 3]:
        pt = splitmix64_bytes(n, n)
        out = empty(n)
        hdr, c = ctrmode.send700(ctx, iv, c, out, dev(pt), n)
        ohdr, oct_, oc = oracle.send700(KEY, iv, oc, pt.tobytes())
        assert hdr == ohdr and host(out)[:n].tobytes() == oct_ and c == oc
        back = empty(n)
        ctrmode.recv700(ctx, iv, hdr, back, out)
        assert host(back)[:n].tobytes() == pt.tobytes()
    torch.cuda.synchronize()


def test_recv_refuses_untrusted_header_sizes(ctx):
    """The header is wire input: a length beyond the caller's buffer, or a choping_sz
    that is not a multiple of 16 in [16, n rounded up to 16], is refused before any launch or
    slice list is built (the reference trusts both, recv.c:1226-1240)."""
    from cryptmpi_2022_amd import _native as N

    n = 200000
    ct = empty(n)
    out = empty(n - 1)  # one byte short
    hdr = bytearray(26)
    hdr[0:4] = n.to_bytes(4, "big")
    hdr[20:21] = b"4"
    hdr[21:25] = (16704).to_bytes(4, "big")
    with pytest.raises(N.CmpiError):
        ctrmode.recv702(ctx, IV32, bytes(hdr), out, ct)
    with pytest.raises(N.CmpiError):
        ctrmode.recv700(ctx, IV32[:16], bytes(hdr), out, ct)
    out = empty(n)
    for chop in (1, 15, 17, ((n + 15) // 16 + 1) * 16):
        hdr[21:25] = chop.to_bytes(4, "big")
        with pytest.raises(N.CmpiError):
            ctrmode.recv702(ctx, IV32, bytes(hdr), out, ct)
    hdr[21:25] = (16704).to_bytes(4, "big")
    ctrmode.recv702(ctx, IV32, bytes(hdr), out, ct)  # a well-formed header still opens
    assert host(out)[:n].tobytes() == oracle.recv702(KEY, IV32, bytes(hdr), host(ct)[:n].tobytes(), premask=False)


def test_served_ops_follow_the_stream(ctx):
    """A served op runs outside stream order, so it must first wait for the work already queued
    on the caller's stream: the input is written by a copy queued behind a long sleep kernel, the
    send / receive right after must see the final bytes (both forms)."""
    n = 4096
    s = ctrmode.Sender702(ctx, IV32)
    pt = splitmix64_bytes(0x5E, n)
    src = dev(pt)
    inp = empty(n, fill=0)
    torch.cuda._sleep(20_000_000)  # ~10 ms of GPU time ahead of the copy
    inp.copy_(src)
    ct = empty(n)
    hdr, _ = s.send(ct, inp, n)
    out = empty(n, fill=0)
    torch.cuda._sleep(20_000_000)
    ct2 = ct.clone()
    ctrmode.recv702(ctx, IV32, hdr, out, ct2)
    assert host(out).tobytes() == pt.tobytes()
    s.close()


@pytest.mark.parametrize("n", [1, 15, 16, 1000, 4096, 65536 - 15])
@pytest.mark.parametrize("skip", [0, 1, 9, 15])
@pytest.mark.parametrize("pinned", [False, True])
def test_ctr_xor_host_skip(ctx, n, skip, pinned):
    """cmpi_ctr_xor_host (the EVP shim's EVP_EncryptUpdate on a CTR context): the message starts
    `skip` bytes into the counter block's keystream; host buffers pageable or page-locked — served
    by the resident kernel when the context runs one (byte-granular form for skip > 0)."""
    import ctypes

    from cryptmpi_2022_amd import _native as N

    cb = bytes(range(200, 216))
    pt = splitmix64_bytes(n * 31 + skip, n)
    if pinned:
        src_t = torch.from_numpy(pt.copy()).pin_memory()
        dst_t = torch.full((n,), 0xEE, dtype=torch.uint8).pin_memory()
        src, dst = src_t.numpy(), dst_t.numpy()
    else:
        src, dst = pt.copy(), np.full(n, 0xEE, np.uint8)
    cbb = (ctypes.c_uint8 * 16).from_buffer_copy(cb)
    N.check(N.lib().cmpi_ctr_xor_host(ctx.handle, ctypes.c_void_p(dst.ctypes.data), ctypes.c_void_p(src.ctypes.data),
                                      n, cbb, skip))
    ks = oracle.ctr_xor(KEY, cb, bytes(skip + n))[skip:]
    assert dst.tobytes() == bytes(a ^ b for a, b in zip(pt.tobytes(), ks))


@pytest.mark.parametrize("served", [False, True])
@pytest.mark.parametrize("nblocks", [1, 7, 4096])
def test_ecb_host_served(served, nblocks):
    """cmpi_ecb_encrypt_host (the shim's EVP_EncryptUpdate on an ECB context: the 602 sub-key
    K' = AES_K(V), send.c:583) launched and served by the ECB context's resident kernel."""
    import ctypes

    from cryptmpi_2022_amd import _native as N

    c = aead.CipherCtx(KEY, "aes-128-ecb")
    if served:
        c.service_start()
    pt = splitmix64_bytes(0xEC + nblocks, 16 * nblocks)
    out = np.zeros(16 * nblocks, np.uint8)
    N.check(N.lib().cmpi_ecb_encrypt_host(c.handle, ctypes.c_void_p(out.ctypes.data),
                                          ctypes.c_void_p(pt.ctypes.data), nblocks))
    assert out.tobytes() == oracle.ecb_encrypt(KEY, pt.tobytes())
    if served:
        c.service_stop()
