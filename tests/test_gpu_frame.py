"""602 / 600 framings on the device vs the oracle's statement-by-statement restatement of the
reference senders (oracle/framing_ref.c: send.c:221-337, :339-884): header, segment prefixes,
nonces, sub-key and ciphertext/tags are bit-exact; receivers (recv.c:219-809) round-trip and
reject forgeries segment by segment."""
import numpy as np
import pytest

import oracle
from cryptmpi_2022_amd import aead, frame
from cryptmpi_2022_amd.synth import splitmix64_bytes

from tests.gpu_util import dev, empty, host, status_buf

pytestmark = pytest.mark.gpu

KEY = bytes(range(16))
SMALL_KEY = bytes(16)  # symmetric_key[32..47] of the reference (zeros in its init)

CASES = [(0, 8, 0), (100, 8, 0), (65535, 8, 0), (65536, 8, 0), (100000, 8, 0), (131072, 3, 0), (524288, 6, 0),
         (1048575, 8, 0), (1048576, 8, 0), (1572881, 8, 0), (1572881, 3, 0), (1572881, 8, 70), (2 << 20, 1, 0)]


def seal_on_gpu(n, threads, pending, fill=0x5A):
    pt = splitmix64_bytes(0xC0FFEE ^ n, n)
    rand16 = splitmix64_bytes(0x5EED + n, 16).tobytes()
    plan = frame.plan602(n, threads, pending)
    header = frame.header602(plan, rand16)
    master = aead.AeadCtx(KEY)
    if plan.subkey:
        seg = aead.AeadCtx(bytes(16))
        seg.rekey_subkey(master, header[4:20])  # K' = AES_K(V) on the device
    else:
        seg = aead.AeadCtx(SMALL_KEY)
    wire = empty(plan.wire_bytes, fill=fill)
    frame.seal602(seg, plan, header, wire, dev(pt) if n else empty(1))
    return pt, rand16, plan, header, wire, seg


@pytest.mark.parametrize("n,threads,pending", CASES)
def test_602_seal_bit_exact(n, threads, pending):
    pt, rand16, plan, header, wire, _ = seal_on_gpu(n, threads, pending)
    want_h, want_w = oracle.seal602(KEY, SMALL_KEY, pt.tobytes(), rand16, threads, pending, wire_fill=0x5A)
    assert header == want_h
    got = host(wire)[: plan.wire_bytes].tobytes()
    assert got == want_w


@pytest.mark.parametrize("n,threads,pending", CASES)
def test_602_open_round_trip_and_forgery(n, threads, pending):
    pt, _, plan, header, wire, seg = seal_on_gpu(n, threads, pending)
    out, st = empty(max(n, 1), fill=0xEE), status_buf(plan.nseg)
    frame.open602(seg, header, out, wire, st)
    assert (host(st)[: plan.nseg] == 1).all()
    assert host(out)[:n].tobytes() == pt.tobytes()
    # flip a tag byte of the last segment: only that segment fails, and it is zero-filled
    w = host(wire)[: plan.wire_bytes].copy()
    w[-1] ^= 0x01
    out2, st2 = empty(max(n, 1), fill=0xEE), status_buf(plan.nseg)
    frame.open602(seg, header, out2, dev(w), st2)
    s = host(st2)[: plan.nseg]
    assert s[-1] == 0 and (s[:-1] == 1).all()
    _, _, po, pl = frame.outer_span(plan, plan.outer - 1)
    start = po + plan.chop * ((pl - 1) // plan.chop) if n > 0 and plan.nseg > 1 else 0
    got = host(out2)[:n]
    assert (got[start:] == 0).all() and got[:start].tobytes() == pt[:start].tobytes()


def test_602_pipelined_outer_messages():
    """Mode '1': sealing outer message by outer message (what a pipelined sender overlaps with
    MPI_Isend, send.c:833-835) yields the same wire as sealing the whole message."""
    n = 1572881
    pt, rand16, plan, header, wire_all, seg = seal_on_gpu(n, 8, 0)
    wire = empty(plan.wire_bytes, fill=0x5A)
    d_pt = dev(pt)
    for o in range(plan.outer):
        frame.seal602(seg, plan, header, wire, d_pt, first=o, count=1)
    assert host(wire).tobytes() == host(wire_all).tobytes()


@pytest.mark.parametrize("n", [0, 1, 1000, 4096, 65535, 1 << 20])
def test_600_frame(n):
    pt = splitmix64_bytes(0x600 + n, n)
    nonce = splitmix64_bytes(0x601 + n, 12).tobytes()
    ctx = aead.AeadCtx(KEY)
    payload = empty(n + 28, fill=0)
    frame.seal600(ctx, nonce, payload, dev(pt) if n else empty(1), n)
    got = host(payload)[: n + 28].tobytes()
    assert got == nonce + oracle.gcm_seal(KEY, nonce, pt.tobytes())  # send.c:294-311
    out, st = empty(max(n, 1)), status_buf(1)
    frame.open600(ctx, out, payload, n, st)
    assert host(st)[0] == 1 and host(out)[:n].tobytes() == pt.tobytes()
