"""CryptMPI's framed message paths from host memory: the 602 pipelined
sender / receiver (MV/src/mpi/pt2pt/send.c:729-850, recv.c:679-809) with one request per outer
512 KiB message, begun and completed in order; the 700 / 702 counter-mode messages straight from
MPI user buffers (send.c:886-1017, :1502-1987; recv.c:812-940, :1025-1403).  Bytes bit-exact vs the
oracle's restatement (oracle/framing_ref.c, oracle/ctrmode_ref.c), pageable and page-locked, in
both request forms: direct (the kernels access the page-locked spans over PCIe, the default up to
16 MiB per request) and DMA (spans copied through device staging)."""
import numpy as np
import pytest
import torch

import oracle
from cryptmpi_2022_amd import _native as N
from cryptmpi_2022_amd import aead, ctrmode, frame
from cryptmpi_2022_amd.synth import splitmix64_bytes

from tests.gpu_util import empty

pytestmark = pytest.mark.gpu

KEY = bytes(range(16))
SMALL_KEY = bytes(16)
IV32 = splitmix64_bytes(0x702, 32).tobytes()


@pytest.fixture(autouse=True, params=["direct", "dma"])
def span_mode(request):
    """Every test in both request forms (cmpi_debug_set_span_direct: 16 MiB default / 0)."""
    N.lib().cmpi_debug_set_span_direct(16 << 20 if request.param == "direct" else 0)
    yield request.param
    N.lib().cmpi_debug_set_span_direct(16 << 20)


def _buf(n: int, pinned: bool, fill: int = 0):
    """Host buffer of n bytes (numpy view): pageable, or page-locked torch memory."""
    if pinned:
        t = torch.full((max(n, 1),), fill, dtype=torch.uint8).pin_memory()
        return t.numpy()[:n], t
    return np.full(max(n, 1), fill, np.uint8)[:n], None


def _seg_ctx(plan, header):
    master = aead.AeadCtx(KEY)
    if plan.subkey:
        seg = aead.AeadCtx(bytes(16))
        seg.rekey_subkey(master, header[4:20], stream=torch.cuda.current_stream())  # K' on the device
        return seg, master
    return aead.AeadCtx(SMALL_KEY), master


@pytest.mark.parametrize("n,threads", [(8 << 20, 8), (1572881, 3), (300000, 8), (1000, 8), (0, 8)])
@pytest.mark.parametrize("pinned", [False, True])
def test_602_host_pipelined_send_and_receive(n, threads, pinned):
    """An 8 MiB 602 message (16 outer messages) sealed from host memory one outer message per
    request, each begun before the previous one is waited (send.c:754-835 overlaps the seal of
    outer k+1 with MPI_Isend of k), waited in order: wire bit-exact vs the oracle; then opened outer
    by outer as it 'lands', in order; a forged segment fails alone (status 0, zero-filled,
    CMPI_EAUTH)."""
    pt = splitmix64_bytes(0xF00D ^ n, n)
    rand16 = splitmix64_bytes(0x5EED ^ n, 16).tobytes()
    plan = frame.plan602(n, threads, 0)
    header = frame.header602(plan, rand16)
    seg, _master = _seg_ctx(plan, header)
    src, _k1 = _buf(n, pinned)
    src[:] = pt
    wire, _k2 = _buf(plan.wire_bytes, pinned, fill=0x5A)
    reqs = [frame.seal602_host_begin(seg, plan, header, wire, src, o) for o in range(plan.outer)]
    for o, r in enumerate(reqs):
        assert r.wait() == N.CMPI_OK, o  # the reference's MPI_Isend of outer o goes here
        wo, wl, _, _ = frame.outer_span(plan, o)
        assert wire[wo: wo + wl].any() or wl == 0
    want_h, want_w = oracle.seal602(KEY, SMALL_KEY, pt.tobytes(), rand16, threads, 0, wire_fill=0x5A)
    assert header == want_h and wire.tobytes() == want_w
    # the synchronous form: the same bytes
    wire2, _k3 = _buf(plan.wire_bytes, pinned, fill=0x5A)
    frame.seal602_host(seg, plan, header, wire2, src)
    assert wire2.tobytes() == want_w
    # receiver: outer messages opened as they arrive
    out, _k4 = _buf(n, pinned, fill=0xEE)
    st = np.full(plan.nseg, 7, np.int32)
    reqs = [frame.open602_host_begin(seg, header, out, wire, o, status=st) for o in range(plan.outer)]
    assert all(r.wait() == N.CMPI_OK for r in reqs)
    assert (st == 1).all() and out.tobytes() == pt.tobytes()
    if n:
        bad = np.frombuffer(want_w, np.uint8).copy()
        bad[-1] ^= 1  # the last segment's tag
        out2, _k5 = _buf(n, pinned, fill=0xEE)
        st2 = np.zeros(plan.nseg, np.int32)
        assert frame.open602_host(seg, header, out2, bad, st2) == N.CMPI_EAUTH
        assert st2[-1] == 0 and (st2[:-1] == 1).all()
        _, _, po, pl = frame.outer_span(plan, plan.outer - 1)
        start = po + plan.chop * ((pl - 1) // plan.chop) if plan.nseg > 1 else 0
        assert not out2[start:].any() and out2[:start].tobytes() == pt[:start].tobytes()


def _ctr_ctx(served: bool):
    """CTR context; served: its message service started (the 700 / 702 ops up to 64 KiB run on
    the resident kernel, synchronously inside *_begin)."""
    ctx = aead.CipherCtx(KEY, "aes-128-ctr")
    if served:
        ctx.service_start()
    return ctx


@pytest.mark.parametrize("served", [False, True])
@pytest.mark.parametrize("pinned", [False, True])
def test_700_host_sequence(pinned, served):
    ctx = _ctr_ctx(served)
    iv = IV32[:16]
    c = oc = 9
    for n in [0, 1, 17, 4096, 65536, 100001, (1 << 21) + 3]:
        pt = splitmix64_bytes(n + 700, n)
        src, _k1 = _buf(n, pinned)
        src[:] = pt
        out, _k2 = _buf(n, pinned, fill=0xAB)
        hdr, c = ctrmode.send700_host(ctx, iv, c, out, src, n)
        ohdr, oct_, oc = oracle.send700(KEY, iv, oc, pt.tobytes())
        assert hdr == ohdr and out.tobytes() == oct_ and c == oc, n
        back, _k3 = _buf(n, pinned, fill=0x11)
        ctrmode.recv700_host(ctx, iv, hdr, back, out)
        assert back.tobytes() == pt.tobytes(), n


@pytest.mark.parametrize("served", [False, True])
@pytest.mark.parametrize("pinned", [False, True])
def test_702_host_sequence_vs_oracle(pinned, served):
    """702 sender from host buffers over the branch mix (ring hit '0', stream B '1', mode '4',
    pipelined '1'), interleaved with the precompute a sender runs while its Isends are pending;
    every header, ciphertext and sender state equal to the oracle's; the receiver's host form
    with the device mask made while the payload is in flight, and without a mask."""
    ctx = _ctr_ctx(served)
    s = ctrmode.Sender702(ctx, IV32, ring_bytes=65536, series_threads=8)
    o = oracle.Sender702(KEY, IV32, max_bytes=65536, series=8)
    for i, n in enumerate([0, 16, 1000, 4096, 30000, 65535, 65536, 200000, 1048576, (1 << 21) + 9, 3000, 70000]):
        pt = splitmix64_bytes(n * 3 + i, n)
        src, _k1 = _buf(n, pinned)
        src[:] = pt
        out, _k2 = _buf(n, pinned, fill=0xCD)
        hdr, nseg = ctrmode.send702_host(s, out, src, n, pending_isends=i % 3)
        ohdr, oct_ = o.send(pt.tobytes(), pending=i % 3)
        assert hdr == ohdr and out.tobytes() == oct_ and nseg >= 1, n
        assert s.state() == o.state(), n
        assert s.precompute(n, 2) == o.precompute(n, 2)
        mask = empty(n + 1024)
        ml = ctrmode.recv702_premask(ctx, IV32, hdr, mask)
        for use_mask in (True, False):
            back, _k3 = _buf(n, pinned, fill=0x33)
            ctrmode.recv702_host(ctx, IV32, hdr, back, out, mask=mask if use_mask else None, mask_len=ml if use_mask else 0)
            assert back.tobytes() == pt.tobytes(), (n, use_mask)
    s.close()


def test_host_recv_refuses_short_buffer():
    ctx = aead.CipherCtx(KEY, "aes-128-ctr")
    hdr = bytearray(26)
    hdr[0:4] = (5000).to_bytes(4, "big")
    with pytest.raises(N.CmpiError):
        ctrmode.recv700_host(ctx, IV32[:16], bytes(hdr), np.zeros(4999, np.uint8), np.zeros(5000, np.uint8))
    with pytest.raises(N.CmpiError):
        ctrmode.recv702_host(ctx, IV32, bytes(hdr), np.zeros(4999, np.uint8), np.zeros(5000, np.uint8))
