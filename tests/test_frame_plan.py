"""Host logic of the 602 framing (no GPU): the engine's plan equals the oracle's restatement of
send.c:392-549 for every (size, thread cap, pending Isends) corner, headers carry the reference
byte layout, and a receiver re-derives the sender's segmentation from the header alone."""
import itertools

import pytest

import oracle
from cryptmpi_2022_amd import frame

SIZES = [0, 1, 15, 16, 17, 100, 65535, 65536, 65537, 100000, 131071, 131072, 524287, 524288, 524289,
         1048575, 1048576, 1048577, 1572881, 33554432, 33554433, 67108864, (1 << 31) - 1]


@pytest.mark.parametrize("threads", [1, 2, 3, 4, 6, 8, 16])
def test_plan_matches_oracle(threads):
    for n, pend in itertools.product(SIZES, [0, 1, 63, 64, 70]):
        assert frame.plan602(n, threads, pend).as_dict() == oracle.plan602(n, threads, pend), (n, threads, pend)


def test_header_layout():
    p = frame.plan602(200000, 8, 0)
    r = bytes(range(100, 116))
    h = frame.header602(p, r)
    assert h[:4] == (200000).to_bytes(4, "big")      # send.c:371-374
    assert h[4:20] == r                               # V (n > 65535)
    assert h[20:21] == b"4"
    assert h[21:25] == p.chop.to_bytes(4, "big")     # send.c:545-549
    want, _ = oracle.seal602(bytes(16), bytes(16), bytes(200000), r)
    assert h == want


@pytest.mark.parametrize("n", [0, 100, 65535, 65536, 524288, 1048575, 1048576, 1572881, 33554433])
@pytest.mark.parametrize("threads", [3, 8])
def test_receiver_rederives_segmentation(n, threads):
    p = frame.plan602(n, threads, 0)
    q = frame.plan602_from_header(frame.header602(p, bytes(16)))
    for k in ("total", "outer", "nseg", "wire_bytes", "mode", "subkey"):
        assert q.as_dict()[k] == p.as_dict()[k], k


def test_outer_spans_tile_the_message():
    p = frame.plan602(1572881, 8, 0)  # mode '1': 3 x 512 KiB + 17 bytes
    assert chr(p.mode) == "1" and p.outer == 4
    w = pt = 0
    for o in range(p.outer):
        wo, wl, po, pl = frame.outer_span(p, o)
        assert (wo, po) == (w, pt)
        w, pt = wo + wl, po + pl
    assert (w, pt) == (p.wire_bytes, p.total)


def test_header600_layout():
    h = frame.header600(1000, b"2")
    assert h[:4] == (1000).to_bytes(4, "big") and h[20:21] == b"2" and h[21:25] == (1000).to_bytes(4, "big")
