"""Oracle self-checks of the counter-mode message paths (CPU): the 700 and 702 restatements
(oracle/ctrmode_ref.c) must round-trip like the reference's sender/receiver pairs, keep the
header layout of send.c:1537-1672 / :917-944, and their streams must equal plain CTR under
IV_Count (SP 800-38A keystream pinned by tests/golden)."""
import random

import pytest

import oracle
from cryptmpi_2022_amd.synth import splitmix64_bytes

KEY = bytes(range(16))
IV32 = splitmix64_bytes(0x702, 32).tobytes()
SIZES = [0, 1, 15, 16, 17, 1000, 1024, 1025, 4095, 4096, 65535, 65536, 65537, 300000, 1048575, 1048576, 1 << 21,
         3 * (1 << 20) + 5]


def _be32(b):
    return int.from_bytes(b, "big")


@pytest.mark.parametrize("series", [16, 3])
def test_702_round_trip_and_header(series):
    s = oracle.Sender702(KEY, IV32, series=series)
    rng = random.Random(series)
    for n in SIZES + [rng.randrange(1, 70000) for _ in range(20)]:
        pt = splitmix64_bytes(n + 7, n).tobytes()
        before = s.state()
        hdr, ct = s.send(pt)
        assert len(hdr) == 26 and _be32(hdr[0:4]) == n
        if n < 65536:
            assert hdr[20:21] == b"1" and _be32(hdr[21:25]) == 524288
            if hdr[4:5] == b"0":
                assert _be32(hdr[5:9]) == before["counter_needto_send"] & 0xFFFFFFFF
            else:
                assert hdr[4:5] == b"1" and _be32(hdr[5:9]) == before["counter_needto_send_large_msg"] & 0xFFFFFFFF
        else:
            assert _be32(hdr[5:9]) == before["counter_needto_send_large_msg"] & 0xFFFFFFFF
            assert hdr[20:21] == (b"4" if n <= 1048575 else b"1")
            assert _be32(hdr[21:25]) % 16 == 0
        for premask in (True, False):
            assert oracle.recv702(KEY, IV32, hdr, ct, premask=premask) == pt, (n, premask)
        if n:
            assert ct != pt or n < 4
        s.precompute(n, rng.randrange(0, 4))


def test_702_large_message_is_one_stream_b():
    """>= 64 KiB: the per-thread slices at IV_Count offsets (send.c:1768-1816) are one contiguous
    CTR stream of Send_common_IV[16..32) from the long-message counter."""
    s = oracle.Sender702(KEY, IV32)
    n = 1048576 + 12345
    pt = splitmix64_bytes(99, n).tobytes()
    hdr, ct = s.send(pt)
    assert ct == oracle.ctr_xor(KEY, oracle.iv_count(IV32[16:], 0), pt)
    assert s.state()["enc_common_counter_long_msg"] == (n + 15) // 16


def test_702_small_from_ring_is_stream_a():
    """< 64 KiB with the ring full enough: XOR with stream A's precomputed mask (init 4 KiB mask)."""
    s = oracle.Sender702(KEY, IV32)
    pt = splitmix64_bytes(5, 3000).tobytes()
    hdr, ct = s.send(pt)
    assert hdr[4:5] == b"0"
    assert ct == oracle.ctr_xor(KEY, IV32[:16], pt)
    st = s.state()
    assert st["counter_needto_send"] == 188 and st["start"] == 3008 and st["compute_size"] == 4096 - 3008


def test_700_round_trip_and_counter():
    c = 0
    iv = IV32[:16]
    for n in SIZES:
        pt = splitmix64_bytes(n, n).tobytes()
        hdr, ct, c2 = oracle.send700(KEY, iv, c, pt)
        assert _be32(hdr[0:4]) == n and _be32(hdr[5:9]) == c & 0xFFFFFFFF and _be32(hdr[21:25]) == 524288
        assert ct == oracle.ctr_xor(KEY, oracle.iv_count(iv, c), pt)
        assert oracle.recv700(KEY, iv, hdr, ct) == pt
        # send.c:1006: (unsigned long)(n - 1) / 16 + 1 — 2^60 for an empty message
        assert c2 == c + ((n - 1) // 16 + 1 if n else 1 << 60)
        c = c2 if n else c
