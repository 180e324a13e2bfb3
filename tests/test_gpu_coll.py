"""Naive secure collectives as batch calls (alltoall.c:764-836 and siblings): fresh nonces,
wire blocks bit-exact vs the oracle for the nonces they carry, round trip, forgery, and an
in-process two-rank Alltoall exchange."""
import numpy as np
import pytest

import oracle
from cryptmpi_2022_amd import aead, coll
from cryptmpi_2022_amd.synth import records

from tests.gpu_util import dev, empty, host, status_buf

pytestmark = pytest.mark.gpu
KEY = bytes(range(16))


@pytest.mark.parametrize("n,p", [(0, 3), (1, 8), (1000, 8), (4096, 5), (1 << 20, 8)])
def test_seal_blocks_wire_and_round_trip(n, p):
    ctx = aead.AeadCtx(KEY)
    pt = records(0xA2A + n, p, n)
    wire = empty(p * (n + 28), fill=0)
    coll.seal_blocks(ctx, wire, dev(pt) if n else empty(1), n, p)
    w = host(wire)[: p * (n + 28)].reshape(p, n + 28)
    nonces = np.ascontiguousarray(w[:, :12])
    assert len({bytes(x) for x in nonces}) == p  # fresh nonce per block
    assert np.array_equal(w[:, 12:], oracle.gcm_seal_batch(KEY, nonces, pt))
    out, st = empty(max(p * n, 1), fill=0xEE), status_buf(p)
    coll.open_blocks(ctx, out, wire, n, p, status=st)
    assert (host(st)[:p] == 1).all() and host(out)[: p * n].tobytes() == pt.tobytes()
    w2 = w.copy()
    w2[p // 2, -1] ^= 0x80
    out2, st2 = empty(max(p * n, 1), fill=0xEE), status_buf(p)
    coll.open_blocks(ctx, out2, dev(w2), n, p, status=st2)
    s = host(st2)[:p]
    assert s[p // 2] == 0 and s.sum() == p - 1
    assert (host(out2)[(p // 2) * n: (p // 2 + 1) * n] == 0).all()


def test_nonces_never_repeat_across_calls():
    ctx = aead.AeadCtx(KEY)
    seen = set()
    for _ in range(4):
        wire = empty(64 * 28)
        coll.seal_blocks(ctx, wire, empty(1), 0, 64)
        w = host(wire)[: 64 * 28].reshape(64, 28)
        seen |= {bytes(x[:12]) for x in w}
    assert len(seen) == 256


def test_two_rank_alltoall_in_process():
    """Rank r seals p blocks for its peers, block (r -> q) travels to rank q, q opens it."""
    p, n = 2, 4096
    ctxs = [aead.AeadCtx(KEY), aead.AeadCtx(KEY)]  # every rank holds the same symmetric key
    send = [records(0x2A2A + r, p, n) for r in range(p)]
    wires = []
    for r in range(p):
        w = empty(p * (n + 28))
        coll.seal_blocks(ctxs[r], w, dev(send[r]), n, p)
        wires.append(host(w)[: p * (n + 28)].reshape(p, n + 28))
    for q in range(p):
        recv_wire = np.stack([wires[r][q] for r in range(p)])  # MPIR_Alltoall_impl on ciphertext
        out, st = empty(p * n), status_buf(p)
        coll.open_blocks(ctxs[q], out, dev(recv_wire), n, p, status=st)
        assert (host(st)[:p] == 1).all()
        got = host(out)[: p * n].reshape(p, n)
        for r in range(p):
            assert got[r].tobytes() == send[r][q].tobytes()


@pytest.mark.parametrize("n", [4096, 1 << 20])
def test_bench_alltoall_e2e_one_rank(n):
    """bench.py's BASELINE config-5 timing path (seal -> exchange -> open) on one rank: runs,
    every block authenticates and the rank gets its own plaintext back."""
    import bench

    res = bench.alltoall_e2e(0, None, lambda: None, n=n, steps=2, warmup=1)
    assert res["ranks"] == 1 and res["all_blocks_authenticated"] and res["ms_per_call"] > 0
