"""AES-128-GCM on the MI355X through the C ABI vs the oracle / golden vectors (bit-exact).

Covers every work decomposition the engine can pick (lanes per record L = 1/2/4, one or many
segments per record), the CryptMPI record layouts (dense, naive-collective wire
nonce||ct||tag with stride n+28, in place), the edge sizes (0, partial blocks, 64 KiB-1,
1 MiB), open's forgery path (status 0 + zero-filled plaintext, aead.h:276-278) and the
full BASELINE config-2 batch through size-independent properties."""
import hashlib

import numpy as np
import pytest

import oracle
from cryptmpi_2022_amd import aead
from cryptmpi_2022_amd.synth import random_nonces, records, splitmix64_bytes
from tests.gpu_util import dev, empty, host, status_buf

pytestmark = pytest.mark.gpu

KEY = bytes.fromhex("000102030405060708090a0b0c0d0e0f")
DIRECT_DEFAULT = (2 << 20) + 64  # cmpi_aead.hip g_host_direct


@pytest.fixture(autouse=True)
def _auto_plan():
    aead.force_plan(0, 0)
    aead.force_wide(0, 0)
    yield
    aead.force_plan(0, 0)
    aead.force_wide(0, 0)
    aead.set_flow_threads(0)
    aead.set_flow_one_wg(True)
    aead.N.lib().cmpi_debug_set_host_direct(DIRECT_DEFAULT)
    aead.N.lib().cmpi_debug_set_lane_pair(2)  # the default


def gpu_seal(ctx, nonces: np.ndarray, pt: np.ndarray) -> np.ndarray:
    nrec, n = pt.shape
    out = empty(nrec * (n + 16), fill=0xAA)
    ctx.seal_batch(out, dev(pt), dev(nonces), n, nrec)
    return host(out)[: nrec * (n + 16)].reshape(nrec, n + 16)


def gpu_open(ctx, nonces: np.ndarray, ct: np.ndarray):
    nrec, m = ct.shape
    n = m - 16
    out = empty(nrec * n, fill=0xAA)
    st = status_buf(nrec)
    ctx.open_batch(out, dev(ct), dev(nonces), n, nrec, status=st)
    return host(out)[: nrec * n].reshape(nrec, n), host(st)[:nrec]


def test_published_kat(golden):
    kat, _ = golden
    for v in kat["gcm"]:
        if v["aad"]:
            continue  # CryptMPI never passes AAD; the engine's GCM has none
        ctx = aead.AeadCtx(bytes.fromhex(v["key"]))
        pt = np.frombuffer(bytes.fromhex(v["pt"]), np.uint8)[None, :].copy()
        nonce = np.frombuffer(bytes.fromhex(v["nonce"]), np.uint8)[None, :].copy()
        out = gpu_seal(ctx, nonce, pt)
        assert out[0].tobytes().hex() == v["ct"] + v["tag"], v["src"]
        back, st = gpu_open(ctx, nonce, out)
        assert st[0] == 1 and back[0].tobytes() == pt[0].tobytes()


def test_openssl_vectors(golden):
    _, ossl = golden
    ctx = aead.AeadCtx(bytes.fromhex(ossl["key"]))
    for e in ossl["gcm"]:
        pt = splitmix64_bytes(e["pt_seed"], e["len"])[None, :]
        nonce = np.frombuffer(bytes.fromhex(e["nonce"]), np.uint8)[None, :].copy()
        out = gpu_seal(ctx, nonce, pt)[0].tobytes()
        if "out" in e:
            assert out.hex() == e["out"], (e["len"], e["nonce_kind"])
        else:
            assert hashlib.sha256(out).hexdigest() == e["out_sha256"], (e["len"], e["nonce_kind"])
        back, st = gpu_open(ctx, nonce, np.frombuffer(out, np.uint8)[None, :].copy())
        assert st[0] == 1 and back[0].tobytes() == pt[0].tobytes()


@pytest.mark.parametrize("pair", [0, 3, 4])
@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 31, 48, 100, 1024, 1040, 4096, 4097, 65535])
@pytest.mark.parametrize("plan", [(0, 0), (1, 1), (2, 1), (4, 1), (4, 3), (1, 2), (2, 7)])
def test_batch_parity_plans(n, plan, pair):
    """Every lane plan, with the lane kernel's record stores one per step or grouped by output
    line in both forms, forced on these small batches (cmpi_debug_set_lane_pair 3 / 4)."""
    aead.force_plan(*plan)
    aead.N.lib().cmpi_debug_set_lane_pair(pair)
    nrec = 24 if n <= 4096 else 4
    pt = records(0x1000 + n, nrec, n)
    nonces = random_nonces(0x2000 + n, nrec)
    ctx = aead.AeadCtx(KEY)
    want = oracle.gcm_seal_batch(KEY, nonces, pt)
    got = gpu_seal(ctx, nonces, pt)
    assert np.array_equal(got, want), f"n={n} plan={plan} plan_used={aead.gcm_plan(ctx, n, nrec)}"
    back, st = gpu_open(ctx, nonces, want)
    assert (st == 1).all() and np.array_equal(back, pt)


def test_auto_plans_cover_all_lane_widths():
    ctx = aead.AeadCtx(KEY)
    seen = {aead.gcm_plan(ctx, n, N)[0] for n, N in [(16, 1 << 20), (1024, 200000), (1024, 65536), (64, 1 << 14)]}
    assert seen == {1, 2, 4}


@pytest.mark.parametrize("n,nrec", [(n, r) for n in (1, 15, 16, 17, 100) for r in (1, 3, 8)] +
                         [(n, r) for n in (260, 512, 600, 1000, 1008) for r in (1, 3, 9, 100)])
def test_short_records_flow_plan(n, nrec):
    """Short records (< 64 data blocks), few of them: the automatic plan is the flow kernel (one
    partial step + lane tree per record; one workgroup's batch finishes its tags in the same
    launch, larger ones by the XOR combine): bit-exact against the oracle, round trip, a forged
    record zero-filled."""
    ctx = aead.AeadCtx(KEY)
    assert aead.gcm_plan(ctx, n, nrec)[0] == 64, aead.gcm_plan(ctx, n, nrec)
    pt = records(0x5100 + n + nrec, nrec, n)
    nonces = random_nonces(0x5200 + n + nrec, nrec)
    want = oracle.gcm_seal_batch(KEY, nonces, pt)
    assert np.array_equal(gpu_seal(ctx, nonces, pt), want)
    forged = want.copy()
    forged[nrec - 1, n + 3] ^= 0x10
    back, st = gpu_open(ctx, nonces, forged)
    assert list(st) == [1] * (nrec - 1) + [0]
    assert np.array_equal(back[: nrec - 1], pt[: nrec - 1]) and not back[nrec - 1].any()


def test_wire_layout_naive_alltoall():
    """alltoall.c:795-834: record i = nonce(12) || ct(n) || tag(16) at i*(n+28)."""
    n, nrec = 1000, 8
    stride = n + 28
    pt = records(77, nrec, n)
    nonces = random_nonces(78, nrec)
    wire = np.zeros((nrec, stride), np.uint8)
    wire[:, :12] = nonces
    wbuf = dev(wire)
    ctx = aead.AeadCtx(KEY)
    ctx.seal_batch(wbuf[12:], dev(pt), wbuf, n, nrec, out_stride=stride, nonce_stride=stride)
    got = host(wbuf).reshape(nrec, stride)
    want = oracle.gcm_seal_batch(KEY, nonces, pt)
    assert np.array_equal(got[:, :12], nonces)
    assert np.array_equal(got[:, 12:], want)
    # receive side: open straight from the wire
    out = empty(nrec * n)
    st = status_buf(nrec)
    ctx.open_batch(out, wbuf[12:], wbuf, n, nrec, status=st, in_stride=stride, nonce_stride=stride)
    assert (host(st)[:nrec] == 1).all()
    assert np.array_equal(host(out).reshape(nrec, n), pt)


@pytest.mark.parametrize("n,nrec", [(4096, 16), (4096, 1), (1000, 3), (1 << 20, 2)])
def test_in_place(n, nrec):
    """Seal and open with out == in (BoringSSL aead.h:84: seal and open may work in place): lane plan
    (16 x 4 KiB), one-workgroup flow launches (1 x 4 KiB, 3 x 1000 B) and the multi-workgroup flow
    plan (2 x 1 MiB); a forged record opened in place comes back zero-filled."""
    pt = records(5, nrec, n)
    nonces = random_nonces(6, nrec)
    buf = np.zeros((nrec, n + 16), np.uint8)
    buf[:, :n] = pt
    d = dev(buf)
    ctx = aead.AeadCtx(KEY)
    ctx.seal_batch(d, d, dev(nonces), n, nrec, in_stride=n + 16, out_stride=n + 16)
    assert np.array_equal(host(d).reshape(nrec, n + 16), oracle.gcm_seal_batch(KEY, nonces, pt))
    st = status_buf(nrec)
    ctx.open_batch(d, d, dev(nonces), n, nrec, status=st, in_stride=n + 16, out_stride=n + 16)
    assert np.array_equal(host(d).reshape(nrec, n + 16)[:, :n], pt) and (host(st)[:nrec] == 1).all()
    forged = oracle.gcm_seal_batch(KEY, nonces, pt)
    forged[nrec - 1, n // 2] ^= 0x10
    d = dev(forged)
    ctx.open_batch(d, d, dev(nonces), n, nrec, status=st, in_stride=n + 16, out_stride=n + 16)
    back = host(d).reshape(nrec, n + 16)[:, :n]
    assert list(host(st)[:nrec]) == [1] * (nrec - 1) + [0]
    assert np.array_equal(back[: nrec - 1], pt[: nrec - 1]) and not back[nrec - 1].any()


@pytest.mark.parametrize("plan", [(0, 0), (4, 5), (1, 1)])
def test_open_forgery(plan):
    aead.force_plan(*plan)
    n, nrec = 1024, 32
    pt = records(9, nrec, n)
    nonces = random_nonces(10, nrec)
    ctx = aead.AeadCtx(KEY)
    ct = oracle.gcm_seal_batch(KEY, nonces, pt)
    bad = [0, 5, 17, 31]
    ct[0, 3] ^= 1        # ciphertext bit
    ct[5, n + 15] ^= 0x80  # tag bit
    ct[17, n - 1] ^= 4
    nonces_t = nonces.copy()
    nonces_t[31, 0] ^= 1  # wrong nonce
    back, st = gpu_open(ctx, nonces_t, ct)
    for i in range(nrec):
        if i in bad:
            assert st[i] == 0 and not back[i].any(), i
        else:
            assert st[i] == 1 and np.array_equal(back[i], pt[i]), i


def test_large_records_multisegment():
    """BASELINE config 5 shape: 8 records of 1 MiB per rank (many segments per record)."""
    n, nrec = 1 << 20, 8
    pt = records(0xB16, nrec, n)
    nonces = random_nonces(0xB17, nrec)
    ctx = aead.AeadCtx(KEY)
    L, nseg, G, r0 = aead.gcm_plan(ctx, n, nrec)
    assert nseg > 1
    want = oracle.gcm_seal_batch(KEY, nonces, pt)
    got = gpu_seal(ctx, nonces, pt)
    assert np.array_equal(got, want)
    want[3, 100] ^= 1
    back, st = gpu_open(ctx, nonces, want)
    assert list(st) == [1, 1, 1, 0, 1, 1, 1, 1]
    assert not back[3].any() and np.array_equal(back[[0, 1, 2, 4, 5, 6, 7]], pt[[0, 1, 2, 4, 5, 6, 7]])


@pytest.mark.parametrize("n,nrec,steps", [(1024, 3, 1), (1040, 2, 1), (4097, 3, 2), (65535, 2, 4), (100000, 3, 3),
                                          (1 << 20, 2, 0), (64 * 16 * 5 - 16, 2, 5)])
@pytest.mark.parametrize("one_wg", [True, False])
def test_wide_decomposition(n, nrec, steps, one_wg):
    """Wide plan (gcm_flow_kernel: one wave per 64*steps-block chunk; chunk 0 takes the remainder,
    G <= r0 < 2G or the whole record; radix-4 lane tree; chunk weights applied in the kernel by a
    wave-cooperative multiply, partials XOR-combined in the same launch or by the combine
    launch): bit-exact seal, round trip, forged record zero-filled, unaligned wire layout."""
    aead.force_wide(1, steps)
    aead.set_flow_one_wg(one_wg)
    ctx = aead.AeadCtx(KEY)
    L, nch, G, r0 = aead.gcm_plan(ctx, n, nrec)
    nx = n // 16 + (n % 16 > 0) + 1
    assert L == 64 and G % 64 == 0 and nch == max(1, nx // G) and r0 == nx - (nch - 1) * G
    assert r0 < 2 * G or nch == 1
    pt = records(0x3100 + n, nrec, n)
    nonces = random_nonces(0x3200 + n, nrec)
    want = oracle.gcm_seal_batch(KEY, nonces, pt)
    assert np.array_equal(gpu_seal(ctx, nonces, pt), want), (L, nch, G, r0)
    forged = want.copy()
    forged[nrec - 1, n // 2] ^= 0x10
    back, st = gpu_open(ctx, nonces, forged)
    assert list(st) == [1] * (nrec - 1) + [0]
    assert np.array_equal(back[: nrec - 1], pt[: nrec - 1]) and not back[nrec - 1].any()
    # naive-collective wire layout (odd stride), in place of the dense one
    stride = n + 28
    wire = np.zeros((nrec, stride), np.uint8)
    wire[:, :12] = nonces
    wbuf = dev(wire)
    ctx.seal_batch(wbuf[12:], dev(pt), wbuf, n, nrec, out_stride=stride, nonce_stride=stride)
    assert np.array_equal(host(wbuf).reshape(nrec, stride)[:, 12:], want)


@pytest.mark.parametrize("threads", [1024, 512])
@pytest.mark.parametrize("n,nrec,steps", [(64 * 16 * 3 - 16, 11, 1), (4097, 5, 2), (1 << 20, 2, 0),
                                          ((1 << 20) - 5, 3, 1), (64 * 16 * 40 + 7, 37, 1)])
def test_flow_kernel_forms(threads, n, nrec, steps):
    """gcm_flow_kernel at 512 and 1024 threads per workgroup; 3-chunk records put up to six
    records in one workgroup, ragged lengths have a partial last block.  Two seals back to back,
    a forged record, and a context re-keyed on the device (tables rebuilt by gcm_tables_kernel,
    bit-identical to the host build)."""
    aead.force_wide(1, steps)
    aead.set_flow_threads(threads)
    key2 = bytes(range(100, 116))
    ctx = aead.AeadCtx(KEY)
    pt = records(0x5100 + n, nrec, n)
    nonces = random_nonces(0x5200 + n, nrec)
    want = oracle.gcm_seal_batch(KEY, nonces, pt)
    for _ in range(2):
        assert np.array_equal(gpu_seal(ctx, nonces, pt), want), aead.gcm_plan(ctx, n, nrec)
    forged = want.copy()
    forged[1, n // 3] ^= 0x40
    back, st = gpu_open(ctx, nonces, forged)
    assert list(st) == [1] + [0] + [1] * (nrec - 2)
    assert not back[1].any() and np.array_equal(back[0], pt[0]) and np.array_equal(back[2:], pt[2:])
    ctx.rekey(key2)
    assert np.array_equal(gpu_seal(ctx, nonces, pt), oracle.gcm_seal_batch(key2, nonces, pt))
    back, st = gpu_open(ctx, nonces, oracle.gcm_seal_batch(key2, nonces, pt))
    assert list(st) == [1] * nrec and np.array_equal(back, pt)


def test_flow_open_without_status():
    """Config 5's shape (8 x 1 MiB, the default plan: 256 workgroups + the XOR combine) opened
    with status == NULL and one forged record: the record is zero-filled, the others are intact,
    and seals right after on the same stream are bit-exact."""
    n, nrec = 1 << 20, 8
    ctx = aead.AeadCtx(KEY)
    pt = records(0x7E00, nrec, n)
    nonces = random_nonces(0x7E01, nrec)
    want = oracle.gcm_seal_batch(KEY, nonces, pt)
    forged = want.copy()
    forged[5, 12345] ^= 0x04
    out = empty(nrec * n, fill=0xAA)
    ctx.open_batch(out, dev(forged), dev(nonces), n, nrec)
    b = host(out)[: nrec * n].reshape(nrec, n)
    assert not b[5].any() and np.array_equal(b[[0, 1, 2, 3, 4, 6, 7]], pt[[0, 1, 2, 3, 4, 6, 7]])
    for _ in range(3):
        assert np.array_equal(gpu_seal(ctx, nonces, pt), want)


def test_flow_two_streams_one_fresh_context():
    """calls on one context from two streams at once — the first use of a chunk-weight
    table by either — stay correct: seals of 8 x 1 MiB and
    3 x 100 000 B launched back to back on two streams of a fresh context, then opened the same way."""
    import torch

    ctx = aead.AeadCtx(KEY)
    shapes = [(1 << 20, 8), (100000, 3)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    data = []
    for (n, nrec), s in zip(shapes, streams):
        pt = records(0x9100 + n, nrec, n)
        nonces = random_nonces(0x9200 + n, nrec)
        out = empty(nrec * (n + 16), fill=0)
        data.append((n, nrec, pt, nonces, dev(pt), dev(nonces), out))
    torch.cuda.synchronize()
    for (n, nrec, _, _, d_pt, d_n, out), s in zip(data, streams):
        ctx.seal_batch(out, d_pt, d_n, n, nrec, stream=s)
    torch.cuda.synchronize()
    outs = []
    for (n, nrec, pt, nonces, _, d_n, out), s in zip(data, streams):
        assert np.array_equal(host(out)[: nrec * (n + 16)].reshape(nrec, n + 16), oracle.gcm_seal_batch(KEY, nonces, pt))
        back, st = empty(nrec * n, fill=0xAA), status_buf(nrec)
        # the fills run on the current stream: s waits for them, or a late fill overwrites the
        # open's statuses / plaintext
        s.wait_stream(torch.cuda.current_stream())
        ctx.open_batch(back, out, d_n, n, nrec, status=st, stream=s)
        outs.append((back, st))
    torch.cuda.synchronize()
    for (n, nrec, pt, *_), (back, st) in zip(data, outs):
        assert (host(st)[:nrec] == 1).all() and np.array_equal(host(back)[: nrec * n].reshape(nrec, n), pt)


def test_flow_consecutive_shapes_one_stream():
    """FLOW batches of changing shapes (1 to 1 500 records, 1 to 2 048 chunks each) sealed and
    opened back to back on one stream without a synchronisation — chunk-weight tables and scratch
    reused and grown between launches — each checked against the oracle afterwards, one forged
    record per open."""
    aead.force_wide(1, 0)
    ctx = aead.AeadCtx(KEY)
    shapes = [(70000, 2), (1 << 20, 8), (4097, 5), (70000, 2), (20000, 1500), (1 << 20, 3)]
    jobs = []
    for i, (n, nrec) in enumerate(shapes):
        pt = records(0xA100 + i, nrec, n)
        nonces = random_nonces(0xA200 + i, nrec)
        want = oracle.gcm_seal_batch(KEY, nonces, pt)
        forged = want.copy()
        forged[nrec - 1, 0] ^= 0x80
        out, back, st = empty(nrec * (n + 16), fill=0), empty(nrec * n, fill=0x55), status_buf(nrec)
        d_n = dev(nonces)
        ctx.seal_batch(out, dev(pt), d_n, n, nrec)
        ctx.open_batch(back, dev(forged), d_n, n, nrec, status=st)
        jobs.append((n, nrec, pt, want, out, back, st))
    for n, nrec, pt, want, out, back, st in jobs:
        assert np.array_equal(host(out)[: nrec * (n + 16)].reshape(nrec, n + 16), want), (n, nrec)
        assert list(host(st)[:nrec]) == [1] * (nrec - 1) + [0], (n, nrec)
        b = host(back)[: nrec * n].reshape(nrec, n)
        assert np.array_equal(b[: nrec - 1], pt[: nrec - 1]) and not b[nrec - 1].any(), (n, nrec)


@pytest.mark.parametrize("one_wg", [True, False])
@pytest.mark.parametrize("threads", [1024, 512])
@pytest.mark.parametrize("n,nrec,steps", [(1, 1, 0), (100, 3, 1), (4096, 1, 0), (4097, 5, 2), (16384, 1, 0),
                                          (64 * 16 * 5 - 16, 3, 1), (64 * 16 * 5 - 15, 3, 1)])
def test_flow_one_workgroup(one_wg, threads, n, nrec, steps):
    """FLOW batches whose chunks all fit one workgroup (single small messages): with the
    one-workgroup finish the tags come from the workgroup's LDS XOR in the same launch and a
    forged record is zero-filled in-kernel; bit-identical to the combine launch and the oracle.
    Shapes on both sides of the 8 / 16 units-per-workgroup edge, seal twice, forged first and
    last records, then a clean open."""
    aead.force_wide(1, steps)
    aead.set_flow_threads(threads)
    aead.set_flow_one_wg(one_wg)
    ctx = aead.AeadCtx(KEY)
    pt = records(0x7100 + n, nrec, n)
    nonces = random_nonces(0x7200 + n, nrec)
    want = oracle.gcm_seal_batch(KEY, nonces, pt)
    for _ in range(2):
        assert np.array_equal(gpu_seal(ctx, nonces, pt), want), aead.gcm_plan(ctx, n, nrec)
    forged = want.copy()
    forged[0, n] ^= 0x01
    forged[nrec - 1, n + 15] ^= 0x80
    back, st = gpu_open(ctx, nonces, forged)
    bad = {0, nrec - 1}
    assert list(st) == [0 if i in bad else 1 for i in range(nrec)]
    for i in range(nrec):
        assert (not back[i].any()) if i in bad else np.array_equal(back[i], pt[i])
    back, st = gpu_open(ctx, nonces, want)
    assert list(st) == [1] * nrec and np.array_equal(back, pt)


@pytest.mark.parametrize("nrec,segments", [(3, 0), (2, 700), (1, 2)])
def test_lane_groups_many_segments(nrec, segments):
    """1 MiB records on the lane-group plan (wide disabled): hundreds of segment partials per
    record, combined by 256 threads per record with H^{kG} weights (more partials than threads)."""
    n = 1 << 20
    aead.force_wide(-1, 0)
    aead.force_plan(4, segments)
    ctx = aead.AeadCtx(KEY)
    L, nseg, G, r0 = aead.gcm_plan(ctx, n, nrec)
    assert L == 4 and (nseg == 2 if segments == 2 else nseg > 256)
    pt = records(0x4100 + nrec, nrec, n)
    nonces = random_nonces(0x4200 + nrec, nrec)
    want = oracle.gcm_seal_batch(KEY, nonces, pt)
    assert np.array_equal(gpu_seal(ctx, nonces, pt), want), (L, nseg, G, r0)
    forged = want.copy()
    forged[0, 12345] ^= 2
    back, st = gpu_open(ctx, nonces, forged)
    assert st[0] == 0 and not back[0].any()
    assert (st[1:] == 1).all() and np.array_equal(back[1:], pt[1:])


def test_wide_auto_for_naive_alltoall_blocks():
    """8 peer blocks of 1 MiB (BASELINE config 5 per rank) pick the wide plan automatically."""
    ctx = aead.AeadCtx(KEY)
    assert aead.gcm_plan(ctx, 1 << 20, 8)[0] == 64
    assert aead.gcm_plan(ctx, 1024, 65536)[0] != 64


@pytest.mark.parametrize("n", [1024, 4096])
def test_config2_full_batch_properties(n):
    """65 536 x 1 KiB (BASELINE config 2) and 65 536 x 4 KiB (the north-star target): seal->open
    round trip over the whole batch, every tag unique, and every record bit-exact against the
    oracle (the multithreaded C oracle seals the full batch in seconds)."""
    import torch

    nrec = 65536
    g = torch.Generator(device="cuda").manual_seed(1234)
    pt = torch.randint(0, 256, (nrec * n,), dtype=torch.uint8, device="cuda", generator=g)
    nonces = torch.randint(0, 256, (nrec * 12,), dtype=torch.uint8, device="cuda", generator=g)
    ctx = aead.AeadCtx(KEY)
    ct = empty(nrec * (n + 16))
    ctx.seal_batch(ct, pt, nonces, n, nrec)
    back = empty(nrec * n)
    st = status_buf(nrec)
    ctx.open_batch(back, ct, nonces, n, nrec, status=st)
    torch.cuda.synchronize()
    assert bool((st == 1).all())
    assert torch.equal(back, pt)
    got = ct.view(nrec, n + 16).cpu().numpy()
    assert len({t.tobytes() for t in got[:, n:]}) == nrec
    want = oracle.gcm_seal_batch(KEY, nonces.view(nrec, 12).cpu().numpy(), pt.view(nrec, n).cpu().numpy())
    assert np.array_equal(got, want)


@pytest.mark.parametrize("n,nrec", [(0, 1), (1, 1), (777, 20), (65536, 1), (1 << 20, 1), (100000, 3),
                                    ((1 << 20) + 5, 2), ((8 << 20) - 3, 1)])
@pytest.mark.parametrize("pinned", [False, True])
def test_host_direct_single_messages(n, nrec, pinned):
    """Single MPI messages through cmpi_gcm_seal_host / open_host (the EVP drop-in's and the 600
    path's call) on the direct path: bit-exact vs the oracle, forged tag -> CMPI_EAUTH, status 0
    and zero-filled plaintext (aead.h:276-278)."""
    import torch

    pt = records(0x6100 + n, nrec, n)
    nonces = random_nonces(0x6200 + n, nrec)
    ctx = aead.AeadCtx(KEY)
    want = oracle.gcm_seal_batch(KEY, nonces, pt)
    L = aead.N.lib()
    if pinned:
        tp = torch.from_numpy(pt.reshape(-1).copy()).pin_memory()
        tc = torch.empty(nrec * (n + 16), dtype=torch.uint8).pin_memory()
        tb = torch.empty(max(nrec * n, 1), dtype=torch.uint8).pin_memory()
        pp, cp, bp = tp.data_ptr(), tc.data_ptr(), tb.data_ptr()
        ct_view = lambda: tc.numpy().reshape(nrec, n + 16)  # noqa: E731
        back_view = lambda: tb.numpy()[: nrec * n].reshape(nrec, n)  # noqa: E731
    else:
        cbuf = np.zeros((nrec, n + 16), np.uint8)
        bbuf = np.zeros((nrec, max(n, 1)), np.uint8)
        pp, cp, bp = pt.ctypes.data, cbuf.ctypes.data, bbuf.ctypes.data
        ct_view = lambda: cbuf  # noqa: E731
        back_view = lambda: bbuf[:, :n]  # noqa: E731
    aead.N.check(L.cmpi_gcm_seal_host(ctx.handle, cp, n + 16, pp, max(n, 1), nonces.ctypes.data, 12, n, nrec))
    assert np.array_equal(ct_view(), want)
    st = np.zeros(nrec, np.int32)
    aead.N.check(L.cmpi_gcm_open_host(ctx.handle, bp, max(n, 1), cp, n + 16, nonces.ctypes.data, 12, n, nrec,
                                      st.ctypes.data))
    assert (st == 1).all() and np.array_equal(back_view(), pt)
    ct_view()[nrec - 1, -1] ^= 1
    rc = L.cmpi_gcm_open_host(ctx.handle, bp, max(n, 1), cp, n + 16, nonces.ctypes.data, 12, n, nrec, st.ctypes.data)
    assert rc == aead.N.CMPI_EAUTH and st[nrec - 1] == 0 and (st[: nrec - 1] == 1).all()
    assert not back_view()[nrec - 1].any()


def test_host_staging_api():
    n, nrec = 777, 20
    pt = records(3, nrec, n)
    nonces = random_nonces(4, nrec)
    ctx = aead.AeadCtx(KEY)
    got = ctx.seal_host_batch(nonces, pt)
    assert np.array_equal(got, oracle.gcm_seal_batch(KEY, nonces, pt))
    back, st = ctx.open_host_batch(nonces, got)
    assert (st == 1).all() and np.array_equal(back, pt)
    # EVP_AEAD_CTX_seal/open single-message mirror
    one = ctx.seal(nonces[0].tobytes(), pt[0].tobytes())
    assert one == oracle.gcm_seal(KEY, nonces[0].tobytes(), pt[0].tobytes())
    assert ctx.open(nonces[0].tobytes(), one) == pt[0].tobytes()
    assert ctx.open(nonces[0].tobytes(), one[:-1] + bytes([one[-1] ^ 1])) is None


def test_subkey602_matches_oracle():
    """602 sub-key (send.c:572-600): K' = AES-ECB_K(V) on the GPU, then GCM under K'."""
    base = aead.CipherCtx(KEY, "aes-128-ecb")
    v = splitmix64_bytes(0x602, 16).tobytes()
    sub = aead.AeadCtx.subkey602(base, v)
    kprime = oracle.ecb_encrypt(KEY, v)
    pt = records(11, 4, 300)
    nonces = np.stack([np.frombuffer(oracle.nonce602(b"0", i), np.uint8) for i in range(4)])
    assert np.array_equal(gpu_seal(sub, nonces, pt), oracle.gcm_seal_batch(kprime, nonces, pt))


@pytest.mark.parametrize("n,off,pad", [(17, 1, 3), (1000, 5, 7), (4096, 3, 1), (33, 2, 0)])
def test_unaligned_records(n, off, pad):
    """Records at arbitrary byte offsets / odd strides (wire layouts with odd n, the 602 5-byte
    segment prefix): the engine reads and writes them in place."""
    nrec = 12
    in_stride, out_stride, n_stride = n + pad, n + 16 + pad + 1, 12 + pad
    pt = records(31 + n, nrec, n)
    nonces = random_nonces(32 + n, nrec)
    inbuf = np.zeros(off + nrec * in_stride, np.uint8)
    nbuf = np.zeros(off + nrec * n_stride, np.uint8)
    for i in range(nrec):
        inbuf[off + i * in_stride: off + i * in_stride + n] = pt[i]
        nbuf[off + i * n_stride: off + i * n_stride + 12] = nonces[i]
    outsz = off + nrec * out_stride
    d_out = empty(outsz, fill=0x77)
    ctx = aead.AeadCtx(KEY)
    ctx.seal_batch(d_out[off:], dev(inbuf)[off:], dev(nbuf)[off:], n, nrec, in_stride=in_stride,
                   out_stride=out_stride, nonce_stride=n_stride)
    got = host(d_out)
    want = oracle.gcm_seal_batch(KEY, nonces, pt)
    for i in range(nrec):
        assert got[off + i * out_stride: off + i * out_stride + n + 16].tobytes() == want[i].tobytes(), i
        gap = got[off + i * out_stride + n + 16: off + (i + 1) * out_stride]
        assert (gap == 0x77).all()  # bytes between records untouched
    back = empty(off + nrec * in_stride, fill=0)
    st = status_buf(nrec)
    ctx.open_batch(back[off:], d_out[off:], dev(nbuf)[off:], n, nrec, status=st, in_stride=out_stride,
                   out_stride=in_stride, nonce_stride=n_stride)
    assert (host(st)[:nrec] == 1).all()
    assert np.array_equal(host(back), inbuf)


@pytest.mark.parametrize("n,nrec,plan", [(300, 4, None), (4096, 3, (4, 0)), (65536, 2, (4, 5)), (100, 40, (2, 0)),
                                         (1 << 20, 1, None), (31, 7, (1, 0))])
def test_derived_subkey_device_keyed(n, nrec, plan):
    """cmpi_ctx_derive_subkey: K' = AES_K(V), key schedule, H and every GHASH table built by the
    key-setup kernel on the stream (no host copy of K'); seal/open through every plan shape,
    incl. multi-segment records whose H^{kG} weights are then also computed on the device."""
    base = aead.CipherCtx(KEY, "aes-128-ecb")
    v = splitmix64_bytes(0x60200 + n, 16).tobytes()
    kprime = oracle.ecb_encrypt(KEY, v)
    pt = records(13 + n, nrec, n)
    nonces = np.stack([np.frombuffer(oracle.nonce602(b"1", 7 + i), np.uint8) for i in range(nrec)])
    try:
        if plan:
            aead.force_plan(*plan)
        sub = aead.AeadCtx.derive_subkey(base, v)
        want = oracle.gcm_seal_batch(kprime, nonces, pt)
        assert np.array_equal(gpu_seal(sub, nonces, pt), want)
        ct = dev(want)
        d_pt, st = empty(nrec * n), status_buf(nrec)
        sub.open_batch(d_pt, ct, dev(nonces), n, nrec, status=st)
        assert (host(st)[:nrec] == 1).all()
        assert host(d_pt)[: nrec * n].tobytes() == pt.tobytes()
    finally:
        aead.force_plan(0, 0)


@pytest.mark.parametrize("n,nrec,wide,plan", [(100000, 3, (1, 2), None), (1 << 20, 2, (1, 0), None),
                                           (65536, 9, (-1, 0), (4, 40)), (4097, 5, (-1, 0), (2, 3))])
def test_derived_subkey_wide_and_pow2_segments(n, nrec, wide, plan):
    """Device-keyed contexts on the wide plan (gcm_flow_kernel with the table kernel's nibble
    tables; chunk weights as products of H^(2^i) in gcm_combine_kernel) and on multi-segment lane
    groups (G rounded to a power of two, same combine): bit-exact vs the oracle under
    K' = AES_K(V), forgery."""
    base = aead.CipherCtx(KEY, "aes-128-ecb")
    v = splitmix64_bytes(0x61200 + n, 16).tobytes()
    kprime = oracle.ecb_encrypt(KEY, v)
    pt = records(17 + n, nrec, n)
    nonces = np.stack([np.frombuffer(oracle.nonce602(b"0", 3 + i), np.uint8) for i in range(nrec)])
    aead.force_wide(*wide)
    if plan:
        aead.force_plan(*plan)
    sub = aead.AeadCtx.derive_subkey(base, v)
    L, nseg, G, r0 = aead.gcm_plan(sub, n, nrec)
    assert (L == 64) == (wide[0] == 1) and (nseg == 1 or G & (G - 1) == 0), (L, nseg, G)
    want = oracle.gcm_seal_batch(kprime, nonces, pt)
    assert np.array_equal(gpu_seal(sub, nonces, pt), want), (L, nseg, G, r0)
    forged = want.copy()
    forged[nrec // 2, -3] ^= 1
    back, st = gpu_open(sub, nonces, forged)
    bad = nrec // 2
    assert st[bad] == 0 and not back[bad].any()
    assert all(st[i] == 1 and np.array_equal(back[i], pt[i]) for i in range(nrec) if i != bad)


def test_rekey_subkey_reuses_context():
    """One context re-keyed per message (what a 602 sender thread does per MPI_Send)."""
    base = aead.AeadCtx(KEY)  # any context holding K serves as the base
    sub = aead.AeadCtx(bytes(16))
    pt = records(99, 5, 1000)
    nonces = np.stack([np.frombuffer(oracle.nonce602(b"0", i), np.uint8) for i in range(5)])
    for m in range(3):
        v = splitmix64_bytes(0x777 + m, 16).tobytes()
        sub.rekey_subkey(base, v)
        assert np.array_equal(gpu_seal(sub, nonces, pt), oracle.gcm_seal_batch(oracle.ecb_encrypt(KEY, v), nonces, pt)), m


def test_device_keyed_ctx_rejects_ctr():
    base = aead.CipherCtx(KEY, "aes-128-ecb")
    sub = aead.AeadCtx.derive_subkey(base, bytes(range(16)))
    rc = aead.N.lib().cmpi_ctr_keystream(sub.handle, None, 1, (aead.ctypes.c_uint8 * 16)(), None)
    assert rc == aead.N.CMPI_EINVAL
    import torch

    torch.cuda.synchronize()  # the key-setup kernel is asynchronous


@pytest.mark.parametrize("direct", [0, 1 << 30])
@pytest.mark.parametrize("out_pad", [0, 28])
def test_host_pipeline_pinned_in_and_out(out_pad, direct):
    """Registered host buffers on both sides move by flat DMA (device pitch = user stride) when
    the output is dense; a gapped output (the wire layout's nonce between records) must keep
    the caller's gap bytes.  direct: the kernel reads / writes the registered pages itself
    (their device address from hipPointerGetAttributes) at the caller's strides."""
    aead.N.lib().cmpi_debug_set_host_direct(direct)
    n, nrec = 1000, 257
    pt = records(0x7171 + out_pad, nrec, n)
    nonces = random_nonces(0x7172, nrec)
    ctx = aead.AeadCtx(KEY)
    want = oracle.gcm_seal_batch(KEY, nonces, pt)
    ostride = n + 16 + out_pad
    out = np.full((nrec, ostride), 0x5A, np.uint8)
    L = aead.N.lib()
    assert L.cmpi_host_register(pt.ctypes.data, pt.nbytes) == 0
    assert L.cmpi_host_register(out.ctypes.data, out.nbytes) == 0
    if out_pad == 0:  # pinned nonces too (own mmap'd pages): they then move by flat DMA
        nbuf = np.zeros(1 << 20, np.uint8)
        nbuf[: nrec * 12] = nonces.reshape(-1)
        nonces = nbuf[: nrec * 12].reshape(nrec, 12)
        assert L.cmpi_host_register(nbuf.ctypes.data, nbuf.nbytes) == 0
    try:
        L.cmpi_debug_set_host_chunk(64 * 1024)
        aead.N.check(L.cmpi_gcm_seal_host(ctx.handle, out.ctypes.data, ostride, pt.ctypes.data, n,
                                          nonces.ctypes.data, 12, n, nrec))
        assert np.array_equal(out[:, : n + 16], want)
        assert (out[:, n + 16:] == 0x5A).all()
    finally:
        L.cmpi_debug_set_host_chunk(0)
        L.cmpi_host_unregister(pt.ctypes.data)
        L.cmpi_host_unregister(out.ctypes.data)
        if out_pad == 0:
            L.cmpi_host_unregister(nbuf.ctypes.data)


@pytest.mark.parametrize("alg", ["aes-128-gcm", "aes-128-ocb"])
@pytest.mark.parametrize("chunk", [4096, 65536, 0, -1])
def test_host_pipeline_chunks(alg, chunk):
    """The pipelined host path (3 streams, 2 staging slots) across many chunks, ragged last chunk,
    forged records reported per record and zero-filled, for pinned (registered) and pageable.
    chunk -1: the direct path (kernel on page-locked host memory, pageable records packed through
    the pinned bounce buffer) on the same cases."""
    aead.N.lib().cmpi_debug_set_host_direct(1 << 30 if chunk < 0 else 0)
    chunk = max(chunk, 0)
    n, nrec = 1000, 301
    pt = records(0x5151 + chunk, nrec, n)
    nonces = random_nonces(0x5152, nrec)
    ctx = aead.AeadCtx(KEY, alg)
    want = (oracle.gcm_seal_batch if alg == "aes-128-gcm" else oracle.ocb_seal_batch)(KEY, nonces, pt)
    try:
        aead.N.lib().cmpi_debug_set_host_chunk(chunk)
        got = ctx.seal_host_batch(nonces, pt)
        assert np.array_equal(got, want)
        forged = got.copy()
        forged[[0, 150, 300], -1] ^= 1
        back, st = ctx.open_host_batch(nonces, forged)
        assert list(np.nonzero(st == 0)[0]) == [0, 150, 300]
        assert (back[[0, 150, 300]] == 0).all() and np.array_equal(back[1:150], pt[1:150])
        back, st = ctx.open_host_batch(nonces, got)
        assert (st == 1).all() and np.array_equal(back, pt)
        # registered (pinned) host buffers
        buf = np.ascontiguousarray(pt)
        assert aead.N.lib().cmpi_host_register(buf.ctypes.data, buf.nbytes) == 0
        try:
            assert np.array_equal(ctx.seal_host_batch(nonces, buf), want)
        finally:
            aead.N.lib().cmpi_host_unregister(buf.ctypes.data)
    finally:
        aead.N.lib().cmpi_debug_set_host_chunk(0)


@pytest.mark.parametrize("nrec,n", [(8, 1 << 20), (8, (1 << 20) - 5)])
def test_config5_shape_default_plan(nrec, n):
    """BASELINE config 5 per rank (8 peer blocks of 1 MiB, alltoall.c:795-834) through the
    planner's default form (flow kernel + XOR combine), plus a ragged length: every byte of every
    record against the oracle, then open round trip and a forged tag in the last record."""
    ctx = aead.AeadCtx(KEY)
    pt = records(0x5E00 + n, nrec, n)
    nonces = random_nonces(0x5E01 + n, nrec)
    want = oracle.gcm_seal_batch(KEY, nonces, pt)
    got = gpu_seal(ctx, nonces, pt)
    assert np.array_equal(got, want), aead.gcm_plan(ctx, n, nrec)
    forged = want.copy()
    forged[nrec - 1, n + 15] ^= 0x01
    back, st = gpu_open(ctx, nonces, forged)
    assert list(st) == [1] * (nrec - 1) + [0]
    assert np.array_equal(back[: nrec - 1], pt[: nrec - 1]) and not back[nrec - 1].any()


@pytest.mark.parametrize("n,steps", [(1 << 20, 0), (64 * 16 * 3 - 5, 1)])
def test_flow_combine_each_tag_byte(n, steps):
    """gcm_xor_combine_kernel's tag check (the received tag is loaded beside the partials): 17
    multi-chunk records, record i < 16 with tag byte i flipped, record 16 intact — each forged
    record rejected and zero-filled, the intact one opened, whatever word of the tag differs."""
    aead.force_wide(1, steps)
    aead.set_flow_one_wg(False)
    nrec = 17
    ctx = aead.AeadCtx(KEY)
    assert aead.gcm_plan(ctx, n, nrec)[1] > 1
    pt = records(0x7A6 + n, nrec, n)
    nonces = random_nonces(0x7A7 + n, nrec)
    want = oracle.gcm_seal_batch(KEY, nonces, pt)
    assert np.array_equal(gpu_seal(ctx, nonces, pt), want)
    forged = want.copy()
    for i in range(16):
        forged[i, n + i] ^= 1 << (i % 8)
    back, st = gpu_open(ctx, nonces, forged)
    assert list(st) == [0] * 16 + [1]
    assert not back[:16].any() and np.array_equal(back[16], pt[16])


@pytest.mark.parametrize("n,nrec", [(32768, 16), (1 << 20, 8), (100000, 3), (65536 + 1, 1), (8 << 20, 1),
                                    (64 * 16 * 3 - 5, 7)])
@pytest.mark.parametrize("threads", [0, 1024])
def test_derived_subkey_flow_plan(n, nrec, threads):
    """602 per-message sub-key contexts (send.c:572-600: K' = AES_K(V) derived on the device) on
    the planner's default flow plan at 602 shapes — OpenMP segments of 32 KiB, 1 MiB, single
    messages just over 64 KiB and of 8 MiB: gcm_flow_kernel<DK> (round keys from HBM, partials
    V·H) + gcm_combine_kernel (chunk weights from H^(2^i), E_K(J0)).  Seal and open bit-exact vs the
    oracle under K', a forged record zero-filled, the context re-keyed to a second V."""
    aead.set_flow_threads(threads)
    base = aead.CipherCtx(KEY, "aes-128-ecb")
    sub = None
    for m, seed in enumerate((0x60600, 0x60601)):
        v = splitmix64_bytes(seed + n, 16).tobytes()
        kprime = oracle.ecb_encrypt(KEY, v)
        if sub is None:
            sub = aead.AeadCtx.derive_subkey(base, v)
        else:
            sub.rekey_subkey(base, v)
        assert aead.gcm_plan(sub, n, nrec)[0] == 64, aead.gcm_plan(sub, n, nrec)
        pt = records(0x6060 + n + m, nrec, n)
        nonces = np.stack([np.frombuffer(oracle.nonce602(b"1" if i == nrec - 1 else b"0", i), np.uint8)
                           for i in range(nrec)])
        want = oracle.gcm_seal_batch(kprime, nonces, pt)
        assert np.array_equal(gpu_seal(sub, nonces, pt), want), aead.gcm_plan(sub, n, nrec)
        forged = want.copy()
        forged[nrec - 1, n // 2] ^= 0x08
        back, st = gpu_open(sub, nonces, forged)
        assert list(st) == [1] * (nrec - 1) + [0]
        assert np.array_equal(back[: nrec - 1], pt[: nrec - 1]) and not back[nrec - 1].any()
