"""Resident message service (include/cmpi_service.h): single GCM messages from host memory —
the per-message EVP_AEAD_CTX_seal / _open of MPI_SEC_Multi_Thread_Send/Recv_OpenMP
(MV/src/mpi/pt2pt/send.c:294-315, recv.c:322) — served by a kernel that stays resident between
messages.  Every byte and status against the oracle (oracle/gcm_ref.c: SP 800-38D, pinned to the
published KATs that SURVEY.md §8c records BoringSSL reproducing and to OpenSSL 3 vectors — the
reference ships no vectors of its own); pinned and pageable buffers; forged tags
zero-filled with CMPI_EAUTH (aead.h:276-278); idle exit and relaunch; re-key; several contexts at
once; host buffers whose device address has bit 31 of its low word set (the sign-extension fault
fixed in service_kernels.hpp lds_ptr64)."""
import ctypes
import time

import numpy as np
import pytest
import torch

import oracle
from cryptmpi_2022_amd import _native as N
from cryptmpi_2022_amd import aead
from cryptmpi_2022_amd.synth import splitmix64_bytes

pytestmark = pytest.mark.gpu

KEY = bytes(range(16))
# 0 .. the service's 512 KiB limit (64 chunks of 8 steps) and one past it (the direct path)
SIZES = [0, 1, 15, 16, 17, 100, 1000, 1024, 1040, 4096, 4097, 8191, 8192, 8193, 30000, 65535, 65536, 65537,
         100000, 131072, 262144, 300001, 524288, 524289]


def _host(n: int, pinned: bool, fill: int = 0):
    if pinned:
        t = torch.full((max(n, 1),), fill, dtype=torch.uint8).pin_memory()
        return t.numpy()[:n], t
    return np.full(max(n, 1), fill, np.uint8)[:n], None


def _seal(ctx, out, pt, nonce: bytes, n: int):
    nb = (ctypes.c_uint8 * 12).from_buffer_copy(nonce)
    return N.lib().cmpi_gcm_seal_host(ctx.handle, ctypes.c_void_p(out.ctypes.data), n + 16,
                                      ctypes.c_void_p(pt.ctypes.data), max(n, 1), nb, 12, n, 1)


def _open(ctx, out, ct, nonce: bytes, n: int, st):
    nb = (ctypes.c_uint8 * 12).from_buffer_copy(nonce)
    return N.lib().cmpi_gcm_open_host(ctx.handle, ctypes.c_void_p(out.ctypes.data), max(n, 1),
                                      ctypes.c_void_p(ct.ctypes.data), n + 16, nb, 12, n, 1,
                                      ctypes.c_void_p(st.ctypes.data))


@pytest.fixture
def svc_ctx():
    ctx = aead.AeadCtx(KEY)
    ctx.service_start(20000)
    yield ctx
    ctx.service_stop()
    ctx.close()


@pytest.mark.parametrize("pinned", [True, False])
def test_service_seal_open_vs_oracle(svc_ctx, pinned):
    for n in SIZES:
        pt = splitmix64_bytes(0x5E7 + n, n)
        nonce = splitmix64_bytes(0x90 + n, 12).tobytes()
        src, _k1 = _host(n, pinned)
        src[:] = pt
        ct, _k2 = _host(n + 16, pinned, fill=0xA5)
        assert _seal(svc_ctx, ct, src, nonce, n) == N.CMPI_OK, n
        want = oracle.gcm_seal(KEY, nonce, pt.tobytes())
        assert ct.tobytes() == want, n
        back, _k3 = _host(n, pinned, fill=0x3C)
        st = np.full(1, 7, np.int32)
        assert _open(svc_ctx, back, ct, nonce, n, st) == N.CMPI_OK, n
        assert st[0] == 1 and back.tobytes() == pt.tobytes(), n
        # a forged tag (byte n % 16; an empty message too): status 0, plaintext zero-filled, CMPI_EAUTH
        ct[n + n % 16] ^= 0x01
        bad, _k4 = _host(n, pinned, fill=0x77)
        st[0] = 7
        assert _open(svc_ctx, bad, ct, nonce, n, st) == N.CMPI_EAUTH, n
        assert st[0] == 0 and not bad.any(), n
    # the oracle's bit-serial GHASH between messages may outlast the 20 ms idle limit: the kernel
    # exits and the next message relaunches it
    src, _k1 = _host(64, pinned)
    ct, _k2 = _host(80, pinned)
    assert _seal(svc_ctx, ct, src, bytes(12), 64) == N.CMPI_OK
    assert svc_ctx.service_running()


def test_service_message_sequence(svc_ctx):
    """Many messages back to back, seal and open interleaved, sizes across every chunk count."""
    rng = np.random.default_rng(11)
    src, _k1 = _host(200000, True)
    ct, _k2 = _host(200016, True)
    back, _k3 = _host(200000, True)
    st = np.zeros(1, np.int32)
    for i in range(300):
        n = int(rng.integers(0, 200000)) if i % 3 else int(rng.integers(0, 2048))
        pt = splitmix64_bytes(i, n)
        nonce = splitmix64_bytes(1000 + i, 12).tobytes()
        src[:n] = pt
        assert _seal(svc_ctx, ct, src, nonce, n) == N.CMPI_OK
        assert ct[: n + 16].tobytes() == oracle.gcm_seal(KEY, nonce, pt.tobytes()), (i, n)
        assert _open(svc_ctx, back, ct, nonce, n, st) == N.CMPI_OK and st[0] == 1
        assert back[:n].tobytes() == pt.tobytes(), (i, n)


def test_service_idle_exit_and_relaunch():
    ctx = aead.AeadCtx(KEY)
    ctx.service_start(300)  # 0.3 ms idle
    pt = splitmix64_bytes(5, 4096)
    nonce = bytes(12)
    want = oracle.gcm_seal(KEY, nonce, pt.tobytes())
    for _ in range(3):
        assert ctx.seal(nonce, pt.tobytes()) == want
        assert ctx.service_running()
        time.sleep(0.05)
        assert not ctx.service_running()  # the kernel returned its CUs
    ctx.service_stop()
    assert ctx.seal(nonce, pt.tobytes()) == want  # the direct path again
    ctx.close()


def test_service_rekey_and_free():
    ctx = aead.AeadCtx(KEY)
    ctx.service_start(0)
    pt = splitmix64_bytes(9, 70000).tobytes()
    nonce = bytes(range(12))
    assert ctx.seal(nonce, pt) == oracle.gcm_seal(KEY, nonce, pt)
    k2 = bytes(range(100, 116))
    ctx.rekey(k2)
    torch.cuda.synchronize()
    assert ctx.seal(nonce, pt) == oracle.gcm_seal(k2, nonce, pt)  # relaunched with the new key
    assert ctx.open(nonce, oracle.gcm_seal(k2, nonce, pt)) == pt
    assert ctx.service_running()
    ctx.close()  # stops the resident kernel


def test_service_two_contexts():
    a, b = aead.AeadCtx(KEY), aead.AeadCtx(bytes(16))
    a.service_start(0)
    b.service_start(0)
    for i in range(20):
        n = 1000 * i + 7
        pt = splitmix64_bytes(i, n).tobytes()
        nonce = splitmix64_bytes(50 + i, 12).tobytes()
        assert a.seal(nonce, pt) == oracle.gcm_seal(KEY, nonce, pt)
        assert b.seal(nonce, pt) == oracle.gcm_seal(bytes(16), nonce, pt)
    a.close()
    b.close()


def test_service_many_contexts_share_slots():
    """More services than hardware queues (6 contexts, 4 stream slots): round-robin messages over
    them are all bit-exact, and none waits for another context's resident kernel to idle out —
    the slot's holder is kicked and the new generation queues behind it (was: ~20 ms per message
    whose stream shared a queue with another resident kernel, tools/svc_many_probe.py)."""
    keys = [bytes([k + 1] * 16) for k in range(6)]
    ctxs = [aead.AeadCtx(k) for k in keys]
    for c in ctxs:
        c.service_start(500000)  # resident for the whole test unless kicked
    lat = []
    for i in range(36):
        k = i % 6
        pt = splitmix64_bytes(900 + i, 1000 + i).tobytes()
        nonce = splitmix64_bytes(950 + i, 12).tobytes()
        t0 = time.perf_counter()
        got = ctxs[k].seal(nonce, pt)
        lat.append(time.perf_counter() - t0)
        assert got == oracle.gcm_seal(keys[k], nonce, pt), i
        assert ctxs[k].open(nonce, got) == pt
    for c in ctxs:
        c.service_stop()
        c.close()
    # the failure this guards against waited for a resident kernel's idle-out / lifetime (>= 100 ms
    # here): 50 ms leaves a loaded box its margin
    assert max(lat[6:]) < 0.05, [round(v * 1e3, 2) for v in lat]


def test_service_stuck_shutdown_then_new_services():
    """A shutdown whose stop fails with the generation still resident (forced by the test hook
    cmpi_debug_set_svc_fake_stuck) leaks the service object instead of freeing it, because a stream
    slot still names it as its owner (svc_launch reads the owner's exit word and writes
    its kick word).  Services started afterwards on other contexts — taking every slot, the
    stuck one's included — serve bit-exact messages."""
    ctx = aead.AeadCtx(KEY)
    ctx.service_start(2000)
    pt = splitmix64_bytes(0x57, 5000).tobytes()
    nonce = splitmix64_bytes(0x58, 12).tobytes()
    assert ctx.seal(nonce, pt) == oracle.gcm_seal(KEY, nonce, pt)
    assert ctx.service_running()
    N.lib().cmpi_debug_set_svc_fake_stuck(1)
    try:
        ctx.close()  # shutdown "fails": the Svc is leaked, its kernel idles out by itself
    finally:
        N.lib().cmpi_debug_set_svc_fake_stuck(0)
    keys = [bytes([0x40 + k] * 16) for k in range(6)]
    ctxs = [aead.AeadCtx(k) for k in keys]
    for c in ctxs:
        c.service_start(500000)
    for i in range(24):
        k = i % 6
        p = splitmix64_bytes(0x600 + i, 777 + 13 * i).tobytes()
        nn = splitmix64_bytes(0x700 + i, 12).tobytes()
        got = ctxs[k].seal(nn, p)
        assert got == oracle.gcm_seal(keys[k], nn, p), i
        assert ctxs[k].open(nn, got) == p
    for c in ctxs:
        c.service_stop()
        c.close()


def test_service_many_contexts_two_threads():
    """Two host threads, each round-robin over three of six serviced contexts (4 stream slots):
    launches on held slots kick other threads' generations while their messages are posted; every
    message completes bit-exact (the concurrent kick / relaunch path)."""
    import threading

    keys = [bytes([k + 31] * 16) for k in range(6)]
    ctxs = [aead.AeadCtx(k) for k in keys]
    for c in ctxs:
        c.service_start(500000)
    errors = []

    def worker(t):
        try:
            for i in range(30):
                k = 3 * t + i % 3
                pt = splitmix64_bytes(1000 * t + i, 700 + 37 * i).tobytes()
                nonce = splitmix64_bytes(5000 * t + i, 12).tobytes()
                got = ctxs[k].seal(nonce, pt)
                if got != oracle.gcm_seal(keys[k], nonce, pt) or ctxs[k].open(nonce, got) != pt:
                    errors.append((t, i))
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=60)
    for c in ctxs:
        c.service_stop()
        c.close()
    assert not any(x.is_alive() for x in th)
    assert errors == []


def test_service_leaves_other_streams_free():
    """While the service kernel is resident, kernels on 8 other (normal-priority) streams and on the
    default stream complete without waiting for it: the service's stream sits in the greatest-
    priority queue pool (at normal priority one of them shared its hardware queue and
    waited up to the kernel's 100 ms lifetime, profiles/r04a_queue_probe.jsonl)."""
    streams = [torch.cuda.Stream() for _ in range(8)]
    x = torch.ones(16, device="cuda")
    for s in streams:  # first use of each stream (queue creation, code object load) before timing
        with torch.cuda.stream(s):
            x.add_(1)
        s.synchronize()
    ctx = aead.AeadCtx(KEY)
    ctx.service_start(500000)  # 0.5 s idle: resident through the whole check
    pt = splitmix64_bytes(77, 4096).tobytes()
    assert ctx.seal(bytes(12), pt) == oracle.gcm_seal(KEY, bytes(12), pt)
    assert ctx.service_running()
    lat = []
    for s in streams + [torch.cuda.current_stream()]:
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            x.add_(1)
        s.synchronize()
        lat.append(time.perf_counter() - t0)
    assert ctx.service_running()  # still resident: nothing above waited for it to exit
    ctx.service_stop()
    ctx.close()
    assert max(lat) < 0.05, [round(v * 1e3, 2) for v in lat]  # was: up to the kernel's 100 ms lifetime


def test_service_refuses_other_contexts():
    ocb = aead.AeadCtx(KEY, "aes-128-ocb")
    with pytest.raises(N.CmpiError):
        ocb.service_start(0)
    ocb.close()
    master = aead.AeadCtx(KEY)
    sub = aead.AeadCtx.subkey602(master, bytes(range(16)))
    with pytest.raises(N.CmpiError):
        sub.service_start(0)
    sub.close()
    master.close()


# ---------------------------------------------------------------- high-bit host addresses
# Round 3's service fault: a descriptor's 64-bit host address travels as two 32-bit words and was
# rebuilt from a sign-extended readfirstlane of the low word, so an address whose low word has bit
# 31 set turned into 0xFFFFFFFF'xxxxxxxx (service_kernels.hpp lds_ptr64).  The allocator only
# sometimes returns such addresses; here the buffers are mapped at fixed ones.
_MAP_CANDIDATES = [0x7F00_8000_0000, 0x7E00_8000_0000, 0x6F00_8000_0000, 0x5F00_C000_0000, 0x4F00_8000_0000]
_MAP_BYTES = 4 << 20


def _libc():
    libc = ctypes.CDLL(None, use_errno=True)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    return libc


def _dev_ptr(p: int) -> int:
    hip = ctypes.CDLL("libamdhip64.so")
    d = ctypes.c_void_p()
    assert hip.hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(p), 0) == 0
    return d.value or 0


@pytest.fixture
def high_bit_region():
    """4 MiB of page-locked host memory mapped at a fixed address whose low 32-bit word has bit 31
    set (MAP_FIXED_NOREPLACE: never over an existing mapping), registered with cmpi_host_register;
    its device address is checked to carry that bit too."""
    libc = _libc()
    PROT_RW, MAP_PRIV_ANON, MAP_FIXED_NOREPLACE = 0x3, 0x22, 0x100000
    base = None
    for a in _MAP_CANDIDATES:
        r = libc.mmap(ctypes.c_void_p(a), _MAP_BYTES, PROT_RW, MAP_PRIV_ANON | MAP_FIXED_NOREPLACE, -1, 0)
        if r is not None and r != ctypes.c_void_p(-1).value and r == a:
            base = a
            break
        if r is not None and r != ctypes.c_void_p(-1).value:
            libc.munmap(ctypes.c_void_p(r), _MAP_BYTES)  # an old kernel ignored the flag: not the address asked
    assert base is not None, "no fixed high-bit address could be mapped"
    ctypes.memset(base, 0, _MAP_BYTES)
    L = N.lib()
    assert L.cmpi_host_register(ctypes.c_void_p(base), _MAP_BYTES) == N.CMPI_OK
    hip = ctypes.CDLL("libamdhip64.so")
    try:
        d = _dev_ptr(base)
        assert d & 0x8000_0000 and (d >> 32) not in (0, 0xFFFF_FFFF), hex(d)
        yield base
    finally:
        torch.cuda.synchronize()
        hip.hipHostUnregister(ctypes.c_void_p(base))
        libc.munmap(ctypes.c_void_p(base), _MAP_BYTES)


@pytest.mark.parametrize("service", [True, False])
def test_high_bit_host_addresses(high_bit_region, service):
    """Seal and open from and into host buffers at addresses 0x....8xxx_xxxx (input at the region
    base, output 2 MiB above it, nonce inside it): through the resident service (one and several
    workgroups) and through the direct path, every byte and status against the oracle, a forged
    message zero-filled."""
    base = high_bit_region
    half = _MAP_BYTES // 2
    buf = (ctypes.c_uint8 * _MAP_BYTES).from_address(base)
    view = np.frombuffer(buf, dtype=np.uint8)
    src, dst = view[:half], view[half:]
    ctx = aead.AeadCtx(KEY)
    if service:
        ctx.service_start(20000)
    L = N.lib()
    nonce_off = half - 64  # the nonce in the region as well (the direct path reads it from there)
    for n in (1, 1000, 4096, 65536, 300001, 524288):
        pt = splitmix64_bytes(0xB17 + n, n)
        nonce = splitmix64_bytes(0x31 + n, 12).tobytes()
        src[:n] = pt
        view[nonce_off:nonce_off + 12] = np.frombuffer(nonce, np.uint8)
        dst[: n + 16] = 0xA5
        np_ptr = ctypes.c_void_p(base + nonce_off)
        assert L.cmpi_gcm_seal_host(ctx.handle, ctypes.c_void_p(base + half), n + 16, ctypes.c_void_p(base), n,
                                    np_ptr, 12, n, 1) == N.CMPI_OK, n
        want = oracle.gcm_seal(KEY, nonce, pt.tobytes())
        assert dst[: n + 16].tobytes() == want, n
        # open: ciphertext at the region base, plaintext into the upper half
        src[: n + 16] = np.frombuffer(want, np.uint8)
        dst[:n] = 0x3C
        st = np.full(1, 7, np.int32)
        assert L.cmpi_gcm_open_host(ctx.handle, ctypes.c_void_p(base + half), n, ctypes.c_void_p(base), n + 16,
                                    np_ptr, 12, n, 1, ctypes.c_void_p(st.ctypes.data)) == N.CMPI_OK, n
        assert st[0] == 1 and dst[:n].tobytes() == pt.tobytes(), n
        src[n + 3] ^= 0x40  # forged tag
        dst[:n] = 0x77
        assert L.cmpi_gcm_open_host(ctx.handle, ctypes.c_void_p(base + half), n, ctypes.c_void_p(base), n + 16,
                                    np_ptr, 12, n, 1, ctypes.c_void_p(st.ctypes.data)) == N.CMPI_EAUTH, n
        assert st[0] == 0 and not dst[:n].any(), n
        if service:
            assert ctx.service_running(), n
    if service:
        ctx.service_stop()
    ctx.close()
