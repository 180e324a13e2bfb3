#!/usr/bin/env python3
"""bench.py — device-resident AES-GCM seal+open throughput on MI355X (BASELINE.json metric).

A "step" = one AES-128-GCM seal of a whole batch of synthetic records followed by one open of
the resulting ct||tag batch (BASELINE config 2: 65 536 x 1 KiB per GPU), inputs resident in
HBM before the timed region.  value = plaintext bytes sealed-and-opened by ALL ranks per second
(GiB/s, n*N / (t_seal + t_open) per record pass), weak scaling: every rank owns
its own batch (records are independent; no data-path collective — SURVEY.md §8e).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload gcm1k|gcm4k|ocb1m|ctr1g|alltoall]
                    [--no-cpu-baseline] [--no-extras]

Multi-GPU: launched by torch.distributed.run (one process per GPU); only the timing barrier and
the max-over-ranks reduction use the process group.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from cryptmpi_2022_amd import aead  # noqa: E402

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md), GB/s
KEY = bytes.fromhex("000102030405060708090a0b0c0d0e0f")

WORKLOADS = {
    # name: (alg, record bytes, records, description)
    "gcm1k": ("gcm", 1024, 65536, "BASELINE config 2: 65536 x 1 KiB AES-128-GCM seal+open"),
    "gcm4k": ("gcm", 4096, 65536, "north-star target: 65536 x 4 KiB AES-128-GCM seal+open"),
    "ocb1m": ("ocb", 1 << 20, 4096, "BASELINE config 3: 4096 x 1 MiB AES-128-OCB seal+open"),
    "ctr1g": ("ctr", 1 << 30, 1, "BASELINE config 4: 1 GiB AES-128-CTR keystream+XOR"),
    # SURVEY §8(d) config 4's second form: the keystream materialised into a 1 GiB mask (the a8
    # mask ring, generateCommonEncMask send.c:1162-1266) and then XORed with the payload
    # (encryption_common_counter send.c:1273-1465) — two kernels, 4n algorithmic bytes
    "ctr1g_mask": ("ctrmask", 1 << 30, 1, "BASELINE config 4, materialised mask: 1 GiB keystream, then XOR"),
    "alltoall": ("gcm", 1 << 20, 8, "BASELINE config 5 per rank: 8 peers x 1 MiB seal+open"),
}


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


class Workload:
    """Device buffers + one step of the hot path for a workload."""

    def __init__(self, name: str, device: int, seed: int):
        self.name = name
        self.alg, self.n, self.nrec, self.desc = WORKLOADS[name]
        self.dev = torch.device("cuda", device)
        g = torch.Generator(device=self.dev).manual_seed(seed)
        n, N = self.n, self.nrec
        self.pt = torch.randint(0, 256, (N * n,), dtype=torch.uint8, device=self.dev, generator=g)
        if self.alg in ("ctr", "ctrmask"):
            self.ctx = aead.CipherCtx(KEY, "aes-128-ctr", device=device)
            self.ct = torch.empty_like(self.pt)
            self.mask = torch.empty_like(self.pt) if self.alg == "ctrmask" else None
            self.ctr0 = bytes(range(0xF0, 0x100))
            self.pt_sample = self.pt[: 1 << 24].clone()  # open writes the plaintext back in place
            self._bind()
            return
        self.ctx = aead.AeadCtx(KEY, "aes-128-gcm" if self.alg == "gcm" else "aes-128-ocb", device=device)
        self.nonces = torch.randint(0, 256, (N * 12,), dtype=torch.uint8, device=self.dev, generator=g)
        self.ct = torch.empty(N * (n + 16), dtype=torch.uint8, device=self.dev)
        self.back = torch.empty(N * n, dtype=torch.uint8, device=self.dev)
        self.status = torch.zeros(N, dtype=torch.int32, device=self.dev)
        ws = self.ctx.workspace_size(n, N)
        self.ws = torch.empty(max(ws, 16), dtype=torch.uint8, device=self.dev) if ws else None
        self._bind()

    # algorithmic HBM bytes per launch: seal/open 2n+28 per record, CTR fused 2n,
    # CTR with a materialised mask 4n (write mask; read mask + payload, write ct)
    def bytes_per_launch(self) -> int:
        if self.alg == "ctr":
            return 2 * self.n
        if self.alg == "ctrmask":
            return 4 * self.n
        return self.nrec * (2 * self.n + 28)

    def _bind(self):
        """Pre-built C-ABI calls (argument tuples converted once): a step enqueues in a few us,
        so the GPU never idles between launches and the HIP-event kernel times agree with
        rocprofv3's kernel durations."""
        from cryptmpi_2022_amd import _native as N

        L, h = N.lib(), self.ctx.handle
        st = ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)
        P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        if self.alg == "ctr":
            cb = (ctypes.c_uint8 * 16).from_buffer_copy(self.ctr0)
            self._seal_call = (L.cmpi_ctr_xor, (h, P(self.ct), P(self.pt), self.n, cb, st))
            self._open_call = (L.cmpi_ctr_xor, (h, P(self.pt), P(self.ct), self.n, cb, st))
            return
        if self.alg == "ctrmask":  # mask = E_K(ctr0 + i) (cmpi_ctr_keystream), then out = in ^ mask
            cb = (ctypes.c_uint8 * 16).from_buffer_copy(self.ctr0)
            ks = (L.cmpi_ctr_keystream, (h, P(self.mask), self.n // 16, cb, st))
            self._seal_call = [ks, (L.cmpi_xor_bytes, (P(self.ct), P(self.pt), P(self.mask), self.n, st))]
            self._open_call = [ks, (L.cmpi_xor_bytes, (P(self.pt), P(self.ct), P(self.mask), self.n, st))]
            return
        n, N_ = self.n, self.nrec
        seal = L.cmpi_gcm_seal_batch if self.alg == "gcm" else L.cmpi_ocb_seal_batch
        opn = L.cmpi_gcm_open_batch if self.alg == "gcm" else L.cmpi_ocb_open_batch
        self._seal_call = (seal, (h, P(self.ct), n + 16, P(self.pt), n, P(self.nonces), 12, n, N_, P(self.ws), st))
        self._open_call = (opn, (h, P(self.back), n, P(self.ct), n + 16, P(self.nonces), 12, n, N_, P(self.status),
                                 P(self.ws), st))

    @staticmethod
    def _run(calls):
        for fn, args in calls if isinstance(calls, list) else [calls]:
            rc = fn(*args)
            if rc:
                from cryptmpi_2022_amd import _native as N

                N.check(rc)

    def seal(self):
        self._run(self._seal_call)

    def open(self):
        self._run(self._open_call)

    def verify(self) -> bool:
        torch.cuda.synchronize(self.dev)
        if self.alg in ("ctr", "ctrmask"):  # ct != pt, and decrypting ct in place restored the plaintext
            return (not torch.equal(self.ct[: 1 << 24], self.pt_sample)) and torch.equal(self.pt[: 1 << 24], self.pt_sample)
        return bool((self.status == 1).all()) and torch.equal(self.back, self.pt)

    def parity_cpu(self) -> dict:
        """Independent check of the timed workload's output, outside the timed region: the bytes
        the GPU produced in the last timed step, compared with the system OpenSSL 3 EVP (the
        stand-in for the reference's BoringSSL, tools/cpu_baseline.c) on the same inputs.
        GCM/OCB: ct||tag of every record (gcm*, alltoall) or of 64 records spread over the batch
        (ocb1m), plus the GPU's open of OpenSSL's ct||tag (statuses, plaintext) with one forged
        record (status 0, zero-filled, aead.h:276-278).  CTR: the keystream XOR at stream offset 0,
        across the 2^32 carry of the counter's low word and at the end of the 1 GiB stream."""
        try:
            return parity_cpu(self)
        except Exception as e:  # report, never hide
            return {"parity_cpu": False, "error": repr(e)}

    def free(self):
        self.ctx.close()
        for a in ("_seal_call", "_open_call", "pt", "pt_sample", "ct", "back", "nonces", "status", "ws", "mask"):
            if hasattr(self, a):
                delattr(self, a)
        torch.cuda.empty_cache()


class OpenSSLRef:
    """tools/libcpu_baseline.so (system OpenSSL 3 EVP AES-128-GCM/OCB/CTR): the independent
    implementation the bench checks the GPU's bytes against (the reference's BoringSSL cannot be
    built here)."""

    def __init__(self):
        P, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        self.C = ctypes.CDLL(os.path.join(ROOT, "tools", "libcpu_baseline.so"))
        self.C.cb_aead_batch.argtypes = [I, I, P, P, P, S, P, S, I, ctypes.c_long, I]
        self.C.cb_aead_batch.restype = I
        self.C.cb_ctr.argtypes = [P, P, P, P, S, I]
        self.C.cb_ctr.restype = I
        self.threads = max(1, min(16, host_cpu_info()["usable"]))

    def aead(self, alg: str, dec: bool, nonces: np.ndarray, inp: np.ndarray, n: int, key: bytes = KEY):
        nrec = nonces.shape[0]
        nonces = np.ascontiguousarray(nonces, np.uint8)
        inp = np.ascontiguousarray(inp, np.uint8)
        out = np.zeros((nrec, n if dec else n + 16), np.uint8)
        bad = self.C.cb_aead_batch(2 if alg == "ocb" else 1, 1 if dec else 0, key, nonces.ctypes.data, inp.ctypes.data,
                                   inp.shape[1], out.ctypes.data, out.shape[1], n, nrec, self.threads)
        return out, bad

    def ctr(self, ctr0: bytes, inp: np.ndarray, key: bytes = KEY) -> np.ndarray:
        inp = np.ascontiguousarray(inp, np.uint8)
        out = np.empty_like(inp)
        cb = (ctypes.c_uint8 * 16).from_buffer_copy(ctr0)
        assert self.C.cb_ctr(key, cb, inp.ctypes.data, out.ctypes.data, inp.size, self.threads) == 0
        return out


def ctr_add(ctr0: bytes, k: int) -> bytes:
    """128-bit big-endian counter block + k (SP 800-38A / EVP_aes_128_ctr)."""
    return ((int.from_bytes(ctr0, "big") + k) % (1 << 128)).to_bytes(16, "big")


def gpu_open_check(w, ref: "OpenSSLRef", idx: np.ndarray, pt: np.ndarray, nn: np.ndarray, ct_ref: np.ndarray) -> bool:
    """The GPU's open of OpenSSL's ct||tag for the sampled records (one tag forged): statuses
    1 / 0, plaintext equal / zero-filled for the forged one (BoringSSL aead.h:276-278)."""
    k, n = len(idx), w.n
    forged = ct_ref.copy()
    forged[k // 2, n] ^= 0x01
    d_in = torch.from_numpy(forged.reshape(-1)).to(w.dev)
    d_n = torch.from_numpy(np.ascontiguousarray(nn).reshape(-1)).to(w.dev)
    d_out = torch.full((k * n,), 0xA5, dtype=torch.uint8, device=w.dev)
    st = torch.full((k,), 7, dtype=torch.int32, device=w.dev)
    ctx = w.ctx
    ws = ctx.workspace_size(n, k)
    d_ws = torch.empty(max(ws, 16), dtype=torch.uint8, device=w.dev) if ws else None
    fn = ctx.open_batch
    try:
        fn(d_out, d_in, d_n, n, k, status=st, workspace=d_ws)
    except Exception:
        pass  # a failed record raises after the launch (CMPI_EAUTH); the statuses tell which
    torch.cuda.synchronize(w.dev)
    got = d_out.view(k, n).cpu().numpy()
    sts = st.cpu().numpy()
    want_st = np.ones(k, np.int32)
    want_st[k // 2] = 0
    want = pt.copy()
    want[k // 2] = 0
    return bool(np.array_equal(sts, want_st) and np.array_equal(got, want))


def parity_cpu(w) -> dict:
    """See Workload.parity_cpu."""
    ref = OpenSSLRef()
    torch.cuda.synchronize(w.dev)
    n, N = w.n, w.nrec
    if w.alg in ("ctr", "ctrmask"):
        windows = {}
        span = 1 << 24  # 16 MiB windows
        lo = int.from_bytes(w.ctr0[12:], "big")
        carry_blk = (1 << 32) - lo  # first block whose low counter word wrapped
        offs = {"offset_0": 0, "across_2^32_carry": max(0, min(carry_blk * 16 - span // 2, n - span)), "end": n - span}
        ok = True
        for name, off in offs.items():
            off -= off % 16
            pt = w.pt[off: off + span].cpu().numpy()
            got = w.ct[off: off + span].cpu().numpy()
            want = ref.ctr(ctr_add(w.ctr0, off // 16), pt)
            eq = bool(np.array_equal(got, want))
            windows[name] = {"byte_offset": off, "bytes": span, "equal": eq}
            ok = ok and eq
        return {"parity_cpu": ok, "ref": "OpenSSL 3 EVP_aes_128_ctr", "ctr0": w.ctr0.hex(),
                "carry_block": carry_blk, "windows": windows}
    k = N if n * N <= (256 << 20) else 64  # every record, or 64 spread over the batch
    idx = np.linspace(0, N - 1, k).round().astype(np.int64) if k < N else np.arange(N)
    it = torch.from_numpy(idx).to(w.dev)
    pt = w.pt.view(N, n).index_select(0, it).cpu().numpy()
    nn = w.nonces.view(N, 12).index_select(0, it).cpu().numpy()
    got = w.ct.view(N, n + 16).index_select(0, it).cpu().numpy()
    want, bad = ref.aead(w.alg, False, nn, pt, n)
    seal_ok = bad == 0 and bool(np.array_equal(got, want))
    nbad = int((got != want).any(axis=1).sum())
    open_ok = gpu_open_check(w, ref, idx[: min(k, 256)], pt[:256], nn[:256], want[:256])
    return {"parity_cpu": seal_ok and open_ok, "ref": f"OpenSSL 3 EVP_aes_128_{w.alg}",
            "records_checked": int(k), "of": int(N), "seal_ct_tag_equal": seal_ok, "records_differing": nbad,
            "gpu_open_of_ref_ct_with_one_forged": open_ok}


# Secondary workloads (extras): enough warm-up for the clock to leave its idle state (10 steps
# after 3 warm-ups measured the 4 KiB GCM seal at 894 GiB/s, 100 steps after 10 at 1 033).
EXTRA_STEPS, EXTRA_WARMUP = 30, 10
WARMUP_S = float(os.environ.get("CMPI_BENCH_WARMUP_S", "0.5"))  # minimum seconds of untimed warm-up before the headline timed region


class KernelEvents:
    """HIP events recorded on the launch stream around every seal and open of the timed region,
    created with hipEventDisableSystemFence (the library's cmpi_debug_event_*): a default event
    (torch.cuda.Event) performs a system-scope fence — cache writeback + invalidate — that left a
    ~6 us bubble before each following launch (rocprofv3 kernel trace)."""

    def __init__(self, n: int):
        from cryptmpi_2022_amd import _native as N

        self.L = N.lib()
        self.ev = [self.L.cmpi_debug_event_new() for _ in range(n)]
        assert all(self.ev), "hipEventCreateWithFlags failed"

    def record(self, i: int, stream) -> None:
        assert self.L.cmpi_debug_event_record(self.ev[i], stream) == 0

    def ms(self, i: int, j: int) -> float:
        t = self.L.cmpi_debug_event_ms(self.ev[i], self.ev[j])
        assert t >= 0.0, "hipEventElapsedTime failed"
        return t

    def free(self) -> None:
        for e in self.ev:
            self.L.cmpi_debug_event_free(e)


class Pipeline:
    """Consecutive steps of a GCM/OCB workload on two streams: the seal of batch i+1 (stream S, the
    current stream) runs while the open of batch i (stream O) finishes — what two ranks' traffic
    looks like to one GPU.  Two buffer sets (ct, plaintext out, statuses, one workspace per stream);
    open i waits for seal i, and seal i+2 waits for open i before it reuses set i mod 2.  Every
    step still seals and opens its whole batch.  Fence-free HIP events (KernelEvents) order the
    streams through hipStreamWaitEvent."""

    def __init__(self, w: Workload):
        from cryptmpi_2022_amd import _native as N

        self.w, self.L = w, N.lib()
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.hip.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
        self.S = torch.cuda.current_stream(w.dev)
        self.O = torch.cuda.Stream(w.dev)
        n, N_, h = w.n, w.nrec, w.ctx.handle
        P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        s_ptr, o_ptr = ctypes.c_void_p(self.S.cuda_stream), ctypes.c_void_p(self.O.cuda_stream)
        seal = self.L.cmpi_gcm_seal_batch if w.alg == "gcm" else self.L.cmpi_ocb_seal_batch
        opn = self.L.cmpi_gcm_open_batch if w.alg == "gcm" else self.L.cmpi_ocb_open_batch
        ws_o = torch.empty_like(w.ws) if w.ws is not None else None
        self.bufs, self.calls = [], []
        for k in range(2):
            ct = w.ct if k == 0 else torch.empty_like(w.ct)
            back = w.back if k == 0 else torch.empty_like(w.back)
            st = w.status if k == 0 else torch.zeros_like(w.status)
            self.bufs.append((ct, back, st))
            self.calls.append(((seal, (h, P(ct), n + 16, P(w.pt), n, P(w.nonces), 12, n, N_, P(w.ws), s_ptr)),
                               (opn, (h, P(back), n, P(ct), n + 16, P(w.nonces), 12, n, N_, P(st), P(ws_o), o_ptr))))
        self.ev = KernelEvents(4)  # seal done / open done, per set
        self.i = 0

    def _wait(self, stream, ev_idx: int) -> None:
        assert self.hip.hipStreamWaitEvent(ctypes.c_void_p(stream.cuda_stream), ctypes.c_void_p(self.ev.ev[ev_idx]), 0) == 0

    def step(self) -> None:
        k = self.i & 1
        if self.i >= 2:
            self._wait(self.S, 2 + k)  # open of the step that last used set k is done
        (sf, sa), (of, oa) = self.calls[k]
        assert sf(*sa) == 0
        self.ev.record(k, self.S.cuda_stream)
        self._wait(self.O, k)
        assert of(*oa) == 0
        self.ev.record(2 + k, self.O.cuda_stream)
        self.i += 1

    def verify(self) -> bool:
        torch.cuda.synchronize(self.w.dev)
        return all(bool((st == 1).all()) and torch.equal(back, self.w.pt) for _, back, st in self.bufs[: min(self.i, 2)])

    def free(self) -> None:
        torch.cuda.synchronize(self.w.dev)
        self.ev.free()
        self.bufs, self.calls = [], []


def time_steps_pipelined(w: Workload, steps: int, warmup: int, barrier, warmup_s: float = 0.0) -> tuple[float, bool]:
    """Wall seconds for `steps` pipelined steps (Pipeline) after the warm-up, and whether every
    buffer set's last open restored the plaintext with all statuses 1."""
    p = Pipeline(w)
    t_w = time.perf_counter()
    i = 0
    while i < warmup or time.perf_counter() - t_w < warmup_s:
        p.step()
        i += 1
        if i % 8 == 0:
            torch.cuda.synchronize(w.dev)
    ok = p.verify()
    barrier()
    torch.cuda.synchronize(w.dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        p.step()
    torch.cuda.synchronize(w.dev)
    barrier()
    wall = time.perf_counter() - t0
    ok = ok and p.verify()
    p.free()
    return wall, ok


def time_steps(w: Workload, steps: int, warmup: int, barrier, warmup_s: float = 0.0, detail: dict | None = None):
    """Returns (wall seconds for `steps` steps, avg seal kernel ms, avg open kernel ms).

    The timed region: `steps` steps, each sealing then opening the whole batch on one stream, with
    fence-free HIP events (KernelEvents) recorded on that stream between the launches — its wall
    clock is the headline; each launch's stream bracket (the kernel plus the dependent launch's
    dispatch gap after the previous kernel; seal + open brackets = the step) goes into `detail`.
    Kernel times: right after it, the same `steps` steps again with every seal and open launched
    through hipExtLaunchKernel with start / stop events (cmpi_debug_time_next_launch) — the
    kernel's own execution, what rocprofv3 --kernel-trace reports.  They are a pass of their own
    because those events widen each launch's dispatch gap (config 2: ~4 us per launch, ~6 % of a
    step, profiles/r06c_*), which the headline must not carry.  The warm-up is `warmup` steps and,
    when warmup_s > 0, at least that many seconds of them (the extras run after the CPU baseline
    has left the GPU idle for seconds: clocks ramp back up first)."""
    t_w = time.perf_counter()
    i = 0
    while i < warmup or time.perf_counter() - t_w < warmup_s:
        w.seal()
        w.open()
        i += 1
        if warmup_s and i % 8 == 0:
            torch.cuda.synchronize(w.dev)
    torch.cuda.synchronize(w.dev)
    assert w.verify(), "round trip failed in warm-up"
    stream = torch.cuda.current_stream(w.dev).cuda_stream
    ev = KernelEvents(2 * steps + 1)
    barrier()
    torch.cuda.synchronize(w.dev)
    t0 = time.perf_counter()
    ev.record(0, stream)
    for i in range(steps):
        w.seal()
        ev.record(2 * i + 1, stream)
        w.open()
        ev.record(2 * i + 2, stream)
    torch.cuda.synchronize(w.dev)
    barrier()
    wall = time.perf_counter() - t0
    seal_br = sum(ev.ms(2 * i, 2 * i + 1) for i in range(steps)) / steps
    open_br = sum(ev.ms(2 * i + 1, 2 * i + 2) for i in range(steps)) / steps
    ev.free()
    if os.environ.get("CMPI_BENCH_NO_KPASS") == "1":  # diagnostics: stream brackets only
        if detail is not None:
            detail["seal_ms_stream_bracket"], detail["open_ms_stream_bracket"] = seal_br, open_br
        return wall, seal_br, open_br
    # kernel-timing pass (outside the timed region)
    kev = KernelEvents(4 * steps)  # per launch: the kernel's start, stop
    timed = kev.L.cmpi_debug_time_next_launch
    for i in range(steps):
        timed(kev.ev[4 * i], kev.ev[4 * i + 1])
        w.seal()
        timed(kev.ev[4 * i + 2], kev.ev[4 * i + 3])
        w.open()
    timed(None, None)
    torch.cuda.synchronize(w.dev)
    seal_ms = sum(kev.ms(4 * i, 4 * i + 1) for i in range(steps)) / steps
    open_ms = sum(kev.ms(4 * i + 2, 4 * i + 3) for i in range(steps)) / steps
    kev.free()
    if detail is not None:
        detail["seal_ms_stream_bracket"] = seal_br
        detail["open_ms_stream_bracket"] = open_br
    return wall, seal_ms, open_ms


def aggregate(wall: float, per_rank_bytes: int, steps: int, pg, device) -> tuple[float, float]:
    """Whole-job rate: the slowest rank's timed wall clock (MAX over ranks) and the bytes all
    ranks processed in it, GiB/s (weak scaling: every rank has the same per-rank batch)."""
    t = torch.tensor([wall], dtype=torch.float64, device=device)
    ws = 1
    if pg is not None:
        pg.all_reduce(t, op=pg.ReduceOp.MAX)
        ws = pg.get_world_size()
    wall_max = float(t.item())
    return wall_max, per_rank_bytes * ws * steps / wall_max / GIB


# The binding on-chip resource of the GCM kernels is the LDS array (DESIGN.md "Roofline"): per
# 16-B counter block 133 ds_read_b32 T-table lookups (rounds 1-2 counter-cached: 1 + 4, rounds 3-9
# 7 x 16, last 16) at 2 LDS cycles per wave-instruction, and per GHASH block 16 ds_read_b128
# byte-table lookups at 4 (MI355X_MICROARCH.md "LDS": 64 banks, lane groups per instruction).
LDS_CLK_HZ = 2.4e9  # MI355X peak engine clock
AES_B32_LOOKUPS, GHASH_B128_LOOKUPS = 133, 16


def lds_roofline(w, kern_ms: float, device: int) -> dict:
    """LDS-array cycles the GCM seal launch needs at minimum (AES of nb data blocks + J0, GHASH of
    nb blocks + the length block, per record) against ncu x clock x kernel time."""
    import torch

    ncu = torch.cuda.get_device_properties(device).multi_processor_count
    nb = (w.n + 15) // 16
    per_block = (AES_B32_LOOKUPS * 2 + GHASH_B128_LOOKUPS * 4) / 64.0  # LDS cycles per block per CU
    cycles = w.nrec * (nb + 1) * per_block
    avail = kern_ms * 1e-3 * ncu * LDS_CLK_HZ
    return {"bound": "lds", "unit": "Gblock/s", "cycles_per_block": round(per_block, 3),
            "achieved": round(w.nrec * (nb + 1) / (kern_ms * 1e-3) / 1e9, 2),
            "peak": round(ncu * LDS_CLK_HZ / per_block / 1e9, 2), "frac": round(cycles / avail, 4),
            "note": "AES 133 ds_read_b32 + GHASH 16 ds_read_b128 per 16-B block; J0 and length block counted"}


def copy_peak_gbs(device: int, nbytes: int = 1 << 30, reps: int = 10) -> float:
    """Achievable HBM bandwidth on this box: device-to-device copy of 1 GiB by the library's
    streaming copy kernel (cmpi_debug_copy: 16 B per lane, grid-stride, 4 workgroups per CU — the
    fastest of 80 forms swept in round 5, 5.6-5.7 TB/s, profiles/r05u_copy_probe2.jsonl; the
    guide's float4 copy measures 6.29 TB/s) — read + write bytes / time, best of `reps` — the
    'measured copy-kernel peak' of BASELINE.md §3.  (Round 4 timed a torch uint8 copy_, 4.9 TB/s,
    which overstated frac_measured.)"""
    from cryptmpi_2022_amd import _native as N

    src = torch.empty(nbytes, dtype=torch.uint8, device=torch.device("cuda", device))
    dst = torch.empty_like(src)
    st = torch.cuda.current_stream(device).cuda_stream
    lib = N.lib()

    def copy():
        N.check(lib.cmpi_debug_copy(dst.data_ptr(), src.data_ptr(), nbytes, st))

    copy()
    torch.cuda.synchronize(device)
    best = float("inf")
    ev = KernelEvents(2)
    for _ in range(reps):
        ev.record(0, st)
        copy()
        ev.record(1, st)
        torch.cuda.synchronize(device)
        best = min(best, ev.ms(0, 1) * 1e-3)
    ev.free()
    del src, dst
    torch.cuda.empty_cache()
    return 2 * nbytes / best / 1e9


def registered_host_buffer(nbytes: int) -> torch.Tensor:
    """Page-locked host memory the way an MPI library registers a user buffer: anonymous memory,
    2 MiB aligned, transparent huge pages requested (madvise MADV_HUGEPAGE), then hipHostRegister.
    (torch pin_memory buffers DMA at the same peak but vary with the process's allocation history:
    23-33 GiB/s for the pipelined seal in round-3 benches, tools/host_regress_probe.py.)  The
    mapping lives as long as the process."""
    libc = ctypes.CDLL(None)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    raw = libc.mmap(None, nbytes + (2 << 20), 3, 0x22, -1, 0)  # PROT_READ|WRITE, MAP_PRIVATE|ANONYMOUS
    if raw in (None, ctypes.c_void_p(-1).value):
        raise OSError("mmap failed")
    base = (raw + (2 << 20) - 1) & ~((2 << 20) - 1)
    libc.madvise(ctypes.c_void_p(base), nbytes, 14)  # MADV_HUGEPAGE (advice only)
    a = np.frombuffer((ctypes.c_uint8 * nbytes).from_address(base), dtype=np.uint8)
    a[:] = 0  # fault the pages in
    from cryptmpi_2022_amd import _native as N

    N.check(N.lib().cmpi_host_register(ctypes.c_void_p(base), nbytes))
    return torch.from_numpy(a)


def host_path_rate(device: int, n: int = 1024, nrec: int = 65536) -> dict:
    """PCIe-inclusive seal rates (the path starts and ends in host memory, BASELINE north_star):
    (a) pinned host -> H2D -> kernel -> D2H -> pinned host serialised on one stream;
    (b) the library's host entry point cmpi_gcm_seal_host on page-locked buffers registered as an
        MPI library registers user memory (registered_host_buffer; chunked 3-stream pipeline,
        H2D / kernel / D2H overlapped), and the same on torch pin_memory buffers; (c) pageable."""
    from cryptmpi_2022_amd import _native as N

    pt = registered_host_buffer(nrec * n)
    pt.copy_(torch.randint(0, 256, (nrec * n,), dtype=torch.uint8))
    nonces = registered_host_buffer(nrec * 12)
    nonces.copy_(torch.randint(0, 256, (nrec * 12,), dtype=torch.uint8))
    out = registered_host_buffer(nrec * (n + 16))
    tp_pt, tp_n, tp_out = pt.clone().pin_memory(), nonces.clone().pin_memory(), out.clone().pin_memory()
    ctx = aead.AeadCtx(KEY, device=device)
    d_pt = torch.empty(nrec * n, dtype=torch.uint8, device=f"cuda:{device}")
    d_n = torch.empty(nrec * 12, dtype=torch.uint8, device=f"cuda:{device}")
    d_ct = torch.empty(nrec * (n + 16), dtype=torch.uint8, device=f"cuda:{device}")

    def serial():
        d_pt.copy_(pt, non_blocking=True)
        d_n.copy_(nonces, non_blocking=True)
        ctx.seal_batch(d_ct, d_pt, d_n, n, nrec)
        out.copy_(d_ct, non_blocking=True)
        torch.cuda.synchronize()

    L, h = N.lib(), ctx.handle
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def host_api(src, dst, nn):
        N.check(L.cmpi_gcm_seal_host(h, P(dst), n + 16, P(src), n, P(nn), 12, n, nrec))

    pg_pt = torch.randint(0, 256, (nrec * n,), dtype=torch.uint8)  # pageable
    pg_n = torch.randint(0, 256, (nrec * 12,), dtype=torch.uint8)
    pg_out = torch.empty(nrec * (n + 16), dtype=torch.uint8)

    def rate(fn, reps=8, warm=3):
        for _ in range(warm):  # the first calls of a process run far slower (21 vs 31 GiB/s pinned)
            fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return nrec * n / ((time.perf_counter() - t0) / reps) / GIB

    back = registered_host_buffer(nrec * n)
    st = (ctypes.c_int32 * nrec)()

    def host_open():
        N.check(L.cmpi_gcm_open_host(h, P(back), n, P(out), n + 16, P(nonces), 12, n, nrec, st))

    def hip_copies():  # the copy mode of rounds 4-5 (hipMemcpyAsync both ways, 16 MiB chunks)
        L.cmpi_debug_set_host_out_direct(0)
        L.cmpi_debug_set_host_chunk(16 << 20)
        try:
            return round(rate(lambda: host_api(pt, out, nonces)), 2)
        finally:
            L.cmpi_debug_set_host_out_direct(5)
            L.cmpi_debug_set_host_chunk(0)

    res = {"config": f"{nrec} x {n} B GCM seal, host buffers in and out",
           "pinned_serial_1stream_GiBps": round(rate(serial), 2),
           "host_api_pinned_pipelined_GiBps": round(rate(lambda: host_api(pt, out, nonces)), 2),
           "host_api_pinned_open_GiBps": round(rate(host_open), 2),
           "host_api_torch_pin_pipelined_GiBps": round(rate(lambda: host_api(tp_pt, tp_out, tp_n)), 2),
           "host_api_pageable_GiBps": round(rate(lambda: host_api(pg_pt, pg_out, pg_n), 4), 2),
           "host_api_pinned_hip_copies_GiBps": hip_copies(),
           "pinned_buffers": "registered_host_buffer (2 MiB aligned, MADV_HUGEPAGE, cmpi_host_register)",
           "copy_mode": "both directions on SDMA through HSA, host-launched kernels (cmpi_debug_set_host_out_direct 5); "
                        "hip_copies: hipMemcpyAsync both ways (mode 0)"}
    host_api(pt, out, nonces)
    host_open()
    res["round_trip"] = bool(torch.equal(back, pt)) and all(x == 1 for x in st)
    ctx.close()
    return res


def host602_rate(device: int, n: int = 8 << 20, reps: int = 8) -> dict:
    """The 602 8 MiB message (mode '1': 16 outer messages of 512 KiB, 128 segments of 64 KiB,
    per-message sub-key K' = AES_K(V) derived on the device) sealed from and opened into
    page-locked host memory (registered_host_buffer), send.c:729-850 / recv.c:679-809:
      seal_per_outer   one cmpi_602_seal_host_begin per outer message, all begun before the first
                       wait (the reference seals outer k+1 while MPI_Isend of k is in flight);
      seal_whole       the synchronous cmpi_602_seal_host of the whole message;
      open_per_outer   one cmpi_602_open_host_begin per outer message, waited in order.
    Best of `reps` after 3 warm-ups.  The wire is then checked against OpenSSL 3 (K' from
    EVP_aes_128_ctr over V, every segment's GCM under "0000000"||flag||BE32(ctr)) and opened back."""
    from cryptmpi_2022_amd import frame

    plan = frame.plan602(n, 8, 0)
    rand16 = bytes(range(16, 32))
    header = frame.header602(plan, rand16)
    master = aead.AeadCtx(KEY, device=device)
    seg = aead.AeadCtx(bytes(16), device=device)
    seg.rekey_subkey(master, header[4:20], stream=torch.cuda.current_stream(device))
    torch.cuda.synchronize(device)
    src = registered_host_buffer(n).numpy()
    src[:] = np.random.default_rng(602).integers(0, 256, n, dtype=np.uint8)
    wire = registered_host_buffer(plan.wire_bytes).numpy()
    back = registered_host_buffer(n).numpy()

    def seal_per_outer():
        reqs = [frame.seal602_host_begin(seg, plan, header, wire, src, o) for o in range(plan.outer)]
        for q in reqs:
            q.wait()

    def seal_whole():
        frame.seal602_host(seg, plan, header, wire, src)

    def open_per_outer():
        reqs = [frame.open602_host_begin(seg, header, back, wire, o) for o in range(plan.outer)]
        for q in reqs:
            q.wait()

    res = {"message_bytes": n, "plan": plan.as_dict(), "buffers": "registered_host_buffer (page-locked)"}
    for name, fn in (("seal_per_outer", seal_per_outer), ("seal_whole", seal_whole), ("open_per_outer", open_per_outer)):
        for _ in range(3):
            fn()
        best = float("inf")
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            best = min(best, time.perf_counter() - t0)
        res[name + "_GiBps"] = round(n / best / GIB, 2)
    res["round_trip"] = bool(np.array_equal(back, src))
    try:  # independent check of the wire: OpenSSL under K' = AES_K(V)
        ref = OpenSSLRef()
        kp = ref.ctr(header[4:20], np.zeros(16, np.uint8)).tobytes()
        seg_len, nseg = plan.chop, plan.nseg
        w = wire[: nseg * (seg_len + 21)].reshape(nseg, seg_len + 21)
        nonces = np.concatenate([np.frombuffer(b"0000000", np.uint8)[None, :].repeat(nseg, 0), w[:, :5]], axis=1)
        want, bad = ref.aead("gcm", False, nonces, src.reshape(nseg, seg_len), seg_len, key=kp)
        res["parity_cpu"] = bad == 0 and bool(np.array_equal(w[:, 5:], want)) and plan.total == nseg * seg_len
    except Exception as e:  # report, never hide
        res["parity_cpu"] = {"error": repr(e)}
    res["parity"] = "every segment's prefix-nonce, ciphertext and tag vs OpenSSL 3 under K' = AES_K(V)"
    seg.close()
    master.close()
    return res


A2A_BLOCKS = 8  # BASELINE config 5: 8 ranks, so every rank seals 8 peer blocks of 1 MiB per call


def _peer_send(dev, rank: int, nblk: int, n: int):
    """alltoall_e2e's send buffer of `rank` (seeded per rank: any rank can rebuild a peer's)."""
    g = torch.Generator(device=dev).manual_seed(4242 + rank)
    return torch.randint(0, 256, (nblk * n,), dtype=torch.uint8, device=dev, generator=g)


def alltoall_e2e(device: int, pg, barrier, n: int = 1 << 20, steps: int = 100, warmup: int = 10,
                 warmup_s: float = 0.3) -> dict:
    """BASELINE config 5 end to end, MPIR_Naive_Sec_Alltoall (alltoall.c:764-836) per rank:
    seal the rank's 8 peer blocks (config 5's p = 8) with fresh nonces into the wire layout
    nonce||ct||tag (one batched call), exchange the wire blocks, open the 8 received blocks (one
    batched call), on one stream.  Transport: RCCL all_to_all_single over xGMI (backend "nccl");
    with a "gloo" group (ranks sharing one GPU, tests/test_gpu_alltoall8.py) the wire blocks go
    through page-locked host memory, as a host MPI would carry them; one rank loops them back
    through a device copy.  With fewer than 8 ranks each peer gets 8/ranks consecutive blocks.
    The per-rank seal/open work is config 5's at every rank count.  Every rank runs this;
    time = MAX over ranks; rate = plaintext bytes each rank sent / time.  After the timed calls
    every rank checks that it received exactly its peers' plaintext (every block authenticated).
    Warm-up: `warmup_s` seconds of the rank's own seal + loopback + open (no collective, so the
    ranks need not agree on a count; the clocks leave the state the CPU-side parity checks of the
    preceding extras left them in: 47.2 -> 44.7 us per call over the first seconds of calls,
    profiles/r05as_e2e_warmup.txt), then `warmup` whole calls."""
    from cryptmpi_2022_amd import _native as N

    p = pg.get_world_size() if pg is not None else 1
    rank = pg.get_rank() if pg is not None else 0
    host = p > 1 and pg.get_backend() == "gloo"
    nblk = -(-A2A_BLOCKS // p) * p  # a multiple of the rank count (8 for 1, 2, 4, 8 ranks)
    dev = torch.device("cuda", device)
    send = _peer_send(dev, rank, nblk, n)
    recv = torch.empty_like(send)
    wire = torch.empty(nblk * (n + 28), dtype=torch.uint8, device=dev)
    wire_in = torch.empty_like(wire)
    h_out = torch.empty(wire.numel(), dtype=torch.uint8).pin_memory() if host else None
    h_in = torch.empty_like(h_out).pin_memory() if host else None
    status = torch.zeros(nblk, dtype=torch.int32, device=dev)
    ctx = aead.AeadCtx(KEY, device=device)
    ws_bytes = max(ctx.workspace_size(n, nblk), 16)
    ws_seal = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    ws_open = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    L = N.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def one():
        N.check(L.cmpi_naive_seal_blocks(ctx.handle, P(wire), P(send), n, nblk, P(ws_seal), st))
        if host:
            h_out.copy_(wire)  # synchronous: the seal is done when the host sends
            pg.all_to_all_single(h_in, h_out)
            wire_in.copy_(h_in, non_blocking=True)
        elif p > 1:
            pg.all_to_all_single(wire_in, wire)
        else:
            wire_in.copy_(wire)
        N.check(L.cmpi_naive_open_blocks(ctx.handle, P(recv), P(wire_in), n, nblk, P(status), P(ws_open), st))

    t_end = time.perf_counter() + warmup_s
    while time.perf_counter() < t_end:
        for _ in range(20):
            N.check(L.cmpi_naive_seal_blocks(ctx.handle, P(wire), P(send), n, nblk, P(ws_seal), st))
            wire_in.copy_(wire)
            N.check(L.cmpi_naive_open_blocks(ctx.handle, P(recv), P(wire_in), n, nblk, P(status), P(ws_open), st))
        torch.cuda.synchronize(dev)
    for _ in range(warmup):
        one()
    torch.cuda.synchronize(dev)
    ok = bool((status == 1).all())
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize(dev)
    barrier()
    wall = time.perf_counter() - t0
    # outside the timed region: every block authenticated, and this rank received exactly its
    # peers' plaintext (chunk `rank` of every peer's send buffer, rebuilt from the peer's seed)
    ok = ok and bool((status == 1).all())
    v = nblk // p
    want = torch.cat([_peer_send(dev, j, nblk, n)[rank * v * n:(rank + 1) * v * n] for j in range(p)])
    peers_ok = bool(torch.equal(recv, want))
    # parity (outside the timed region): this rank's wire blocks of the last call, nonce||ct||tag,
    # against OpenSSL's seal of the same blocks under the nonces the wire carries
    try:
        wv = wire.view(nblk, n + 28).cpu().numpy()
        want_ct, bad = OpenSSLRef().aead("gcm", False, wv[:, :12], send.view(nblk, n).cpu().numpy(), n)
        par = bad == 0 and bool(np.array_equal(wv[:, 12:], want_ct))
    except Exception:
        par = False
    if p > 1:  # MAX of the wall clocks, MIN of the verdicts (host tensors over gloo)
        rdev = torch.device("cpu") if host else dev
        t = torch.tensor([wall], dtype=torch.float64, device=rdev)
        pg.all_reduce(t, op=pg.ReduceOp.MAX)
        okt = torch.tensor([int(ok), int(par), int(peers_ok)], dtype=torch.int32, device=rdev)
        pg.all_reduce(okt, op=pg.ReduceOp.MIN)
        wall = float(t.item())
        ok, par, peers_ok = (bool(x) for x in okt.tolist())
    ctx.close()
    transport = ("gloo all_to_all_single through page-locked host memory" if host else
                 "RCCL all_to_all_single (xGMI)" if p > 1 else "1 rank: device copy (blocks looped back)")
    return {"ranks": p, "blocks_per_rank": nblk, "block_bytes": n, "ms_per_call": round(wall / steps * 1e3, 4),
            "GiBps_per_rank": round(nblk * n * steps / wall / GIB, 2),
            "GiBps_all_ranks": round(p * nblk * n * steps / wall / GIB, 2),
            "transport": transport, "all_blocks_authenticated": ok, "recv_matches_peers": peers_ok,
            "parity_cpu": par,
            "parity": "every rank's wire blocks (nonce||ct||tag) vs OpenSSL 3 EVP_aes_128_gcm seal under the wire nonces"}


def naive_collectives_e2e(device: int, pg, barrier, n: int = 1 << 20, steps: int = 20, warmup: int = 3,
                          warmup_s: float = 0.1) -> dict:
    """The other naive secure collectives end to end at config 5's shape (p = 8 peers of 1 MiB;
    with fewer than 8 ranks each rank stands for 8/ranks of them, as alltoall_e2e): per call,
    one batched seal and one batched open per rank around the stock collective on the wire blocks
    (RCCL over xGMI; one rank: a device copy).  Root 0.
      allgather  MPIR_Naive_Sec_Allgather (allgather.c:839-899): seal own blocks, all-gather, open 8
      gather     approach 301 (gather.c:1508-1606): seal own blocks, gather to the root, root opens 8
      scatter    MPIR_Naive_Sec_Scatter (scatter.c:659-730): root seals 8, scatter, open own blocks
      bcast      MPI_Naive_Sec_Bcast (bcast.c:1510-1580): root seals 1, broadcast, the others open it
                 (one rank: it opens its own block)
    Every rank runs this; time = MAX over ranks; statuses checked after the timed calls.  Before
    each collective: `warmup_s` seconds of the rank's own batched seal + open (no collective: the
    clocks' warm-up, as alltoall_e2e), then `warmup` whole calls."""
    from cryptmpi_2022_amd import _native as N

    p = pg.get_world_size() if pg is not None else 1
    rank = pg.get_rank() if pg is not None else 0
    v = -(-A2A_BLOCKS // p)  # blocks this rank stands for
    tot = v * p
    w = n + 28
    dev = torch.device("cuda", device)
    g = torch.Generator(device=dev).manual_seed(5151 + rank)
    send = torch.randint(0, 256, (tot * n,), dtype=torch.uint8, device=dev, generator=g)
    recv = torch.empty_like(send)
    wire_mine = torch.empty(v * w, dtype=torch.uint8, device=dev)
    wire_all = torch.empty(tot * w, dtype=torch.uint8, device=dev)
    status = torch.zeros(tot, dtype=torch.int32, device=dev)
    ctx = aead.AeadCtx(KEY, device=device)
    ws = torch.empty(max(ctx.workspace_size(n, tot), 16), dtype=torch.uint8, device=dev)
    L = N.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def seal(wire, src, k):
        N.check(L.cmpi_naive_seal_blocks(ctx.handle, P(wire), P(src), n, k, P(ws), st))

    def opn(dst, wire, k):
        N.check(L.cmpi_naive_open_blocks(ctx.handle, P(dst), P(wire), n, k, P(status), P(ws), st))

    def allgather():
        seal(wire_mine, send, v)
        if p > 1:
            pg.all_gather_into_tensor(wire_all, wire_mine)
        else:
            wire_all.copy_(wire_mine)
        opn(recv, wire_all, tot)
        return tot

    def gather():
        seal(wire_mine, send, v)
        if p > 1:
            parts = list(wire_all.split(v * w)) if rank == 0 else None
            pg.gather(wire_mine, parts, dst=0)
        else:
            wire_all.copy_(wire_mine)
        if rank == 0:
            opn(recv, wire_all, tot)
            return tot
        return 0

    def scatter():
        if rank == 0:
            seal(wire_all, send, tot)
        if p > 1:
            pg.scatter(wire_mine, list(wire_all.split(v * w)) if rank == 0 else None, src=0)
        else:
            wire_mine.copy_(wire_all)
        opn(recv, wire_mine, v)
        return v

    def bcast():
        if rank == 0:
            seal(wire_mine, send, 1)
        if p > 1:
            pg.broadcast(wire_mine[:w], src=0)
        if rank != 0 or p == 1:
            opn(recv, wire_mine, 1)
            return 1
        return 0

    res = {"ranks": p, "block_bytes": n, "peers": tot, "root": 0,
           "transport": "RCCL (xGMI)" if p > 1 else "1 rank: device copy (blocks looped back)"}
    for name, fn in (("allgather", allgather), ("gather", gather), ("scatter", scatter), ("bcast", bcast)):
        t_end = time.perf_counter() + warmup_s
        while time.perf_counter() < t_end:
            for _ in range(20):
                seal(wire_all, send, tot)
                opn(recv, wire_all, tot)
            torch.cuda.synchronize(dev)
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize(dev)
        status.zero_()
        barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        k = 0
        for _ in range(steps):
            k = fn()
        torch.cuda.synchronize(dev)
        barrier()
        wall = time.perf_counter() - t0
        ok = bool((status[:k] == 1).all()) if k else True
        if p == 1 and k:
            ok = ok and torch.equal(recv[: k * n], send[: k * n])
        t = torch.tensor([wall], dtype=torch.float64, device=dev)
        okt = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        if p > 1:
            pg.all_reduce(t, op=pg.ReduceOp.MAX)
            pg.all_reduce(okt, op=pg.ReduceOp.MIN)
        res[name] = {"ms_per_call": round(float(t.item()) / steps * 1e3, 4), "blocks_opened_per_rank": k,
                     "all_blocks_authenticated": bool(okt.item())}
    ctx.close()
    return res


def config1_message(device: int, n: int = 64 << 10, iters: int = 200) -> dict:
    """BASELINE config 1's unit of work (one 64 KiB MPI_Send/MPI_Recv message, 600 framing:
    send.c:221-337 / recv.c:219-341) on this engine: per-message seal + open latency
    (a) device-resident (cmpi_600_seal / cmpi_600_open, fence-free events) and (b) host-inclusive
    from pinned memory (H2D + seal + D2H, H2D + open + D2H, synchronised per message as MPI would),
    next to (c) OpenSSL AES-NI on one host core for the same message (the reference seals per
    message on the CPU).  Small single messages are latency-bound on the GPU; batching is the
    lever (config 2)."""
    from cryptmpi_2022_amd import _native as N

    dev = torch.device("cuda", device)
    L = N.lib()
    ctx = aead.AeadCtx(KEY, device=device)
    st = torch.cuda.current_stream(dev).cuda_stream
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    msg = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev)
    payload = torch.empty(n + 28, dtype=torch.uint8, device=dev)
    back = torch.empty(n, dtype=torch.uint8, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    nonce_buf = (ctypes.c_uint8 * 12)(*range(12))
    nonce = ctypes.cast(nonce_buf, ctypes.c_void_p)
    h_msg = msg.cpu().pin_memory()
    h_payload = torch.empty(n + 28, dtype=torch.uint8).pin_memory()
    h_back = torch.empty(n, dtype=torch.uint8).pin_memory()

    def seal():
        N.check(L.cmpi_600_seal(ctx.handle, nonce, P(payload), P(msg), n, ctypes.c_void_p(st)))

    def opn():
        N.check(L.cmpi_600_open(ctx.handle, P(back), P(payload), n, P(status), ctypes.c_void_p(st)))

    for _ in range(20):
        seal()
        opn()
    torch.cuda.synchronize(dev)
    ev = KernelEvents(2 * iters + 1)
    ev.record(0, st)
    for i in range(iters):
        seal()
        ev.record(2 * i + 1, st)
        opn()
        ev.record(2 * i + 2, st)
    torch.cuda.synchronize(dev)
    seal_us = sum(ev.ms(2 * i, 2 * i + 1) for i in range(iters)) / iters * 1e3
    open_us = sum(ev.ms(2 * i + 1, 2 * i + 2) for i in range(iters)) / iters * 1e3
    ev.free()
    ok = bool(status.item() == 1) and torch.equal(back, msg)

    def host_msg():
        msg.copy_(h_msg, non_blocking=True)
        seal()
        h_payload.copy_(payload, non_blocking=True)
        torch.cuda.synchronize(dev)  # MPI_Send of the payload would start here
        payload.copy_(h_payload, non_blocking=True)
        opn()
        h_back.copy_(back, non_blocking=True)
        torch.cuda.synchronize(dev)

    for _ in range(20):
        host_msg()
    t0 = time.perf_counter()
    for _ in range(iters):
        host_msg()
    host_us = (time.perf_counter() - t0) / iters * 1e6
    ok = ok and torch.equal(h_back, h_msg)
    # the engine's own host-memory calls (what the EVP drop-in and p2p.Endpoint run per message):
    # up to 2 MiB the direct path — the kernel reads and writes the page-locked buffers itself
    h_ct = torch.empty(n + 16, dtype=torch.uint8).pin_memory()
    h_st = np.zeros(1, np.int32)
    api_us = {}
    for kind, (src, ctb, dst) in {"pinned": (h_msg, h_ct, h_back),
                                  "pageable": (h_msg.clone(), torch.empty(n + 16, dtype=torch.uint8),
                                               torch.empty(n, dtype=torch.uint8))}.items():
        def host_api():
            N.check(L.cmpi_gcm_seal_host(ctx.handle, P(ctb), n + 16, P(src), n, nonce, 12, n, 1))
            N.check(L.cmpi_gcm_open_host(ctx.handle, P(dst), n, P(ctb), n + 16, nonce, 12, n, 1,
                                         ctypes.c_void_p(h_st.ctypes.data)))

        dst.zero_()
        for _ in range(20):
            host_api()
        t0 = time.perf_counter()
        for _ in range(iters):
            host_api()
        api_us[kind] = round((time.perf_counter() - t0) / iters * 1e6, 2)
        ok = ok and torch.equal(dst, src) and int(h_st[0]) == 1
        # the same calls served by the resident message service (include/cmpi_service.h, opt-in)
        ctx.service_start(0)
        dst.zero_()
        for _ in range(20):
            host_api()
        t0 = time.perf_counter()
        for _ in range(iters):
            host_api()
        api_us["service_" + kind] = round((time.perf_counter() - t0) / iters * 1e6, 2)
        ok = ok and torch.equal(dst, src) and int(h_st[0]) == 1 and ctx.service_running()
        ctx.service_stop()
    res = {"message_bytes": n, "framing": "600 (nonce||ct||tag, 25-byte header on the host)",
           "device_seal_us": round(seal_us, 2), "device_open_us": round(open_us, 2),
           "host_pinned_seal_open_us": round(host_us, 2),
           "host_api_seal_open_us": api_us,
           "host_api_note": "pinned / pageable: one kernel launch per call (direct path); service_*: "
                            "messages posted to the resident service kernel (cmpi_service_start)",
           "verified": ok}
    try:
        C = ctypes.CDLL(os.path.join(ROOT, "tools", "libcpu_baseline.so"))
        Pc, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        C.cb_aead_batch.argtypes = [I, I, Pc, Pc, Pc, S, Pc, S, I, ctypes.c_long, I]
        pt = h_msg.numpy().copy()
        ct = np.empty(n + 16, np.uint8)
        bk = np.empty(n, np.uint8)
        nn = np.frombuffer(bytes(range(12)), np.uint8).copy()
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 0.5:
            C.cb_aead_batch(1, 0, KEY, nn.ctypes.data, pt.ctypes.data, n, ct.ctypes.data, n + 16, n, 1, 1)
            assert C.cb_aead_batch(1, 1, KEY, nn.ctypes.data, ct.ctypes.data, n + 16, bk.ctypes.data, n, n, 1, 1) == 0
            reps += 1
        res["openssl_1core_seal_open_us"] = round((time.perf_counter() - t0) / reps * 1e6, 2)
    except OSError as e:
        res["openssl_1core_seal_open_us"] = {"error": str(e)}
    ctx.close()
    return res


def host_cpu_info() -> dict:
    """The host cores this process may use: CPU model, affinity mask size and the cgroup CPU
    quota (cgroup v2 cpu.max or v1 cfs_quota/period); usable = min(affinity, quota)."""
    import math

    info = {"model": None, "affinity": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count(), "quota": None}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    q = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            a, b = f.read().split()
            if a != "max":
                q = int(a) / int(b)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                a = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                b = int(f.read())
            if a > 0:
                q = a / b
        except (OSError, ValueError):
            pass
    info["quota"] = q
    info["usable"] = max(1, min(info["affinity"], math.floor(q) if q else info["affinity"]))
    return info


# cpu_bench sample per workload: (records, record bytes) of the same shape as the GPU workload,
# bounded so the 1-process run stays within ~10 s of CPU work (3 warm-ups + 10 timed passes each way)
CPU_SAMPLE = {"gcm1k": (65536, 1024), "gcm4k": (16384, 4096), "ocb1m": (64, 1 << 20), "ctr1g": (256, 1 << 20),
              "alltoall": (8, 1 << 20)}
CPU_SEED_PT, CPU_SEED_NONCE = 0xC0FFEE, 0x5EED


def cpu_reference_baseline(workload: str, device: int) -> dict:
    """Rank-0 CPU baseline = the reference's CPU path as this image can build it: AEAD seal/open
    with AES-NI/PCLMUL through the EVP interface (tools/cpu_bench.c: system OpenSSL 3, the
    stand-in for the reference's BoringSSL, send.c:292-315), timed on this box's host cores in a
    child process (forked workers; OpenSSL 3 contends on internal locks across threads of one
    process), 1 worker and `usable` workers, 3 warm-ups + median of 10 passes each way.  The
    first 16 tags are checked against this engine's GPU seal of the same inputs."""
    import subprocess

    from cryptmpi_2022_amd.synth import splitmix64_bytes

    alg = WORKLOADS[workload][0]
    N, n = CPU_SAMPLE[workload]
    info = host_cpu_info()
    exe = os.path.join(ROOT, "tools", "cpu_bench")
    runs = {}
    for procs in sorted({1, info["usable"]}):
        out = subprocess.run([exe, alg, str(n), str(N), str(procs), "3", "10", str(CPU_SEED_PT), str(CPU_SEED_NONCE)],
                             capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            raise RuntimeError(f"cpu_bench rc={out.returncode}: {out.stderr.strip()[-300:]}")
        runs[procs] = json.loads(out.stdout.strip().splitlines()[-1])
    allr = runs[info["usable"]]
    # parity of the baseline: the GPU's tags for the same first 16 records
    match = None
    if alg in ("gcm", "ocb"):
        k = min(16, N)
        pt = torch.from_numpy(splitmix64_bytes(CPU_SEED_PT, k * n)).to(f"cuda:{device}")
        nn = torch.from_numpy(splitmix64_bytes(CPU_SEED_NONCE, 12 * k)).to(f"cuda:{device}")
        ct = torch.empty(k * (n + 16), dtype=torch.uint8, device=f"cuda:{device}")
        ctx = aead.AeadCtx(KEY, "aes-128-gcm" if alg == "gcm" else "aes-128-ocb", device=device)
        ctx.seal_batch(ct, pt, nn, n, k)
        torch.cuda.synchronize(device)
        tags = ct.view(k, n + 16)[:, n:].cpu().numpy()
        ctx.close()
        match = [bytes(t).hex() for t in tags] == allr["tags16"]
    return {"value": round(allr["seal_open_GiBps"], 3), "unit": "GiB/s", "cores": info["usable"], "kind": "reference",
            "impl": "stand-in for the reference's BoringSSL AES-NI/PCLMUL path: system OpenSSL 3 EVP "
                    "(BoringSSL's crypto/ sources are absent; its prebuilt libcrypto is never run), "
                    f"{info['usable']} forked worker processes, static partition over records (send.c:292)",
            "sample": f"{N} x {n} B {alg.upper()} seal+open per pass (3 warm-ups, median of 10 passes each way)",
            "seal_GiBps": round(allr["seal_GiBps"], 3), "open_GiBps": round(allr["open_GiBps"], 3),
            "one_core": {k_: round(runs[1][k_], 3) for k_ in ("seal_GiBps", "open_GiBps", "seal_open_GiBps")},
            "host": info, "round_trip": allr["round_trip"], "tags_match_gpu": match}


def config1_exchange(n: int = 64 << 10, iters: int = 200) -> dict:
    """BASELINE config 1's counterpart: 2-process secure MPI_Send/MPI_Recv ping-pong with 600
    framing (tools/config1_exchange.py, child processes of this one), one-way latency per
    message with GPU seal/open vs the same ping-pong in plaintext over the same transport."""
    import socket
    import subprocess

    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "tools", "config1_exchange.py"), "--msg-bytes", str(n),
           "--iters", str(iters)]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240,
                         env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    if out.returncode or not lines:
        raise RuntimeError(f"config1_exchange rc={out.returncode}: {out.stderr.strip()[-400:]}")
    return json.loads(lines[-1])


def async_host_rate(device: int, n: int = 1 << 20, nreq: int = 64, reps: int = 3) -> dict:
    """The isend/wait split on the host path (include/cmpi_async.h): nreq messages of n bytes
    (pinned host buffers) sealed one after the other with the synchronous host call, vs all
    begun at once (MPI_Isend eager encryption) and completed with waitall."""
    from cryptmpi_2022_amd import _native as N

    L = N.lib()
    ctx = aead.AeadCtx(KEY, device=device)
    pt = torch.randint(0, 256, (nreq, n), dtype=torch.uint8).pin_memory()
    out = torch.empty((nreq, n + 16), dtype=torch.uint8).pin_memory()
    nn = torch.randint(0, 256, (nreq, 12), dtype=torch.uint8).pin_memory()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def sync():
        for i in range(nreq):
            N.check(L.cmpi_gcm_seal_host(ctx.handle, P(out[i]), n + 16, P(pt[i]), n, P(nn[i]), 12, n, 1))

    def overlapped():
        reqs = (ctypes.c_void_p * nreq)()
        for i in range(nreq):
            N.check(L.cmpi_gcm_seal_host_begin(ctx.handle, P(out[i]), n + 16, P(pt[i]), n, P(nn[i]), 12, n, 1,
                                               ctypes.byref(reqs, i * ctypes.sizeof(ctypes.c_void_p))))
        N.check(L.cmpi_waitall(reqs, nreq))

    def rate(fn):
        fn()
        best = float("inf")
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            best = min(best, time.perf_counter() - t0)
        return nreq * n / best / GIB

    r_sync, r_ovl = rate(sync), rate(overlapped)
    ctx.close()
    return {"config": f"{nreq} messages x {n} B GCM seal, pinned host buffers", "sync_host_GiBps": round(r_sync, 2),
            "async_begin_waitall_GiBps": round(r_ovl, 2), "speedup": round(r_ovl / r_sync, 2)}


def ctr702_rates(device: int, steps: int = 50) -> dict:
    """702 messages device-resident (include/cmpi_ctrmode.h): 4 KiB from the mask ring (stream A,
    one XOR pass) with the sender's precompute refilling it, 1 MiB and 8 MiB over stream B
    (sliced CTR), receiver included; message rates from HIP events on the stream."""
    from cryptmpi_2022_amd import ctrmode

    ctx = aead.CipherCtx(KEY, "aes-128-ctr", device=device)
    iv = bytes(range(32))
    s = ctrmode.Sender702(ctx, iv)
    res = {}
    for n in (4096, 1 << 20, 8 << 20):
        pt = torch.randint(0, 256, (n,), dtype=torch.uint8, device=f"cuda:{device}")
        ct = torch.empty_like(pt)
        back = torch.empty_like(pt)
        mask = torch.empty(n + 1024, dtype=torch.uint8, device=f"cuda:{device}")
        for _ in range(5):
            hdr, _ = s.send(ct, pt, n)
            s.precompute(n, 2)
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(steps):
            hdr, _ = s.send(ct, pt, n)
            s.precompute(n, 2)
            ml = ctrmode.recv702_premask(ctx, iv, hdr, mask)
            ctrmode.recv702(ctx, iv, hdr, back, ct, mask=mask, mask_len=ml)
        torch.cuda.synchronize(device)
        dt = (time.perf_counter() - t0) / steps
        res[f"{n}"] = {"us_per_message_send_precompute_recv": round(dt * 1e6, 2),
                       "GiBps": round(n / dt / GIB, 2), "verified": bool(torch.equal(back, pt))}
    s.close()
    ctx.close()
    res["note"] = ("timed from Python: five ctypes calls per message (send, precompute, premask, receive) "
                   "bound the 4 KiB rate; the C-timed per-op latencies, launched and served, are in "
                   "extras.c_timed_latency")
    return res


def c_timed_latency(iters: int = 300) -> dict:
    """Per-message latencies timed from C (tools/msg_latency: no Python on the path), medians of
    `iters` calls: device-resident 702 4 KiB messages (send.c:1537-1731 / recv.c:1107-1220), with
    a launch per op (the host spins on a word a one-wave kernel writes after the message) and
    served by the CTR context's resident service (each call complete on return: send, and the
    receiver's XOR once the payload has landed — its premask runs while the payload is in flight,
    recv.c:1107-1196); single GCM messages through the resident service; and the 602 8 MiB
    message from page-locked memory."""
    import subprocess

    exe = os.path.join(ROOT, "tools", "msg_latency")
    if not os.path.exists(exe):
        return {"error": "tools/msg_latency not built (make -C tools msg_latency)"}
    p = subprocess.run([exe, str(iters)], capture_output=True, text=True, timeout=240)
    if p.returncode != 0:
        return {"error": p.stderr[-400:]}
    d = json.loads(p.stdout.strip().splitlines()[-1])
    keep = ("flag_kernel_host_spin_us", "c702_4k_send_only_flag_us", "c702_4k_send_recv_nomask_flag_us",
            "c702_4k_send_premask_recv_flag_us", "c702_4k_send_precompute_recv_pipelined_us",
            "c702_4k_send_call_cpu_us", "c702_4k_recv_direct_call_cpu_us", "c702_4k_served_send_only_us",
            "c702_4k_served_recv_mask_us", "c702_4k_served_send_recv_nomask_us",
            "c702_4k_served_send_premask_recv_us", "ctr_host_4k_launch_us", "ctr_host_4k_served_us",
            "ctr_pageable_4k_launch_us", "ctr_pageable_4k_served_us", "ecb_16b_launch_us", "ecb_16b_served_us",
            "svc_pinned_seal_1k_us",
            "svc_pinned_open_1k_us", "svc_pinned_seal_64k_us", "svc_pinned_open_64k_us", "c602_8m_seal_per_outer_us",
            "c602_8m_seal_whole_us", "c602_8m_open_per_outer_us")
    out = {k: d[k] for k in keep if k in d}
    for k in ("c602_8m_seal_per_outer_us", "c602_8m_seal_whole_us", "c602_8m_open_per_outer_us"):
        if k in d:
            out[k.replace("_us", "_GiBps")] = round((8 << 20) / (d[k] * 1e-6) / GIB, 2)
    if "c702_4k_served_send_only_us" in d and "c702_4k_served_recv_mask_us" in d:
        out["c702_4k_served_send_plus_recv_us"] = round(d["c702_4k_served_send_only_us"] + d["c702_4k_served_recv_mask_us"], 2)
    out["iters"] = iters
    return out


def c_pingpong_600(iters: int = 2000) -> dict:
    """CryptMPI's per-message 600 exchange between two processes, in C, through the BoringSSL ABI
    (tools/evp_pingpong.c: send.c:221-337 / recv.c:219-341 framing, shared-memory transport,
    static large_send/recv_buffer, malloc'd user buffers): one-way latency medians of the plaintext
    exchange, the secure one through libcmpi_evp.so (the drop-in's defaults: resident service on;
    and with CMPI_EVP_SERVICE_US=0, a kernel launch per call) and through OpenSSL 3 on the calling
    core; crypto_added = secure - plaintext."""
    import subprocess

    gpu, cpu = os.path.join(ROOT, "tools", "evp_pingpong"), os.path.join(ROOT, "tools", "evp_pingpong_ossl")
    if not (os.path.exists(gpu) and os.path.exists(cpu)):
        return {"error": "tools/evp_pingpong not built (make -C tools pingpong)"}

    def run(exe, mode, n, env=None):
        p = subprocess.run([exe, mode, str(n), str(iters)], capture_output=True, text=True, timeout=120,
                           env=dict(os.environ, **(env or {})))
        if p.returncode != 0:
            raise RuntimeError(f"{os.path.basename(exe)} {mode} {n}: rc {p.returncode} {p.stderr[-300:]}")
        d = json.loads(p.stdout.strip().splitlines()[-1])
        assert d["verified"], "ping-pong payload mismatch"
        return d["oneway_us_median"]

    out = {"iters": iters, "unit": "us one-way (round trip / 2), median"}
    for n in (1024, 65536):
        k = f"{n // 1024}k"
        plain = run(gpu, "plain", n)
        served = run(gpu, "secure", n)
        launch = run(gpu, "secure", n, {"CMPI_EVP_SERVICE_US": "0"})
        ossl = run(cpu, "secure", n)
        out[k] = {"plain_us": plain, "secure_dropin_us": served, "secure_dropin_launch_per_call_us": launch,
                  "secure_openssl_1core_us": ossl, "crypto_added_dropin_us": round(served - plain, 2),
                  "crypto_added_dropin_launch_per_call_us": round(launch - plain, 2),
                  "crypto_added_openssl_1core_us": round(ossl - plain, 2)}
    return out


def cpu_port_baseline(workload: str, seconds: float = 4.0) -> dict:
    """Secondary CPU datum: the oracle's C restatement (portable table AES, bit-serial GHASH;
    oracle/liboracle.so), all usable host threads, on a bounded sample of the workload."""
    import oracle
    from cryptmpi_2022_amd.synth import random_nonces, records

    alg, n, N, _ = WORKLOADS[workload]
    threads = host_cpu_info()["usable"]
    res = {}
    # --- oracle port: size the sample so one seal+open pass takes ~seconds/2
    if alg == "ctr":
        nbytes = 64 << 20
        data = np.frombuffer(records(5, 1, nbytes).tobytes(), np.uint8)
        t0 = time.perf_counter()
        reps = 0
        while time.perf_counter() - t0 < seconds / 2:
            oracle.ctr_xor_mt(KEY, bytes(16), data, threads)
            reps += 1
        dt = time.perf_counter() - t0
        res["port"] = {"value": round(reps * nbytes / dt / GIB, 4), "sample": f"{reps} x 64 MiB CTR stream"}
    else:
        sample = max(1, min(N, int(4 * (1 << 20) // max(n, 1))))  # 4 MiB of records
        pt = records(3, sample, n)
        nn = random_nonces(4, sample)
        seal = oracle.gcm_seal_batch if alg == "gcm" else oracle.ocb_seal_batch
        t0 = time.perf_counter()
        passes = 0
        t_seal = t_open = 0.0
        while time.perf_counter() - t0 < seconds / 2:
            a = time.perf_counter()
            ct = seal(KEY, nn, pt, threads)
            b = time.perf_counter()
            if alg == "gcm":
                oracle.gcm_open_batch(KEY, nn, ct, threads)
            else:
                seal(KEY, nn, pt, threads)  # OCB open in the oracle is single-message; seal ~ same cost
            c = time.perf_counter()
            t_seal += b - a
            t_open += c - b
            passes += 1
        res["port"] = {"value": round(passes * sample * n / (t_seal + t_open) / GIB, 4),
                       "sample": f"{passes} passes x {sample} x {n} B seal+open"}
    res["cores"] = threads
    return res


def load_pmc(workload: str):
    """HBM traffic per launch of the dominant kernel from a committed rocprofv3 --pmc summary
    (profiles/pmc_<workload>.json): (bytes, label naming the file, its round and kernel) or
    (None, reason).  The counters come from separate --pmc passes of tools/gpu_pmc.sh, not from
    this run (rocprofv3 cannot collect them inside the bench's timed region)."""
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(p):
        return None, "no committed PMC summary"
    try:
        with open(p) as f:
            d = json.load(f)
    except Exception as e:
        return None, f"unreadable {p}: {e!r}"
    label = (f"profiles/pmc_{workload}.json ({d.get('round', 'round unrecorded')}, "
             f"kernel {d.get('dominant_kernel')}, rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, "
             "separate passes, not this run)")
    return d.get("traffic_bytes_per_launch"), label


def seal_kernel_name(w) -> str:
    """The seal launch's kernel(s) for this workload, from the plan the library will run
    (cmpi_debug_gcm_plan for GCM: {L, nseg, G, r0}; L = 64 is the flow decomposition)."""
    if w.alg == "ocb":
        return "ocb_batch_kernel<false> + ocb_final_kernel<false>"
    if w.alg == "ctr":
        return "ctr_kernel"
    L, nseg, _, _ = aead.gcm_plan(w.ctx, w.n, w.nrec)
    if L == 64:
        return "gcm_flow_kernel<false,...>" + (" + gcm_xor_combine_kernel<false>" if nseg > 1 else "")
    # third template argument: the record-store form (2 = line-aligned stores, the default at L = 4)
    return f"gcm_lane_kernel<{L}, false, {2 if L == 4 else 0}>" + (" + gcm_combine_kernel<false>" if nseg > 1 else "")


def spawn_ranks(n: int) -> None:
    """`--gpus N` without a launcher: start N ranks (one process per GPU) through
    torch.distributed.run on 127.0.0.1 with the same arguments, as the driver would, and exit with
    its status.  Runs before anything touches the GPU in this process (device_count() does not
    initialise HIP on this image); refuses when fewer than N GPUs are visible."""
    import socket
    import subprocess

    dry = "--dry-run" in sys.argv
    avail = torch.cuda.device_count()
    if not dry and avail < n:
        print(f"bench.py: --gpus {n} needs {n} visible GPUs, found {avail}", file=sys.stderr)
        sys.exit(2)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    sys.exit(subprocess.call(cmd, env=env))


def dry_run(args, ws: int, rank: int) -> None:
    """--dry-run: the multi-rank plumbing without a GPU (gloo): barrier, timed region, MAX over
    ranks, one JSON line from rank 0 — used by the CPU test of the launcher."""
    pg = None
    if ws > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")
        pg = dist
        dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.01)
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if pg is not None:
        pg.all_reduce(t, op=pg.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": ws, "steps": args.steps,
                          "warmup": args.warmup, "dry_run": True, "wall_max_s": round(float(t.item()), 4)}))
    if pg is not None:
        pg.destroy_process_group()


METRIC = "GiB/s device-resident AES-GCM seal+open on batched buffers, 1/2/4/8 GPU"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="gcm1k", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--serial", action="store_true", help="time only the one-stream pass (the default since round 6)")
    ap.add_argument("--with-pipelined", action="store_true",
                    help="also time the two-stream overlapped pass (reported as ms_per_step_pipelined)")
    ap.add_argument("--pipelined", action="store_true", help="headline = the two-stream overlapped pass")
    ap.add_argument("--dry-run", action="store_true", help="multi-rank plumbing only (no GPU), for tests")
    args = ap.parse_args()

    ws, rank, local = dist_env()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        spawn_ranks(args.gpus)  # does not return
    if ws != args.gpus:
        print(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    if args.dry_run:
        dry_run(args, ws, rank)
        return
    torch.cuda.set_device(local)
    pg = None
    if ws > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        pg = dist

        def barrier():
            dist.barrier(device_ids=[local])
    else:
        def barrier():
            pass

    w = Workload(args.workload, local, seed=1000 + rank)
    # One untimed step and its round-trip check BEFORE the warm-up: the check is the process's
    # first use of torch's comparison / reduction kernels, whose one-time lazy initialisation left
    # the timed region right after it ~15 % slow (config 2: 70.6 vs 60.8 us per seal launch in
    # fresh processes on one box, tools/timing_compare_probe.py, profiles/r05q_*; rounds 1-4
    # reported that first-pass figure as the sustained per-kernel time).
    w.seal()
    w.open()
    assert w.verify(), "round trip failed"
    # W warm-up steps, and at least WARMUP_S seconds of them (clocks out of their idle state)
    tdet: dict = {}
    wall, seal_ms, open_ms = time_steps(w, args.steps, args.warmup, barrier, warmup_s=WARMUP_S, detail=tdet)
    ok = w.verify()
    wall_serial = wall
    # the headline is this one-stream pass (each step seals then opens its batch).  On request
    # (--with-pipelined / --pipelined) also timed: the same K steps with consecutive batches
    # overlapped on two streams (seal of batch i+1 while batch i opens, the round-3 headline) — at
    # steady state it is no faster (config 2: 0.1220 vs 0.1196 ms per step, profiles/r05r_*).  Not
    # run by default since round 6: its overlapped seal launches take twice as long each and mixed
    # into a rocprofv3 summary of the default run they pulled the dominant kernel's average away
    # from the serial launches this line's roofline is computed from.
    wall_pipe = None
    if w.alg in ("gcm", "ocb") and (args.pipelined or args.with_pipelined) and not args.serial:
        wall_pipe, ok_p = time_steps_pipelined(w, args.steps, args.warmup, barrier, warmup_s=0.2)
        ok = ok and ok_p
        if args.pipelined:
            wall = wall_pipe
    pipelined = args.pipelined and wall_pipe is not None
    parity = w.parity_cpu() if rank == 0 else None  # outside the timed region
    per_rank_bytes = w.n * w.nrec  # plaintext bytes per step per rank
    wall_max, value = aggregate(wall, per_rank_bytes, args.steps, pg, w.dev)
    bpl = w.bytes_per_launch()
    kern_ms = seal_ms  # dominant kernel: the seal launch (open is within a few % of it)
    achieved = bpl / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src = load_pmc(args.workload)
    kname = seal_kernel_name(w)
    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_seconds_min": WARMUP_S,
        "ms_per_step": round(wall_max / args.steps * 1e3, 4),
        "ms_per_step_serial": round(wall_serial / args.steps * 1e3, 4),
        "ms_per_step_pipelined": None if wall_pipe is None else round(wall_pipe / args.steps * 1e3, 4),
        "headline_schedule": "pipelined (two streams)" if pipelined else "serial (one stream)",
        "steps_timed_as": ("two streams: the seal of batch i+1 overlaps the open of batch i (double-buffered); "
                           "every step seals and opens the whole batch") if pipelined else "one stream, seal then open",
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (torch.randint plaintext and nonces in HBM; fixed key)",
        "config": {"workload": args.workload, "desc": w.desc, "records_per_gpu": w.nrec, "record_bytes": w.n,
                   "parallelism": f"records sharded, {ws} independent rank(s), no collective"},
        "seal_GiBps_per_gpu": round(per_rank_bytes / (seal_ms * 1e-3) / GIB, 2),
        "open_GiBps_per_gpu": round(per_rank_bytes / (open_ms * 1e-3) / GIB, 2),
        "seal_GiBps_per_gpu_stream_bracket": round(per_rank_bytes / (tdet["seal_ms_stream_bracket"] * 1e-3) / GIB, 2),
        "rates_note": ("seal/open GiBps from the kernels' own execution (hipExtLaunchKernel events, the kernel-"
                       "timing pass); *_stream_bracket from the timed region's stream events, dispatch gaps "
                       "included; value from the timed region's wall clock"),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": f"seal launch ({kname})",
                     "kernel_ms": round(kern_ms, 4), "bytes_per_launch": bpl,
                     "kernel_ms_timing": ("hipExtLaunchKernel start/stop events of every seal launch of a pass of "
                                          "`steps` steps run right after the timed region (the kernel's execution, "
                                          "as rocprofv3 --kernel-trace reports it)"),
                     "launch_ms_stream_bracket": round(tdet["seal_ms_stream_bracket"], 4),
                     "launch_ms_stream_bracket_note": ("fence-free events recorded on the stream between the "
                                                       "launches of the timed region: the kernel plus the dependent "
                                                       "launch's dispatch gap; seal + open brackets = the step"),
                     "frac_stream_bracket": round(bpl / (tdet["seal_ms_stream_bracket"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
        "lds_roofline": lds_roofline(w, kern_ms, local) if w.alg == "gcm" else None,
        "verified_round_trip": ok,
        "parity_cpu": None if parity is None else parity["parity_cpu"],
        "parity": parity,
    }
    w.free()
    if rank == 0:
        try:
            peak_meas = copy_peak_gbs(local)
            result["roofline"]["peak_measured"] = round(peak_meas, 1)
            result["roofline"]["frac_measured"] = round(achieved / peak_meas, 4)
            result["roofline"]["peak_measured_note"] = (
                "library copy kernel (16 B per lane, grid-stride, 4 workgroups per CU), best of 80 copy "
                "forms swept on this hardware in round 5 (5.6-5.7 TB/s, profiles/r05u_copy_probe2.jsonl); "
                "below the guide's 6.29 TB/s float4 copy: no form reached 6.0 TB/s here")
        except Exception as e:  # report, never hide
            result["roofline"]["peak_measured"] = {"error": repr(e)}
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_reference_baseline(args.workload, local)
        except Exception as e:  # report, never hide
            result["cpu_baseline"] = {"error": repr(e)}
        try:
            cb = cpu_port_baseline(args.workload)
            result["cpu_baseline_port"] = dict(cb.get("port", {}), unit="GiB/s", cores=cb["cores"], kind="port",
                                               impl="oracle/ C restatement (portable table AES, bit-serial GHASH)")
        except Exception as e:
            result["cpu_baseline_port"] = {"error": repr(e)}
    if rank == 0 and ws == 1 and not args.no_extras and args.workload == "gcm1k":
        extras = {}
        for name in ("gcm4k", "ocb1m", "ctr1g", "ctr1g_mask", "alltoall"):
            try:
                we = Workload(name, local, seed=77)
                edet: dict = {}
                wl, s_ms, o_ms = time_steps(we, EXTRA_STEPS, EXTRA_WARMUP, barrier, warmup_s=0.3, detail=edet)
                extras[name] = {"seal_open_GiBps": round(we.n * we.nrec * EXTRA_STEPS / wl / GIB, 2),
                                "seal_GiBps": round(we.n * we.nrec / (s_ms * 1e-3) / GIB, 2),
                                "open_GiBps": round(we.n * we.nrec / (o_ms * 1e-3) / GIB, 2),
                                "seal_GiBps_stream_bracket": round(
                                    we.n * we.nrec / (edet["seal_ms_stream_bracket"] * 1e-3) / GIB, 2),
                                "seal_hbm_frac": round(we.bytes_per_launch() / (s_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                "verified": we.verify()}
                par = we.parity_cpu()
                extras[name]["parity_cpu"] = par["parity_cpu"]
                extras[name]["parity"] = par
                we.free()
            except Exception as e:  # report, never hide
                extras[name] = {"error": repr(e)}
        try:
            extras["config1_message_64k"] = config1_message(local)
        except Exception as e:
            extras["config1_message_64k"] = {"error": repr(e)}
        try:
            extras["host_path_pcie"] = host_path_rate(local)
        except Exception as e:
            extras["host_path_pcie"] = {"error": repr(e)}
        try:
            extras["host_602_8mib"] = host602_rate(local)
        except Exception as e:
            extras["host_602_8mib"] = {"error": repr(e)}
        for name, fn in (("async_host", lambda: async_host_rate(local)), ("ctr702", lambda: ctr702_rates(local)),
                         ("config1_exchange_64k", config1_exchange), ("c_timed_latency", c_timed_latency),
                         ("c_pingpong_600", c_pingpong_600)):
            try:
                extras[name] = fn()
            except Exception as e:  # report, never hide
                extras[name] = {"error": repr(e)}
        result["extras"] = extras
    if not args.no_extras:  # config 5 end to end: a collective, so every rank runs it
        try:
            a2a = alltoall_e2e(local, pg, barrier)
        except Exception as e:  # report, never hide (the headline above is already measured)
            a2a = {"error": repr(e)}
        # the other collectives: on one rank by default (RCCL gather / scatter across ranks run
        # only with CMPI_BENCH_COLLECTIVES=1, so a multi-GPU scaling run cannot stall on them)
        colls = {"skipped": "multi-rank run without CMPI_BENCH_COLLECTIVES=1"}
        if ws == 1 or os.environ.get("CMPI_BENCH_COLLECTIVES") == "1":
            try:
                colls = naive_collectives_e2e(local, pg, barrier)
            except Exception as e:  # report, never hide
                colls = {"error": repr(e)}
        if rank == 0:
            result.setdefault("extras", {})["alltoall_e2e"] = a2a
            result["extras"]["naive_collectives_e2e"] = colls
    if rank == 0:
        print(json.dumps(result))
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
