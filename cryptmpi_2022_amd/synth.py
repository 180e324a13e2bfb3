"""Deterministic synthetic inputs: splitmix64 byte streams for plaintexts,
keys and RAND_bytes-style nonces, plus the 602-style counter nonces of
MV/src/mpi/pt2pt/send.c:651-670.  Host-side numpy only; no crypto here."""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64_words(seed: int, count: int) -> np.ndarray:
    """`count` successive splitmix64 outputs for state `seed` (state advanced before mixing)."""
    with np.errstate(over="ignore"):
        i = np.arange(1, count + 1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + i * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def splitmix64_bytes(seed: int, nbytes: int) -> np.ndarray:
    w = splitmix64_words(seed, (nbytes + 7) // 8)
    return w.view(np.uint8)[:nbytes].copy()


def records(seed: int, nrec: int, n: int) -> np.ndarray:
    """(nrec, n) u8 plaintexts: record i is splitmix64_bytes(seed ^ i, n) — per-record streams
    so any record can be regenerated alone (bench parity sampling)."""
    if nrec * n <= (1 << 24):
        return np.stack([splitmix64_bytes(seed ^ i, n) for i in range(nrec)]) if nrec else np.empty((0, n), np.uint8)
    # big batches: one stream, row-major (same distribution; used where per-record regeneration is not needed)
    return splitmix64_bytes(seed, nrec * n).reshape(nrec, n)


def random_nonces(seed: int, nrec: int) -> np.ndarray:
    """(nrec, 12) u8 nonces standing in for RAND_bytes(nonce, 12) (send.c:298, alltoall.c:800)."""
    return splitmix64_bytes(seed, nrec * 12).reshape(nrec, 12)


def nonces602(nrec: int, flag: bytes = b"0", last_flag: bytes | None = None) -> np.ndarray:
    """(nrec, 12) u8: "0000000" || flag || BE32(i) (send.c:651-670; last segment flag '1' in the
    pipeline path, send.c:781-804)."""
    out = np.full((nrec, 12), 0x30, dtype=np.uint8)
    out[:, 7] = flag[0]
    if last_flag is not None and nrec:
        out[-1, 7] = last_flag[0]
    idx = np.arange(nrec, dtype=np.uint32)
    out[:, 8:12] = idx.astype(">u4").view(np.uint8).reshape(nrec, 4)
    return out
