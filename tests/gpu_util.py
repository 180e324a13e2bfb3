"""Helpers for the -m gpu parity tests: numpy <-> torch device buffers."""
from __future__ import annotations

import numpy as np


def dev(a: np.ndarray):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).reshape(-1).view(np.uint8).copy()).to("cuda")


def empty(nbytes: int, fill: int | None = None):
    import torch

    t = torch.empty(max(nbytes, 1), dtype=torch.uint8, device="cuda")
    if fill is not None:
        t.fill_(fill)
    return t


def host(t) -> np.ndarray:
    import torch

    torch.cuda.synchronize()
    return t.cpu().numpy()


def status_buf(n: int):
    import torch

    return torch.full((max(n, 1),), -1, dtype=torch.int32, device="cuda")
