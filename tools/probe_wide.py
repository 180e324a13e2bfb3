#!/usr/bin/env python3
"""Phase timeline of gcm_wide_kernel (cmpi_debug_set_wide_probe): per-workgroup wall-clock
stamps (100 MHz) of start, tables staged, own Horner loop done, all Horner done, weight tables
staged, weights done, end — medians over workgroups, relative to the earliest start, in us."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from cryptmpi_2022_amd import _native as N, aead  # noqa: E402

PH = ["start", "staged", "horner", "horner_all", "wstaged", "weights", "end"]
res = {}
FLAGS = [int(x) for x in (sys.argv[1:] or ["1"])]  # cmpi_debug_set_flow flags per pass
for flags in FLAGS:
  N.lib().cmpi_debug_set_flow(1024, flags)
  for name, (n, nrec), steps in [("a2a_auto", (1 << 20, 8), 0), ("a2a_S4", (1 << 20, 8), 4), ("1x64k", (65536, 1), 0),
                                 ("64x1m_auto", (1 << 20, 64), 0)]:
      bench.WORKLOADS["_pw"] = ("gcm", n, nrec, name)
      aead.force_wide(1, steps)
      w = bench.Workload("_pw", 0, seed=3)
      buf = torch.zeros(8 * 4096, dtype=torch.int64, device="cuda")
      for _ in range(3):
          w.seal()
      torch.cuda.synchronize()
      N.lib().cmpi_debug_set_wide_probe(buf.data_ptr())
      w.seal()
      torch.cuda.synchronize()
      N.lib().cmpi_debug_set_wide_probe(None)
      b = buf.view(-1, 8).cpu()
      b = b[b[:, 0] > 0]
      t0 = int(b[:, 0].min())
      rel = (b[:, :7] - t0).double() / 100.0  # us
      med = rel.median(dim=0).values.tolist()
      mx = rel.max(dim=0).values.tolist()
      res[f"{name}:f{flags}"] = {"wgs": int(b.shape[0]), "plan": aead.gcm_plan(w.ctx, n, nrec),
                   "median_us": dict(zip(PH, [round(x, 2) for x in med])),
                   "max_us": dict(zip(PH, [round(x, 2) for x in mx]))}
      print(name, flags, res[f"{name}:f{flags}"], flush=True)
      w.free()
aead.force_wide(0, 0)
N.lib().cmpi_debug_set_flow(1024, 0)
print(json.dumps(res))
