"""alltoall_e2e (config 5 end to end, one rank) repeated, with and without bench.py's time-based
warm-up, after a CPU-only pause like the bench's preceding parity checks:
python tools/e2e_warmup_probe.py [rounds]"""
import json
import sys
import time

sys.path.insert(0, ".")
import bench  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
res = {"warmup_s=0": [], "warmup_s=0.3": []}
for _ in range(rounds):
    for ws in (0.0, 0.3):
        time.sleep(1.0)  # GPU idle, as during the CPU-side parity checks
        r = bench.alltoall_e2e(0, None, lambda: None, warmup_s=ws)
        assert r["all_blocks_authenticated"] and r["recv_matches_peers"] and r["parity_cpu"], r
        res[f"warmup_s={ws:g}"].append(r["ms_per_call"])
        print(ws, r["ms_per_call"], flush=True)
print(json.dumps(res))
