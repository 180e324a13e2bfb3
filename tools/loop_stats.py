#!/usr/bin/env python3
"""Instruction mix of the loops in one kernel of an hipcc -S listing (used to size VALU vs LDS
per block).  Usage: tools/loop_stats.py <file.s> <mangled kernel name>"""
import collections
import re
import sys

src, kern = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(kern + ":"))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        labels[m.group(1)] = i
loops = []
for i, l in enumerate(body):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", l)
    if m:
        t = m.group(1) or m.group(2)
        if t in labels and labels[t] < i:
            loops.append((labels[t], i, t))


def mix(a, b):
    c = collections.Counter()
    for l in body[a:b + 1]:
        s = l.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        if op.startswith("v_"):
            k = "valu"
        elif op.startswith("ds_"):
            k = op
        elif op.startswith(("global_", "buffer_")):
            k = "vmem"
        elif op.startswith("s_waitcnt"):
            k = "waitcnt"
        elif op.startswith("s_"):
            k = "salu"
        else:
            k = op
        c[k] += 1
        if op.startswith("v_"):
            c["op:" + op] += 1
    return c


for a, b, t in loops:
    c = mix(a, b)
    if c["ds_read_b32"] + c["ds_read_b128"] < 16:
        continue
    print(f"loop {t} lines {a}-{b}:")
    base = {k: v for k, v in c.items() if not k.startswith("op:")}
    print("  ", dict(sorted(base.items())))
    ops = sorted(((v, k[3:]) for k, v in c.items() if k.startswith("op:")), reverse=True)
    print("   ", ", ".join(f"{k}:{v}" for v, k in ops[:25]))
