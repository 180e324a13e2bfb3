"""Instruction mix of a kernel's basic blocks from `make -C cryptmpi_2022_amd asm` output.
usage: python tools/isa_mix.py <mangled-kernel-substring> [top_blocks]"""
import collections, re, sys

src = open("cryptmpi_2022_amd/build/cmpi_aead-gfx950.s").read().splitlines()
pat, top = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3
start = next(i for i, l in enumerate(src) if l.startswith(pat) or (l.endswith(":") and pat in l and not l.startswith("\t")))
end = next(i for i in range(start + 1, len(src)) if src[i].startswith("\t.section") or ".Lfunc_end" in src[i])
blocks, cur, name = [], [], "entry"
for l in src[start + 1:end]:
    if re.match(r"^\.LBB\S+:", l):
        blocks.append((name, cur)); cur, name = [], l.split(":")[0]
        continue
    s = l.strip()
    if not s or s.startswith((";", ".")):
        continue
    cur.append(s.split()[0])
blocks.append((name, cur))
blocks.sort(key=lambda b: -len(b[1]))
for name, ins in blocks[:top]:
    c = collections.Counter(ins)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    ds = sum(v for k, v in c.items() if k.startswith("ds_"))
    sal = sum(v for k, v in c.items() if k.startswith("s_"))
    vm = sum(v for k, v in c.items() if k.startswith(("global_", "buffer_", "flat_")))
    print(f"{name}: {len(ins)} instr  VALU {valu}  DS {ds}  SALU/S {sal}  VMEM {vm}")
    print("   ", ", ".join(f"{k} {v}" for k, v in c.most_common(28)))
