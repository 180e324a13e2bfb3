#!/usr/bin/env python3
"""Generator of tools/probe/aes_bitslice_gen.hpp (tools/probe/ctr_bs_kernel.hpp and the probes; out of the product library since round 6): bitsliced AES-128 rounds for gfx950
as v_bitop3_b32 (3-input LUT) networks.

Bitsliced layout: a lane's 32-bit register holds ONE bit of the state
of 32 blocks (bit j of the register = block j).  Plane p = 8*i + b is bit b (b = 0 the LSB) of
state byte i (FIPS-197 byte order, column-major: byte i sits in column i/4, row i%4).  A round
is then a straight-line network of bitwise ops over 128 planes.

Pipeline:
 1. the AES S-box as the 113-gate Boyar-Peralta circuit (XOR/AND/XNOR), checked here against
    the S-box computed from GF(2^8) inversion + the affine map (all 256 inputs);
 2. one round's subject graph: 16 S-boxes -> the round key XORed into the S-box outputs (the
    key of a middle round is pre-multiplied by InvMixColumns on the host, since MixColumns is
    linear: MC(s ^ MC^-1(k)) = MC(s) ^ k) -> ShiftRows (wiring) -> MixColumns as 2-input XORs
    (none in the last round);
 3. technology mapping to 3-input LUTs (cut enumeration, area flow, exact-area recovery),
    with the gfx9 constant-bus rule: at most one key plane (an SGPR) per LUT;
 4. the mapped network simulated against a plain AES round on random states;
 5. C++ emitted in an order that keeps live planes low (the four S-boxes of one output column,
    then that column's MixColumns).

Run:  python3 tools/gen_bitslice.py  (rewrites the header, prints the LUT counts)."""
from __future__ import annotations

import os
import random
import sys

# ------------------------------------------------------------------ AES reference pieces
def _gmul(a: int, b: int) -> int:
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= 0x11B
        b >>= 1
    return r


def sbox_table() -> list[int]:
    inv = [0] * 256
    for a in range(1, 256):
        for b in range(1, 256):
            if _gmul(a, b) == 1:
                inv[a] = b
                break
    out = []
    for a in range(256):
        x = inv[a]
        s = x
        for i in range(1, 5):
            s ^= ((x << i) | (x >> (8 - i))) & 0xFF
        out.append(s ^ 0x63)
    return out


SBOX = sbox_table()

# Boyar-Peralta 113-gate S-box (x0 = MSB ... x7 = LSB; s0 = MSB of the output).
BP = """
y14 = x3 ^ x5
y13 = x0 ^ x6
y9 = x0 ^ x3
y8 = x0 ^ x5
t0 = x1 ^ x2
y1 = t0 ^ x7
y4 = y1 ^ x3
y12 = y13 ^ y14
y2 = y1 ^ x0
y5 = y1 ^ x6
y3 = y5 ^ y8
t1 = x4 ^ y12
y15 = t1 ^ x5
y20 = t1 ^ x1
y6 = y15 ^ x7
y10 = y15 ^ t0
y11 = y20 ^ y9
y7 = x7 ^ y11
y17 = y10 ^ y11
y19 = y10 ^ y8
y16 = t0 ^ y11
y21 = y13 ^ y16
y18 = x0 ^ y16
t2 = y12 & y15
t3 = y3 & y6
t4 = t3 ^ t2
t5 = y4 & x7
t6 = t5 ^ t2
t7 = y13 & y16
t8 = y5 & y1
t9 = t8 ^ t7
t10 = y2 & y7
t11 = t10 ^ t7
t12 = y9 & y11
t13 = y14 & y17
t14 = t13 ^ t12
t15 = y8 & y10
t16 = t15 ^ t12
t17 = t4 ^ t14
t18 = t6 ^ t16
t19 = t9 ^ t14
t20 = t11 ^ t16
t21 = t17 ^ y20
t22 = t18 ^ y19
t23 = t19 ^ y21
t24 = t20 ^ y18
t25 = t21 ^ t22
t26 = t21 & t23
t27 = t24 ^ t26
t28 = t25 & t27
t29 = t28 ^ t22
t30 = t23 ^ t24
t31 = t22 ^ t26
t32 = t31 & t30
t33 = t32 ^ t24
t34 = t23 ^ t33
t35 = t27 ^ t33
t36 = t24 & t35
t37 = t36 ^ t34
t38 = t27 ^ t36
t39 = t29 & t38
t40 = t25 ^ t39
t41 = t40 ^ t37
t42 = t29 ^ t33
t43 = t29 ^ t40
t44 = t33 ^ t37
t45 = t42 ^ t41
z0 = t44 & y15
z1 = t37 & y6
z2 = t33 & x7
z3 = t43 & y16
z4 = t40 & y1
z5 = t29 & y7
z6 = t42 & y11
z7 = t45 & y17
z8 = t41 & y10
z9 = t44 & y12
z10 = t37 & y3
z11 = t33 & y4
z12 = t43 & y13
z13 = t40 & y5
z14 = t29 & y2
z15 = t42 & y9
z16 = t45 & y14
z17 = t41 & y8
t46 = z15 ^ z16
t47 = z10 ^ z11
t48 = z5 ^ z13
t49 = z9 ^ z10
t50 = z2 ^ z12
t51 = z2 ^ z5
t52 = z7 ^ z8
t53 = z0 ^ z3
t54 = z6 ^ z7
t55 = z16 ^ z17
t56 = z12 ^ t48
t57 = t50 ^ t53
t58 = z4 ^ t46
t59 = z3 ^ t54
t60 = t46 ^ t57
t61 = z14 ^ t57
t62 = t52 ^ t58
t63 = t49 ^ t58
t64 = z4 ^ t59
t65 = t61 ^ t62
t66 = z1 ^ t63
s0 = t59 ^ t63
s6 = t56 ^ ~t62
s7 = t48 ^ ~t60
t67 = t64 ^ t65
s3 = t53 ^ t66
s4 = t51 ^ t66
s5 = t47 ^ t65
s1 = t64 ^ ~s3
s2 = t55 ^ ~t67
"""


def parse_bp():
    gates = []
    for line in BP.strip().splitlines():
        lhs, rhs = [p.strip() for p in line.split("=")]
        if "&" in rhs:
            a, b = [p.strip() for p in rhs.split("&")]
            gates.append((lhs, "and", a, b))
        else:
            a, b = [p.strip() for p in rhs.split("^")]
            if b.startswith("~"):
                gates.append((lhs, "xnor", a, b[1:]))
            else:
                gates.append((lhs, "xor", a, b))
    return gates


def check_bp(gates) -> None:
    for a in range(256):
        env = {f"x{i}": (a >> (7 - i)) & 1 for i in range(8)}
        for lhs, op, x, y in gates:
            u, v = env[x], env[y]
            env[lhs] = (u & v) if op == "and" else (u ^ v ^ (1 if op == "xnor" else 0))
        out = sum(env[f"s{i}"] << (7 - i) for i in range(8))
        if out != SBOX[a]:
            raise SystemExit(f"S-box circuit wrong at {a:#x}")


# ------------------------------------------------------------------ subject graph
class Graph:
    """Nodes: ('in', name) | ('key', name) | (op, a, b) with op in and/xor/xnor."""

    def __init__(self):
        self.nodes = []
        self.names = []

    def add(self, node, name=""):
        self.nodes.append(node)
        self.names.append(name)
        return len(self.nodes) - 1

    def inp(self, name):
        return self.add(("in", name), name)

    def key(self, name):
        return self.add(("key", name), name)

    def gate(self, op, a, b):
        return self.add((op, a, b))


def build_round(last: bool):
    """-> graph, inputs[128], keys[128], outputs[128] (plane index 8*byte + bit)."""
    g = Graph()
    gates = parse_bp()
    ins = [g.inp(f"x{p}") for p in range(128)]
    keys = [g.key(f"k{p}") for p in range(128)]
    sb = [[None] * 8 for _ in range(16)]  # sb[byte][bit] after S-box + key
    for i in range(16):
        env = {f"x{j}": ins[8 * i + (7 - j)] for j in range(8)}  # x0 = MSB
        for lhs, op, a, b in gates:
            env[lhs] = g.gate(op, env[a], env[b])
        for j in range(8):
            sb[i][7 - j] = env[f"s{j}"]
    # ShiftRows: output byte (r, c) = input byte (r, c + r); the key plane of the position the
    # byte moves to is XORed into the S-box output
    sr = [None] * 16
    for c in range(4):
        for r in range(4):
            q = 4 * c + r
            src = sb[4 * ((c + r) % 4) + r]
            sr[q] = [g.gate("xor", src[b], keys[8 * q + b]) for b in range(8)]
    if last:
        return g, ins, keys, [sr[p // 8][p % 8] for p in range(128)]
    outs = [None] * 128
    for c in range(4):
        a = [sr[4 * c + r] for r in range(4)]
        t = [[g.gate("xor", a[r][b], a[(r + 1) % 4][b]) for b in range(8)] for r in range(4)]
        for r in range(4):
            # out_r = xtime(a_r ^ a_r+1) ^ (a_r+1 ^ a_r+2) ^ a_r+3
            u = t[(r + 1) % 4]
            for b in range(8):
                xt = [t[r][b - 1]] if b > 0 else [t[r][7]]
                if b in (1, 3, 4):
                    xt.append(t[r][7])
                terms = xt + [u[b], a[(r + 3) % 4][b]]
                acc = terms[0]
                for x in terms[1:]:
                    acc = g.gate("xor", acc, x)
                outs[8 * (4 * c + r) + b] = acc
    return g, ins, keys, outs


# ------------------------------------------------------------------ LUT3 mapping
def tt_of(g: Graph, root: int, leaves: tuple) -> int:
    """8-bit truth table of root over leaves (leaf i = variable i; index bit 2-i for a,b,c)."""
    var = {}
    pats = [0xF0, 0xCC, 0xAA]  # a, b, c in bitop3 order: index = a<<2 | b<<1 | c
    for i, l in enumerate(leaves):
        var[l] = pats[i]
    memo = {}

    def ev(n):
        if n in var:
            return var[n]
        if n in memo:
            return memo[n]
        node = g.nodes[n]
        if node[0] in ("in", "key"):
            raise RuntimeError("leaf outside cut")
        x, y = ev(node[1]), ev(node[2])
        v = (x & y) if node[0] == "and" else (x ^ y) ^ (0xFF if node[0] == "xnor" else 0)
        memo[n] = v & 0xFF
        return memo[n]

    return ev(root)


def map_lut3(g: Graph, outputs: list[int], passes: int = 6):
    n = len(g.nodes)
    is_key = [g.nodes[i][0] == "key" for i in range(n)]
    is_leaf = [g.nodes[i][0] in ("in", "key") for i in range(n)]
    cuts = [None] * n
    for i in range(n):
        if is_leaf[i]:
            cuts[i] = [(i,)]
            continue
        a, b = g.nodes[i][1], g.nodes[i][2]
        cs = set()
        for ca in cuts[a]:
            for cb in cuts[b]:
                u = tuple(sorted(set(ca) | set(cb)))
                if len(u) > 3 or sum(is_key[x] for x in u) > 1:
                    continue
                cs.add(u)
        # dominance pruning
        cl = sorted(cs, key=len)
        kept = []
        for c in cl:
            sc = set(c)
            if not any(set(k) <= sc for k in kept):
                kept.append(c)
        cuts[i] = kept + [(i,)]  # trivial cut last (used only as a leaf of fanouts)
    fo = [0] * n
    for i in range(n):
        if not is_leaf[i]:
            fo[g.nodes[i][1]] += 1
            fo[g.nodes[i][2]] += 1
    for o in outputs:
        fo[o] += 1
    # area flow
    af = [0.0] * n
    best = [None] * n
    for i in range(n):
        if is_leaf[i]:
            continue
        bv, bc = None, None
        for c in cuts[i][:-1]:
            v = 1.0 + sum(af[l] / max(1, fo[l]) for l in c)
            if bv is None or v < bv - 1e-9 or (abs(v - bv) < 1e-9 and len(c) < len(bc)):
                bv, bc = v, c
        af[i], best[i] = bv, bc
    refs = [0] * n

    def ref(i):  # returns LUTs added
        if is_leaf[i]:
            return 0
        refs[i] += 1
        if refs[i] > 1:
            return 0
        return 1 + sum(ref(l) for l in best[i])

    def deref(i):
        if is_leaf[i]:
            return 0
        refs[i] -= 1
        if refs[i] > 0:
            return 0
        return 1 + sum(deref(l) for l in best[i])

    for o in outputs:
        ref(o)
    for _ in range(passes):
        for i in range(n):
            if is_leaf[i] or refs[i] == 0:
                continue
            # exact area of each cut: deref current, ref candidate, measure, undo
            cur = best[i]
            a0 = deref_cut = sum(deref(l) for l in cur)
            bc, bv = cur, None
            for c in cuts[i][:-1]:
                best_i_save = best[i]
                best[i] = c
                v = sum(ref(l) for l in c)
                sum(deref(l) for l in c)
                best[i] = best_i_save
                if bv is None or v < bv or (v == bv and len(c) < len(bc)):
                    bv, bc = v, c
            best[i] = bc
            sum(ref(l) for l in bc)
            del a0, deref_cut
    luts = [i for i in range(n) if not is_leaf[i] and refs[i] > 0]
    return luts, best


def simulate_mapped(g, luts, best, ins, keys, outputs, inval, keyval):
    val = {}
    for p in range(128):
        val[ins[p]] = inval[p]
        val[keys[p]] = keyval[p]
    order = sorted(luts)
    for i in order:
        c = best[i]
        tt = tt_of(g, i, c)
        xs = [val[l] for l in c] + [0] * (3 - len(c))
        r = 0
        for bit in range(64):
            idx = 0
            for k in range(3):
                idx = idx * 2 + ((xs[k] >> bit) & 1 if k < len(c) else 0)
            # pad: unused variables read as 0 -> index uses only real vars in the high positions
            r |= ((tt >> _pad_index(idx, len(c))) & 1) << bit
        val[i] = r
    return [val[o] for o in outputs]


def _pad_index(idx, nvars):
    # a cut of size < 3 still uses variable slots a(,b); the unused low slots are 0
    return idx


def xtime(x):
    return ((x << 1) ^ (0x1B if x & 0x80 else 0)) & 0xFF


def ref_round(state: list[int], key: list[int], last: bool) -> list[int]:
    s = [SBOX[x] for x in state]
    t = [0] * 16
    for c in range(4):
        for r in range(4):
            t[4 * c + r] = s[4 * ((c + r) % 4) + r]
    if not last:
        u = [0] * 16
        for c in range(4):
            a = t[4 * c:4 * c + 4]
            for r in range(4):
                u[4 * c + r] = xtime(a[r]) ^ xtime(a[(r + 1) % 4]) ^ a[(r + 1) % 4] ^ a[(r + 2) % 4] ^ a[(r + 3) % 4]
        t = u
    return [t[i] ^ key[i] for i in range(16)]


def inv_mix_key(k: list[int]) -> list[int]:
    out = [0] * 16
    for c in range(4):
        a = k[4 * c:4 * c + 4]
        for r in range(4):
            out[4 * c + r] = (_gmul(a[r], 14) ^ _gmul(a[(r + 1) % 4], 11) ^ _gmul(a[(r + 2) % 4], 13)
                              ^ _gmul(a[(r + 3) % 4], 9))
    return out


def verify(g, luts, best, ins, keys, outputs, last, trials=4):
    rng = random.Random(7)
    for _ in range(trials):
        states = [[rng.randrange(256) for _ in range(16)] for _ in range(64)]
        key = [rng.randrange(256) for _ in range(16)]
        kin = key if last else inv_mix_key(key)
        inval = [sum(((states[j][p // 8] >> (p % 8)) & 1) << j for j in range(64)) for p in range(128)]
        keyval = [(0xFFFFFFFFFFFFFFFF if (kin[p // 8] >> (p % 8)) & 1 else 0) for p in range(128)]
        got = simulate_mapped(g, luts, best, ins, keys, outputs, inval, keyval)
        for j in range(64):
            want = ref_round(states[j], key, last)
            have = [sum(((got[8 * i + b] >> j) & 1) << b for b in range(8)) for i in range(16)]
            if have != want:
                raise SystemExit("mapped round wrong")


# ------------------------------------------------------------------ emission
def emit(g, luts, best, ins, keys, outputs, last, fname):
    """C++ body: s[128] in, s[128] out (in place through temporaries), k = key planes pointer."""
    lutset = set(luts)
    # order: per output column, the LUTs its 32 outputs need (DFS), so temporaries die early
    order, seen = [], set()

    def visit(i):
        if i in seen or i not in lutset:
            return
        seen.add(i)
        for l in best[i]:
            visit(l)
        order.append(i)

    cols = [list(range(32 * c, 32 * c + 32)) for c in range(4)]
    out_of = {}
    for p, o in enumerate(outputs):
        out_of.setdefault(o, []).append(p)
    for col in cols:
        for p in col:
            visit(outputs[p])
    name = {}
    for p in range(128):
        name[ins[p]] = f"s[{p}]"
        name[keys[p]] = f"k[{p}]"
    lines = [f"// {len(luts)} LUT3 ops ({'last round' if last else 'middle round'}); generated by tools/gen_bitslice.py",
             f"__device__ __forceinline__ void {fname}(uint32_t (&s)[128], const uint32_t* __restrict__ k) {{"]
    lines.append("  uint32_t o[128];")
    cnt = 0
    for i in order:
        c = best[i]
        tt = tt_of(g, i, c)
        args = [name[l] for l in c]
        v = f"t{i}"
        if len(c) == 3:
            expr = f"bop3({args[0]}, {args[1]}, {args[2]}, 0x{tt:02x})"
        elif len(c) == 2:
            # variables a, b only: tt over index a<<2|b<<1|c with c free -> 2-input function
            expr = bop2(args, tt)
        else:
            expr = bop1(args, tt)
        lines.append(f"  const uint32_t {v} = {expr};")
        name[i] = v
        cnt += 1
    for p, o in enumerate(outputs):
        lines.append(f"  o[{p}] = {name[o]};")
    lines.append("#pragma unroll")
    lines.append("  for (int i = 0; i < 128; ++i) s[i] = o[i];")
    lines.append("}")
    return "\n".join(lines) + "\n"


def bop2(args, tt):
    # tt uses a (0xF0) and b (0xCC); reduce to a 2-input function of a, b
    f = {(x, y): (tt >> ((x << 2) | (y << 1))) & 1 for x in (0, 1) for y in (0, 1)}
    a, b = args
    if f == {(0, 0): 0, (0, 1): 1, (1, 0): 1, (1, 1): 0}:
        return f"({a} ^ {b})"
    if f == {(0, 0): 1, (0, 1): 0, (1, 0): 0, (1, 1): 1}:
        return f"~({a} ^ {b})"
    if f == {(0, 0): 0, (0, 1): 0, (1, 0): 0, (1, 1): 1}:
        return f"({a} & {b})"
    full = sum(f[(x, y)] << ((x << 2) | (y << 1) | z) for x in (0, 1) for y in (0, 1) for z in (0, 1))
    return f"bop3({a}, {b}, {b}, 0x{full:02x})"


def bop1(args, tt):
    f0, f1 = tt & 1, (tt >> 4) & 1
    a = args[0]
    if (f0, f1) == (0, 1):
        return a
    if (f0, f1) == (1, 0):
        return f"~{a}"
    raise RuntimeError("constant LUT")


def main():
    gates = parse_bp()
    check_bp(gates)
    out_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "probe", "aes_bitslice_gen.hpp")
    parts = ["// aes_bitslice_gen.hpp — GENERATED by tools/gen_bitslice.py; do not edit.\n"
             "// Bitsliced AES-128 rounds as gfx950 v_bitop3_b32 networks (ctr_kernels.hpp ctr_bs_kernel).\n"
             "#pragma once\n#include <stdint.h>\n\nnamespace cmpi::bs {\n\n"
             "// the truth table must be a compile-time constant of the builtin: a macro, not a function\n"
             "#define bop3(a, b, c, tt) __builtin_amdgcn_bitop3_b32((a), (b), (c), (tt))\n\n"]
    for last in (False, True):
        g, ins, keys, outs = build_round(last)
        luts, best = map_lut3(g, outs)
        verify(g, luts, best, ins, keys, outs, last)
        sizes = [len(best[i]) for i in luts]
        print(f"{'last' if last else 'middle'} round: {len(luts)} LUTs "
              f"(3-in {sizes.count(3)}, 2-in {sizes.count(2)}, 1-in {sizes.count(1)}), "
              f"{len(luts) / 32:.1f} per block", file=sys.stderr)
        parts.append("\n" + emit(g, luts, best, ins, keys, outs, last, "round_last" if last else "round_mid"))
    parts.append("\n}  // namespace cmpi::bs\n#undef bop3\n")
    if "--dry" not in sys.argv:
        with open(out_path, "w") as f:
            f.write("".join(parts))


if __name__ == "__main__":
    main()
