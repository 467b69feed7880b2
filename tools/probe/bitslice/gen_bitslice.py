#!/usr/bin/env python3
"""Generate the bitsliced AES S-box circuit used by the bitsliced HIP kernels.

Derivation (FIPS-197 §5.1.1: S(x) = A·x⁻¹ ⊕ 0x63 over GF(2⁸)/x⁸+x⁴+x³+x+1):
  * map x into the tower field GF((2⁴)²) = GF(2⁴)[β]/(β²+β+λ), GF(2⁴) = GF(2)[ω]/(ω⁴+ω+1)
    (the isomorphism is a GF(2)-linear 8x8 matrix, found numerically below);
  * invert there: x = aβ+b, Δ = λa² + ab + b², x⁻¹ = (aΔ⁻¹)β + (a+b)Δ⁻¹;
  * map back and apply the affine transform (one linear 8x8 matrix + constant).
Linear layers use greedy common-subexpression XOR networks; 2-input gates are then
fused into 3-input LUT ops (gfx950 v_bitop3_b32) wherever an intermediate has one use.

The circuit is verified exhaustively (all 256 inputs) in bit-parallel numpy.
Output: fpnn_amd/csrc/bs_sbox.inc (straight-line C++ over uint32_t, 32 blocks per word).

Truth-table convention for bitop3(a, b, c, T): bit ((a<<2)|(b<<1)|c) of T is the result,
i.e. T = f(0xF0, 0xCC, 0xAA) -- verified on the device by tests/test_gpu_bitslice.py.
"""
from __future__ import annotations

import argparse
import itertools
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ----------------------------------------------------------------------------------
# GF(2^8) (AES) arithmetic

def gmul(a, b, poly=0x11B):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= poly
        b >>= 1
    return r


def gpow(a, n):
    r = 1
    for _ in range(n):
        r = gmul(r, a)
    return r


def ginv(a):
    return 0 if a == 0 else gpow(a, 254)


def sbox_ref(x):
    i = ginv(x)
    s = i
    for k in range(1, 5):
        s ^= ((i << k) | (i >> (8 - k))) & 0xFF
    return s ^ 0x63


SBOX = [sbox_ref(x) for x in range(256)]
assert SBOX[0] == 0x63 and SBOX[1] == 0x7C and SBOX[0x53] == 0xED


# ----------------------------------------------------------------------------------
# Tower field inside the AES field

def find_tower():
    # omega: root of y^4 + y + 1 in GF(256)
    omega = next(w for w in range(2, 256) if gpow(w, 4) ^ w ^ 1 == 0)
    gf16 = []  # element with omega-coordinates v (4 bits) -> AES byte
    for v in range(16):
        e = 0
        for i in range(4):
            if v >> i & 1:
                e ^= gpow(omega, i)
        gf16.append(e)
    assert len(set(gf16)) == 16
    # lambda in GF(16) with z^2+z+lambda irreducible over GF(16)
    for lam_v in range(1, 16):
        lam = gf16[lam_v]
        if any(gmul(z, z) ^ z ^ lam == 0 for z in gf16):
            continue
        beta = next((bb for bb in range(256) if gmul(bb, bb) ^ bb ^ lam == 0), None)
        if beta is None:
            continue
        # tower coordinates t = (a_v << 4) | b_v  <->  AES byte a*beta + b
        to_aes = [gmul(gf16[t >> 4], beta) ^ gf16[t & 15] for t in range(256)]
        if len(set(to_aes)) != 256:
            continue
        from_aes = [0] * 256
        for t, x in enumerate(to_aes):
            from_aes[x] = t
        return omega, gf16, lam_v, beta, to_aes, from_aes
    raise RuntimeError("no tower found")


OMEGA, GF16, LAM_V, BETA, TO_AES, FROM_AES = find_tower()


def gf16_mul(a, b):  # omega-basis 4-bit vectors
    return GF16.index(gmul(GF16[a], GF16[b]))


def linear_matrix(f):
    """8x8 GF(2) matrix M (rows = output bits) of a linear map f on bytes."""
    cols = [f(1 << j) for j in range(8)]
    for x in range(256):  # check linearity
        y = 0
        for j in range(8):
            if x >> j & 1:
                y ^= cols[j]
        assert y == f(x), "map not linear"
    return [[(cols[j] >> i) & 1 for j in range(8)] for i in range(8)]


# ----------------------------------------------------------------------------------
# Circuit builder (SSA over 32-bit words; nodes are 2-input gates or NOT)

class Circuit:
    def __init__(self, n_inputs):
        self.ops = []  # (op, a, b)  op in {'in','xor','and','or','not','const1'}
        self.inputs = [self._add(("in", i, None)) for i in range(n_inputs)]
        self.memo = {}

    def _add(self, node):
        self.ops.append(node)
        return len(self.ops) - 1

    def xor(self, a, b):
        if a == b:
            raise ValueError("x^x")
        k = ("xor",) + tuple(sorted((a, b)))
        if k not in self.memo:
            self.memo[k] = self._add(("xor", min(a, b), max(a, b)))
        return self.memo[k]

    def and_(self, a, b):
        k = ("and",) + tuple(sorted((a, b)))
        if k not in self.memo:
            self.memo[k] = self._add(("and", min(a, b), max(a, b)))
        return self.memo[k]

    def not_(self, a):
        k = ("not", a)
        if k not in self.memo:
            self.memo[k] = self._add(("not", a, None))
        return self.memo[k]

    def xor_many(self, sigs):
        sigs = list(sigs)
        assert sigs
        acc = sigs[0]
        for s in sigs[1:]:
            acc = self.xor(acc, s)
        return acc

    def linear(self, matrix, ins):
        """Outputs y_i = XOR_j M[i][j] x_j via greedy pair-merging CSE (Paar)."""
        rows = [set(j for j in range(len(ins)) if matrix[i][j]) for i in range(len(matrix))]
        sig = list(ins)
        while True:
            counts = {}
            for r in rows:
                for p in itertools.combinations(sorted(r), 2):
                    counts[p] = counts.get(p, 0) + 1
            if not counts:
                break
            (p, q), c = max(counts.items(), key=lambda kv: (kv[1], -kv[0][0], -kv[0][1]))
            if c < 2:
                break
            sig.append(self.xor(sig[p], sig[q]))
            nid = len(sig) - 1
            for r in rows:
                if p in r and q in r:
                    r.discard(p)
                    r.discard(q)
                    r.add(nid)
        outs = []
        for r in rows:
            assert r, "zero row"
            outs.append(self.xor_many(sig[j] for j in sorted(r)))
        return outs

    def evaluate(self, inputs):
        vals = []
        for op, a, b in self.ops:
            if op == "in":
                vals.append(inputs[a])
            elif op == "xor":
                vals.append(vals[a] ^ vals[b])
            elif op == "and":
                vals.append(vals[a] & vals[b])
            elif op == "not":
                vals.append(~vals[a])
            else:
                raise ValueError(op)
        return vals


def gf16_mul_circuit(c, a, b):
    """c = a*b in GF(16), omega basis: sum of products per output bit."""
    terms = [[] for _ in range(4)]
    for i in range(4):
        for j in range(4):
            prod = gf16_mul(1 << i, 1 << j)
            for k in range(4):
                if prod >> k & 1:
                    terms[k].append((i, j))
    out = []
    for k in range(4):
        acc = None
        for i, j in terms[k]:
            t = c.and_(a[i], b[j])
            acc = t if acc is None else c.xor(acc, t)
        out.append(acc)
    return out


def gf16_linear_circuit(c, f, a):
    """Apply a GF(2)-linear map on GF(16) (4x4) to bits a."""
    cols = [f(1 << j) for j in range(4)]
    m = [[(cols[j] >> i) & 1 for j in range(4)] for i in range(4)]
    return c.linear(m, a)


def gf16_inverse_truth():
    inv = []
    for v in range(16):
        e = GF16[v]
        inv.append(GF16.index(ginv(e)) if e else 0)
    return inv


def build_sbox():
    c = Circuit(8)
    x = c.inputs
    # 1. AES bits -> tower bits (linear)
    m_in = linear_matrix(lambda v: FROM_AES[v])
    t = c.linear(m_in, x)  # t[0..3] = b (low), t[4..7] = a (high)
    b, a = t[0:4], t[4:8]
    # 2. delta = lam*a^2 + a*b + b^2 ; the a^2, lam*a^2 and b^2 parts are linear
    lin = lambda v_a, v_b: gf16_mul(LAM_V, gf16_mul(v_a, v_a)) ^ gf16_mul(v_b, v_b)  # noqa: E731
    cols = [lin(1 << j, 0) for j in range(4)] + [lin(0, 1 << j) for j in range(4)]
    m_lin = [[(cols[j] >> i) & 1 for j in range(8)] for i in range(4)]
    sq = c.linear(m_lin, a + b)
    ab = gf16_mul_circuit(c, a, b)
    delta = [c.xor(sq[k], ab[k]) for k in range(4)]
    # 3. delta^-1: 4-input LUT per output bit, realised later as bitop3 muxes
    inv_tt = gf16_inverse_truth()
    dinv = [lut4(c, delta, [(inv_tt[v] >> k) & 1 for v in range(16)]) for k in range(4)]
    # 4. x^-1 = (a*dinv) beta + ((a+b)*dinv)
    hi = gf16_mul_circuit(c, a, dinv)
    apb = [c.xor(a[k], b[k]) for k in range(4)]
    lo = gf16_mul_circuit(c, apb, dinv)
    # 5. tower -> AES bits, then affine: S = A*inv ^ 0x63 (linear part merged)
    def aff(v):
        y = TO_AES[v]
        s = y
        for k in range(1, 5):
            s ^= ((y << k) | (y >> (8 - k))) & 0xFF
        return s
    m_out = linear_matrix(aff)
    y = c.linear(m_out, lo + hi)
    y = [c.not_(y[k]) if (0x63 >> k) & 1 else y[k] for k in range(8)]
    return c, y


def lut4(c, ins, table):
    """4-input boolean function as a sum of minterm ANDs -- only a placeholder node;
    the fusion pass turns it into bitop3 muxes (cost 3)."""
    node = c._add(("lut4", tuple(ins), tuple(table)))
    return node


# ----------------------------------------------------------------------------------
# Fusion into bitop3 (3-input LUT) ops

def truth_of(fn):
    a, b, cc = 0xF0, 0xCC, 0xAA
    return fn(a, b, cc) & 0xFF


def fuse(c, outputs):
    """Return a list of emitted ops: ('bitop3', dst, (x,y,z), table) / ('lut4', ...) /
    ('and'/'xor'/'not'...) over signal ids, where each emitted node computes a function
    of <= 3 'materialized' signals."""
    ops = c.ops
    uses = [0] * len(ops)
    for i, (op, a, b) in enumerate(ops):
        if op in ("xor", "and"):
            uses[a] += 1
            uses[b] += 1
        elif op == "not":
            uses[a] += 1
        elif op == "lut4":
            for s in a:
                uses[s] += 1
    for o in outputs:
        uses[o] += 1

    # For each node compute an expression tree over "leaves" (materialized signals),
    # absorbing single-use children while the leaf count stays <= 3.
    expr = {}  # id -> (leaves tuple, python function of leaf values)

    def leaf(i):
        return ((i,), lambda v: v[0])

    for i, (op, a, b) in enumerate(ops):
        if op in ("in", "lut4"):
            continue

        def child(s):
            if s in expr and uses[s] == 1:
                return expr[s]
            return leaf(s)

        if op == "not":
            la, fa = child(a)
            cand = (la, (lambda fa: lambda v: ~fa(v))(fa))
            if len(la) > 3:
                cand = (((a,), lambda v: ~v[0]))
            expr[i] = cand
            continue
        la, fa = child(a)
        lb, fb = child(b)
        merged = tuple(dict.fromkeys(la + lb))
        g = (lambda x, y: x ^ y) if op == "xor" else (lambda x, y: x & y)
        if len(merged) <= 3:
            ia = [merged.index(s) for s in la]
            ib = [merged.index(s) for s in lb]
            expr[i] = (merged, (lambda fa, fb, ia, ib, g: lambda v: g(fa([v[k] for k in ia]),
                                                                      fb([v[k] for k in ib])))(fa, fb, ia, ib, g))
        else:  # cannot absorb both; try absorbing one child only
            best = None
            for la2, fa2, lb2, fb2 in ((la, fa, (b,), lambda v: v[0]), ((a,), lambda v: v[0], lb, fb)):
                m2 = tuple(dict.fromkeys(la2 + lb2))
                if len(m2) <= 3 and (best is None or len(m2) < len(best[0])):
                    ia = [m2.index(s) for s in la2]
                    ib = [m2.index(s) for s in lb2]
                    best = (m2, (lambda fa, fb, ia, ib, g: lambda v: g(fa([v[k] for k in ia]),
                                                                       fb([v[k] for k in ib])))(fa2, fb2, ia, ib, g))
            if best is None:
                best = ((a, b), (lambda g: lambda v: g(v[0], v[1]))(g))
            expr[i] = best

    # materialize: walk from outputs, emit nodes that are leaves of someone or outputs
    emitted = []
    done = set(i for i, (op, _, _) in enumerate(ops) if op == "in")
    order = []

    def need(i):
        if i in done:
            return
        op = ops[i]
        if op[0] == "lut4":
            for s in op[1]:
                need(s)
            done.add(i)
            order.append(("lut4", i, op[1], op[2]))
            return
        leaves, fn = expr[i]
        for s in leaves:
            need(s)
        done.add(i)
        vals = [0xF0, 0xCC, 0xAA][:len(leaves)]
        tt = fn(vals + [0] * (3 - len(vals))) & 0xFF if len(leaves) == 3 else None
        order.append(("expr", i, leaves, fn))

    for o in outputs:
        need(o)
    return order


def eval_order(order, n_inputs, inputs):
    vals = {i: inputs[i] for i in range(n_inputs)}
    for item in order:
        kind, i, leaves, fn = item
        if kind == "lut4":
            tab = fn
            idx = np.zeros_like(inputs[0])
            out = np.zeros_like(inputs[0])
            # bit-parallel: evaluate via minterms
            a = [vals[s] for s in leaves]
            for v in range(16):
                if tab[v]:
                    m = np.full_like(inputs[0], 0xFFFFFFFF)
                    for k in range(4):
                        m &= a[k] if (v >> k) & 1 else ~a[k]
                    out |= m
            vals[i] = out
        else:
            vals[i] = fn([vals[s] for s in leaves]) & 0xFFFFFFFF
    return vals


def table_of(fn, nleaves):
    base = [0xF0, 0xCC, 0xAA]
    v = fn(base[:nleaves] + [0] * (3 - nleaves)) & 0xFF
    if nleaves == 1:
        # f(a): expand over (a, *, *)
        pass
    return v


def cost(order):
    n = 0
    for kind, i, leaves, fn in order:
        if kind == "lut4":
            n += 3  # mux(x3, f0(x0..x2), f1(x0..x2))
        else:
            n += 1
    return n


# ----------------------------------------------------------------------------------

def verify(order, outputs):
    xs = np.arange(256, dtype=np.uint32)
    # pack 256 inputs into 8 words of 32 lanes each
    ok = True
    for base in range(0, 256, 32):
        blk = xs[base:base + 32]
        ins = [np.array([np.uint32(sum(((int(blk[l]) >> k) & 1) << l for l in range(32)))], dtype=np.uint32)
               for k in range(8)]
        vals = eval_order(order, 8, ins)
        for l in range(32):
            y = sum(((int(vals[outputs[k]][0]) >> l) & 1) << k for k in range(8))
            if y != SBOX[base + l]:
                ok = False
    return ok


def emit_cpp(order, outputs, path):
    """Straight-line device code: `#define`-free inline function body over uint32_t."""
    name = {i: f"x[{i}]" for i in range(8)}
    lines = []
    tmp = 0
    for kind, i, leaves, fn in order:
        var = f"t{tmp}"
        tmp += 1
        name[i] = var
        if kind == "lut4":
            a = [name[s] for s in leaves]
            tab = fn  # 16 entries, index v = bits (a3 a2 a1 a0)
            lo = sum(tab[v] << j for j, v in enumerate(range(8)))
            # f = a3 ? F1(a2,a1,a0) : F0(a2,a1,a0); bitop3 operand order (a2, a1, a0)
            t0 = lut3_table(lambda A, B, C: pick(tab, 0, A, B, C))
            t1 = lut3_table(lambda A, B, C: pick(tab, 1, A, B, C))
            lines.append(f"const uint32_t {var}_0 = BOP3({a[2]}, {a[1]}, {a[0]}, 0x{t0:02x});")
            lines.append(f"const uint32_t {var}_1 = BOP3({a[2]}, {a[1]}, {a[0]}, 0x{t1:02x});")
            lines.append(f"const uint32_t {var} = BOP3({a[3]}, {var}_1, {var}_0, 0xca);")  # a3 ? f1 : f0
            continue
        n = len(leaves)
        ops = [name[s] for s in leaves]
        while len(ops) < 3:
            ops.append("0u")
        base = [0xF0, 0xCC, 0xAA]
        tt = fn(base[:n] + [0] * (3 - n)) & 0xFF
        lines.append(f"const uint32_t {var} = BOP3({ops[0]}, {ops[1]}, {ops[2]}, 0x{tt:02x});")
    for k in range(8):
        lines.append(f"y[{k}] = {name[outputs[k]]};")
    body = "\n".join("    " + l for l in lines)
    text = ("// GENERATED by tools/gen_bitslice.py -- do not edit.\n"
            "// Bitsliced AES S-box: x[k] / y[k] hold bit k of one state byte of 32 blocks.\n"
            f"// {cost(order)} bitop3 ops; verified on all 256 inputs by the generator.\n"
            "// BOP3(a, b, c, T) = v_bitop3_b32 with T = f(0xF0, 0xCC, 0xAA).\n"
            "__device__ __forceinline__ void bs_sbox(const uint32_t x[8], uint32_t y[8]) {\n"
            + body + "\n}\n")
    with open(path, "w") as f:
        f.write(text)
    return len(lines)


def pick(tab, hi, A, B, C):
    # A = a2, B = a1, C = a0 as 0/1 ints (bitwise over masks handled by lut3_table)
    return tab[(hi << 3) | (A << 2) | (B << 1) | C]


def lut3_table(f):
    t = 0
    for idx in range(8):
        A, B, C = (idx >> 2) & 1, (idx >> 1) & 1, idx & 1
        if f(A, B, C):
            t |= 1 << idx
    return t


def check_emitted(path):
    """Interpret the emitted C++ under the documented bitop3 convention (all 256 inputs)."""
    import re
    body = open(path).read()
    stmts = re.findall(r"const uint32_t (\w+) = BOP3\(([^,]+), ([^,]+), ([^,]+), (0x[0-9a-f]+)\);", body)
    outs = dict(re.findall(r"y\[(\d)\] = (\w+);", body))
    def bop3(a, b, c, t):
        r = np.zeros_like(a)
        for idx in range(8):
            if t >> idx & 1:
                m = (a if idx & 4 else ~a) & (b if idx & 2 else ~b) & (c if idx & 1 else ~c)
                r |= m
        return r
    xs = np.arange(256, dtype=np.uint32)
    env = {f"x[{k}]": ((xs >> k) & 1) * np.uint32(0xFFFFFFFF) for k in range(8)}
    env["0u"] = np.zeros(256, dtype=np.uint32)
    for name, a, b, c, t in stmts:
        env[name] = bop3(env[a], env[b], env[c], int(t, 16))
    y = np.zeros(256, dtype=np.uint32)
    for k in range(8):
        y |= (env[outs[str(k)]] & 1) << k
    return all(int(y[x]) == SBOX[x] for x in range(256))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "fpnn_amd", "csrc", "bs_sbox.inc"))
    args = ap.parse_args()
    c, outs = build_sbox()
    raw = sum(1 for op in c.ops if op[0] in ("xor", "and", "not"))
    luts = sum(1 for op in c.ops if op[0] == "lut4")
    order = fuse(c, outs)
    print(f"tower: omega=0x{OMEGA:02x} lambda(v)={LAM_V} beta=0x{BETA:02x}")
    print(f"2-input gates: {raw} (+{luts} lut4); fused ops: {cost(order)}")
    assert verify(order, outs), "circuit does not reproduce the S-box"
    print("verified: all 256 inputs")
    n = emit_cpp(order, outs, args.out)
    assert check_emitted(args.out), "emitted code does not reproduce the S-box"
    print("wrote", args.out, n, "lines; emitted text re-verified")


if __name__ == "__main__":
    main()
