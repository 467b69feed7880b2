"""The special-prime reductions and inversion chains of k_ecdh.hip (field kinds FK_K1,
FK_P256, FK_P224, FK_P192), restated limb for limb in Python and checked against plain
modular arithmetic -- including the carry-range assumptions the device code relies on
(column sums < 2^64, final carries in {-1, 0, 1} or {0, 1}, values < 2p before the last
conditional subtraction).  The GPU tests check the kernels themselves against the
reference's fixtures and the oracle (tests/test_gpu_ecdh.py); this pins the arithmetic
design on CPU."""
import random

import pytest

M = 1 << 32
P = {
    "secp256k1": (1 << 256) - (1 << 32) - 977,
    "secp256r1": (1 << 256) - (1 << 224) + (1 << 192) + (1 << 96) - 1,
    "secp224r1": (1 << 224) - (1 << 96) + 1,
    "secp192r1": (1 << 192) - (1 << 64) - 1,
}
NW = {"secp256k1": 8, "secp256r1": 8, "secp224r1": 7, "secp192r1": 6}


def limbs(x, n):
    return [(x >> (32 * i)) & (M - 1) for i in range(n)]


def value(u):
    return sum(w << (32 * i) for i, w in enumerate(u))


def settle(u, cr, p, nw):
    """value = U + cr * 2^(32 nw), cr in {-1, 0, 1} -> [0, p) (p256_fold / p224_fold tail)."""
    assert cr in (-1, 0, 1)
    U, top = value(u), 1 << (32 * nw)
    if cr < 0:
        return (U + p) % top
    if cr > 0 or U >= p:
        return (U - p) % top
    return U


def k1_fold(t):  # k_ecdh.hip k1_fold: three carry chains, a top fold, one subtraction
    p = P["secp256k1"]

    def addc(x, y, c):
        s = x + y + c
        assert 0 <= x < M and 0 <= y < M and c in (0, 1)
        return s & (M - 1), s >> 32

    ml = [(t[8 + i] * 977) & (M - 1) for i in range(8)]
    mh = [(t[8 + i] * 977) >> 32 for i in range(8)]
    u, c1 = [0] * 8, 0
    for i in range(8):
        u[i], c1 = addc(t[i], ml[i], c1)
    c2 = 0
    for i in range(1, 8):
        u[i], c2 = addc(u[i], t[7 + i], c2)
    u8, c2 = addc(c1, t[15], c2)
    c3 = 0
    for i in range(1, 8):
        u[i], c3 = addc(u[i], mh[i - 1], c3)
    u8, c3 = addc(u8, mh[7], c3)
    u9 = c2 + c3
    assert value(u) + ((u8 + (u9 << 32)) << 256) == value(t[:8]) + value(t[8:]) * ((1 << 32) + 977)
    a = u8 * 977
    a1 = (a >> 32) + u9 * 977
    assert a1 < 1 << 11
    s1, k = addc(a1, u8, 0)
    cy = 0
    u[0], cy = addc(u[0], a & (M - 1), cy)
    u[1], cy = addc(u[1], s1, cy)
    u[2], cy = addc(u[2], u9 + k, cy)
    for i in range(3, 8):
        u[i], cy = addc(u[i], 0, cy)
    v = value(u) + (cy << 256)
    assert v < 2 * p
    return v - p if v >= p else v


def p256_fold(t):  # k_ecdh.hip p256_fold: nine 8-limb chains, a signed top, one fold, settle
    W = 1 << 256

    def add(x, y):  # add_n<8>: (sum mod 2^256, carry)
        s = value(x) + value(y)
        return limbs(s % W, 8), s >> 256

    def sub(x, y):  # sub_n<8>: (difference mod 2^256, borrow)
        s = value(x) - value(y)
        return limbs(s % W, 8), 1 if s < 0 else 0

    c = t
    s2 = [0, 0, 0, c[11], c[12], c[13], c[14], c[15]]
    s3 = [0, 0, 0, c[12], c[13], c[14], c[15], 0]
    s4 = [c[8], c[9], c[10], 0, 0, 0, c[14], c[15]]
    s5 = [c[9], c[10], c[11], c[13], c[14], c[15], c[13], c[8]]
    s6 = [c[11], c[12], c[13], 0, 0, 0, c[8], c[10]]
    s7 = [c[12], c[13], c[14], c[15], 0, 0, c[9], c[11]]
    s8 = [c[13], c[14], c[15], c[8], c[9], c[10], 0, c[12]]
    s9 = [c[14], c[15], 0, c[9], c[10], c[11], 0, c[13]]
    v, cv = add(s2, s3)
    w, cw = add(v, v)
    k = 2 * cv + cw
    u, cy = add(c[:8], w)
    k += cy
    for s_ in (s4, s5):
        u, cy = add(u, s_)
        k += cy
    for s_ in (s6, s7, s8, s9):
        u, bo = sub(u, s_)
        k -= bo
    assert -4 <= k <= 6
    kp, kn = max(k, 0), max(-k, 0)
    u, ca = add(u, [kp, 0, 0, kn, 0, 0, kn, kp])
    u, cb = sub(u, [kn, 0, 0, kp, 0, 0, kp, kn])
    return settle(u, ca - cb, P["secp256r1"], 8)


def p224_fold(t):  # k_ecdh.hip p224_fold: four 7-limb chains, a signed top, one fold, settle
    W = 1 << 224

    def add(x, y):
        s = value(x) + value(y)
        return limbs(s % W, 7), s >> 224

    def sub(x, y):
        s = value(x) - value(y)
        return limbs(s % W, 7), 1 if s < 0 else 0

    c = t
    u, k = add(c[:7], [0, 0, 0, c[7], c[8], c[9], c[10]])
    u, cy = add(u, [0, 0, 0, c[11], c[12], c[13], 0])
    k += cy
    u, bo = sub(u, [c[7], c[8], c[9], c[10], c[11], c[12], c[13]])
    k -= bo
    u, bo = sub(u, [c[11], c[12], c[13], 0, 0, 0, 0])
    k -= bo
    assert -2 <= k <= 2
    kp, kn = max(k, 0), max(-k, 0)
    u, ca = add(u, [kn, 0, 0, kp, 0, 0, 0])
    u, cb = sub(u, [kp, 0, 0, kn, 0, 0, 0])
    return settle(u, ca - cb, P["secp224r1"], 7)


def p192_fold(t):  # k_ecdh.hip p192_fold: three 6-limb chains, one fold chain, one subtraction
    W = 1 << 192

    def add(x, y):
        s = value(x) + value(y)
        return limbs(s % W, 6), s >> 192

    c = t
    u, k = add(c[:6], [c[6], c[7], c[6], c[7], 0, 0])
    u, cy = add(u, [0, 0, c[8], c[9], c[8], c[9]])
    k += cy
    u, cy = add(u, [c[10], c[11], c[10], c[11], c[10], c[11]])
    k += cy
    assert 0 <= k <= 3
    u, cy = add(u, [k, 0, k, 0, 0, 0])
    p = P["secp192r1"]
    v = value(u) + (cy << 192)
    assert v < 2 * p
    return v - p if v >= p else v


FOLD = {"secp256k1": k1_fold, "secp256r1": p256_fold, "secp224r1": p224_fold, "secp192r1": p192_fold}


def sqr_limbs(a, nw):
    """sqrN: cross products once, doubled by a one-bit shift, plus the squares."""
    A, t, acc = limbs(a, nw), [0] * (2 * nw), 0
    for i in range(1, 2 * nw - 1):
        j = max(0, i - (nw - 1))
        while 2 * j < i:
            acc += A[j] * A[i - j]
            j += 1
        t[i], acc = acc & (M - 1), acc >> 32
    t[2 * nw - 1] = acc
    assert acc < M
    for i in range(2 * nw - 1, 0, -1):
        t[i] = ((t[i] << 1) | (t[i - 1] >> 31)) & (M - 1)
    t[0], cin = 0, 0
    for i in range(nw):
        w = ((t[2 * i + 1] << 32) | t[2 * i]) + cin + A[i] * A[i]
        t[2 * i], t[2 * i + 1], cin = w & (M - 1), (w >> 32) & (M - 1), w >> 64
    assert cin == 0
    return t


@pytest.mark.parametrize("curve", sorted(P))
def test_fold_matches_mod(curve):
    p, nw, fold = P[curve], NW[curve], FOLD[curve]
    rng = random.Random(len(curve))
    edge = [0, 1, 2, p - 1, p - 2, 1 << (32 * nw - 1), (1 << 96) - 1, 1 << 64]
    vals = edge + [rng.randrange(p) for _ in range(600)]
    for _ in range(3000):
        x, y = rng.choice(vals), rng.choice(vals)
        assert fold(limbs(x * y, 2 * nw)) == x * y % p
        assert fold(sqr_limbs(x, nw)) == x * x % p
    for _ in range(1500):  # arbitrary words below p^2, extreme limbs included
        ws = [rng.choice([0, M - 1, rng.randrange(M)]) for _ in range(2 * nw)]
        if value(ws) < p * p:
            assert fold(ws) == value(ws) % p


def _sq(x, n, p):
    for _ in range(n):
        x = x * x % p
    return x


def inv_chain(curve, a):  # k_ecdh.hip finv, special forms
    p = P[curve]

    def blk(x, n, y):
        return _sq(x, n, p) * y % p
    x2 = blk(a, 1, a)
    x3 = blk(x2, 1, a)
    x6 = blk(x3, 3, x3)
    if curve == "secp256k1":
        x9 = blk(x6, 3, x3)
        x11 = blk(x9, 2, x2)
        x22 = blk(x11, 11, x11)
        x44 = blk(x22, 22, x22)
        x88 = blk(x44, 44, x44)
        x176 = blk(x88, 88, x88)
        x220 = blk(x176, 44, x44)
        x223 = blk(x220, 3, x3)
        t = blk(blk(blk(x223, 23, x22), 5, a), 3, x2)
        return blk(t, 2, a)
    x12 = blk(x6, 6, x6)
    x15 = blk(x12, 3, x3)
    if curve == "secp256r1":
        x30 = blk(x15, 15, x15)
        x32 = blk(x30, 2, x2)
        t = _sq(blk(x32, 32, a), 96, p)
        t = blk(blk(blk(t, 32, x32), 32, x32), 30, x30)
        return blk(t, 2, a)
    x24 = blk(x12, 12, x12)
    x48 = blk(x24, 24, x24)
    x96 = blk(x48, 48, x48)
    x127 = blk(blk(blk(x96, 24, x24), 6, x6), 1, a)
    if curve == "secp224r1":
        return blk(x127, 97, x96)
    x62 = blk(blk(x48, 12, x12), 2, x2)
    return blk(blk(x127, 63, x62), 2, a)


@pytest.mark.parametrize("curve", sorted(P))
def test_inversion_chain_is_fermat(curve):
    p = P[curve]
    rng = random.Random(7 * len(curve))
    for a in [0, 1, 2, p - 1] + [rng.randrange(p) for _ in range(20)]:
        assert inv_chain(curve, a) == pow(a, p - 2, p)


# ---- ecc_chains.hpp: the generated asm blocks, interpreted -------------------------------
# Every asm block of fpnn_amd/csrc/ecc_chains.hpp is parsed and run here instruction by
# instruction (one lane: carries as 0/1) on random and all-carry operands, and its outputs are
# checked against big-integer arithmetic -- operand order (v_subrev / v_subbrev), carry
# hand-offs and the borrow run through the top word are pinned on CPU before any GPU run.
import os  # noqa: E402
import re  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fpnn_amd", "csrc")


def test_ecc_chains_header_matches_generator():
    out = subprocess.run([sys.executable, os.path.join(CSRC, "gen_chains.py")], capture_output=True, text=True,
                         check=True).stdout
    assert out == open(os.path.join(CSRC, "ecc_chains.hpp")).read(), "regenerate: python3 gen_chains.py > ecc_chains.hpp"


def _blocks():
    src = open(os.path.join(CSRC, "ecc_chains.hpp")).read()
    pat = re.compile(r"template <>\n__device__ __forceinline__ \w+ (\w+)<(\d+)>\((.*?)\) \{(.*?)\n\}\n", re.S)
    for m in pat.finditer(src):
        name, n, body = m.group(1), int(m.group(2)), m.group(4)
        asm = re.search(r"asm\((.*?)\n\s*: (.*?)\n\s*: (.*?)\n\s*: ", body, re.S)
        lines = [ln for ln in re.findall(r'"(.*?)(?:\\n\\t)?"', asm.group(1))]
        outs = re.findall(r'"[=+&]*(\w)"\((.*?)\)', asm.group(2))
        ins = re.findall(r'"(\w)"\((.*?)\)', asm.group(3))
        yield name, n, lines, [(c, v, True) for c, v in outs] + [(c, v, False) for c, v in ins]


def _run(lines, operands, env):
    """env: variable name -> value (inputs); returns the outputs by variable name."""
    reg = {}
    nout = sum(1 for _, _, o in operands if o)
    for k, (_, var, is_out) in enumerate(operands):
        reg[f"%{k}"] = env.get(var, 0)
    # "+v" outputs are also inputs (tied): the parser marks them as outputs whose value is read
    regs = dict(reg)
    regs["vcc"] = 0

    def val(x):
        return int(x) if re.fullmatch(r"\d+", x) else regs[x]

    for ln in lines:
        op, args = ln.split(None, 1)
        a = [x.strip() for x in args.split(",")]
        if op == "v_add_co_u32":
            s = val(a[2]) + val(a[3]); regs[a[0]], regs[a[1]] = s % M, s >> 32
        elif op == "v_addc_co_u32":
            s = val(a[2]) + val(a[3]) + val(a[4]); regs[a[0]], regs[a[1]] = s % M, s >> 32
        elif op in ("v_sub_co_u32", "v_subrev_co_u32", "v_subb_co_u32", "v_subbrev_co_u32"):
            x, y = (val(a[3]), val(a[2])) if "rev" in op else (val(a[2]), val(a[3]))
            b = val(a[4]) if "subb" in op else 0
            s = x - y - b; regs[a[0]], regs[a[1]] = s % M, 1 if s < 0 else 0
        elif op == "v_cndmask_b32":
            regs[a[0]] = val(a[2]) if val(a[3]) else val(a[1])
        elif op == "v_mad_u64_u32":
            s = val(a[2]) * val(a[3]) + val(a[4]); regs[a[0]], regs[a[1]] = s % (1 << 64), s >> 64
        else:
            raise AssertionError(f"unmodelled instruction {op}")
    return {operands[k][1]: regs[f"%{k}"] for k in range(nout)}


@pytest.mark.parametrize("seed", [1, 2])
def test_ecc_chains_asm_semantics(seed):
    rng = random.Random(seed)
    p = P["secp256k1"]
    pl = {6: limbs(P["secp192r1"], 6), 7: limbs(P["secp224r1"], 7), 8: limbs(p, 8)}
    seen = set()
    for name, n, lines, ops in _blocks():
        seen.add(name)
        for trial in range(300):
            def rnd(k):
                return [rng.choice([0, 1, M - 1, M - 2, rng.randrange(M)]) for _ in range(k)]
            if name in ("add_n", "sub_n"):
                a, b = rnd(n), rnd(n)
                env = {f"a[{i}]": a[i] for i in range(n)} | {f"b[{i}]": b[i] for i in range(n)}
                out = _run(lines, ops, env)
                r = [out[f"r[{i}]"] for i in range(n)]
                A, B = value(a), value(b)
                want = A + B if name == "add_n" else A - B
                assert value(r) == want % (1 << (32 * n)), (name, n)
                assert out["c"] == (1 if (want >= 1 << (32 * n) or want < 0) else 0), (name, n)
            elif name == "reduce_n":
                pp = pl[n]
                P_ = value(pp)
                v = rng.randrange(2 * P_)
                t, top = limbs(v % (1 << (32 * n)), n), v >> (32 * n)
                env = {f"t[{i}]": t[i] for i in range(n)} | {f"p[{i}]": pp[i] for i in range(n)} | {"top": top}
                out = _run(lines, ops, env)
                assert value([out[f"r[{i}]"] for i in range(n)]) == v % P_, (name, n)
            elif name == "fsub_n":
                pp = pl[n]
                P_ = value(pp)
                x, y = rng.randrange(P_), rng.randrange(P_)
                a, b = limbs(x, n), limbs(y, n)
                env = {f"a[{i}]": a[i] for i in range(n)} | {f"b[{i}]": b[i] for i in range(n)} | \
                      {f"p[{i}]": pp[i] for i in range(n)}
                out = _run(lines, ops, env)
                assert value([out[f"r[{i}]"] for i in range(n)]) == (x - y) % P_, (name, n)
            elif name == "mac_col":
                x, y = rnd(n), rnd(n)
                lo = rng.randrange(1 << 64)
                env = {f"x[{j}]": x[j] for j in range(n)} | {f"y[{j}]": y[j] for j in range(n)} | {"lo": lo}
                out = _run(lines, ops, env)
                want = lo + sum(x[j] * y[j] for j in range(n))
                assert out["lo"] + (out["hi"] << 64) == want, (name, n)
            else:
                raise AssertionError(f"untested block {name}")
    assert seen == {"add_n", "sub_n", "reduce_n", "fsub_n", "mac_col"}
