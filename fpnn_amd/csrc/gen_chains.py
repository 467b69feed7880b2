#!/usr/bin/env python3
"""Generates ecc_chains.hpp: the multi-limb carry chains of k_ecdh.hip's field arithmetic
as single inline-asm blocks (one v_add_co / v_addc / v_sub_co / v_subb per limb, the carry
in vcc from one limb to the next, no padding between them), and the product-scan columns
(every partial product of a column in one block: hipcc pads each asm block's end with a
wait state, so one block per column instead of one per partial product).

Why asm: written with __builtin_addc / __builtin_subc, hipcc pads every carry hand-off with
two wait states (`s_nop`) -- over a thousand per ladder step, each costing an issue slot of
the wave -- although gfx950 forwards the carry without them (tools/probe/carry_hazard.hip:
0 wrong lanes of 8.4M for unpadded vcc and SGPR-pair chains on all-carry inputs).

  python3 gen_chains.py > ecc_chains.hpp
"""

SIZES = (6, 7, 8, 12, 14, 16)  # 2 * NW for the squares: 12, 14, 16


def asm_block(lines, outs, ins, clobber='"vcc"'):
    s = "    asm(" + "\n        ".join('"%s\\n\\t"' % ln for ln in lines[:-1]) + ("\n        " if len(lines) > 1 else "")
    s += '"%s"\n' % lines[-1]
    s += "        : " + ", ".join(outs) + "\n"
    s += "        : " + ", ".join(ins) + "\n"
    s += "        : " + clobber + ");\n"
    return s


def gen_add(n):
    # r = a + b; returns the carry out (0 / 1)
    outs = [f'"=&v"(r[{i}])' for i in range(n)] + ['"=v"(c)']
    ins = [f'"v"(a[{i}])' for i in range(n)] + [f'"v"(b[{i}])' for i in range(n)]
    A = lambda i: f"%{n + 1 + i}"  # noqa: E731
    B = lambda i: f"%{2 * n + 1 + i}"  # noqa: E731
    lines = [f"v_add_co_u32 %0, vcc, {A(0)}, {B(0)}"]
    lines += [f"v_addc_co_u32 %{i}, vcc, {A(i)}, {B(i)}, vcc" for i in range(1, n)]
    lines += [f"v_cndmask_b32 %{n}, 0, 1, vcc"]
    return (f"template <>\n__device__ __forceinline__ uint32_t add_n<{n}>(uint32_t *r, const uint32_t *a, "
            f"const uint32_t *b) {{\n    uint32_t c;\n" + asm_block(lines, outs, ins) + "    return c;\n}\n")


def gen_sub(n):
    # r = a - b; returns the borrow out (0 / 1)
    outs = [f'"=&v"(r[{i}])' for i in range(n)] + ['"=v"(c)']
    ins = [f'"v"(a[{i}])' for i in range(n)] + [f'"v"(b[{i}])' for i in range(n)]
    A = lambda i: f"%{n + 1 + i}"  # noqa: E731
    B = lambda i: f"%{2 * n + 1 + i}"  # noqa: E731
    lines = [f"v_sub_co_u32 %0, vcc, {A(0)}, {B(0)}"]
    lines += [f"v_subb_co_u32 %{i}, vcc, {A(i)}, {B(i)}, vcc" for i in range(1, n)]
    lines += [f"v_cndmask_b32 %{n}, 0, 1, vcc"]
    return (f"template <>\n__device__ __forceinline__ uint32_t sub_n<{n}>(uint32_t *r, const uint32_t *a, "
            f"const uint32_t *b) {{\n    uint32_t c;\n" + asm_block(lines, outs, ins) + "    return c;\n}\n")


def gen_reduce(n):
    # value = t + top * 2^(32n) < 2p  ->  r = value mod p: d = t - p with the borrow run
    # through top (its borrow out = "top == 0 and t < p" = keep t), then r = keep ? t : d.
    # p in VGPRs: a VOP2 carry op already reads vcc over the constant bus (one per instruction)
    outs = [f'"=&v"(r[{i}])' for i in range(n)] + [f'"=&v"(d[{i}])' for i in range(n)] + ['"=&v"(dt)']
    ins = [f'"v"(t[{i}])' for i in range(n)] + [f'"v"(p[{i}])' for i in range(n)] + ['"v"(top)']
    T = lambda i: f"%{2 * n + 1 + i}"  # noqa: E731
    P = lambda i: f"%{3 * n + 1 + i}"  # noqa: E731
    D = lambda i: f"%{n + i}"  # noqa: E731
    top = f"%{4 * n + 1}"
    lines = [f"v_subrev_co_u32 {D(0)}, vcc, {P(0)}, {T(0)}"]
    lines += [f"v_subbrev_co_u32 {D(i)}, vcc, {P(i)}, {T(i)}, vcc" for i in range(1, n)]
    lines += [f"v_subbrev_co_u32 %{2 * n}, vcc, 0, {top}, vcc"]
    lines += [f"v_cndmask_b32 %{i}, {D(i)}, {T(i)}, vcc" for i in range(n)]
    return (f"template <>\n__device__ __forceinline__ void reduce_n<{n}>(uint32_t *r, const uint32_t *t, uint32_t top, "
            f"const uint32_t *p) {{\n    uint32_t d[{n}], dt;\n" + asm_block(lines, outs, ins) + "}\n")


def gen_fsub(n):
    # r = a - b mod p (a, b < p): borrow chain in an SGPR pair, p & borrow by cndmask, add back
    outs = ([f'"=&v"(r[{i}])' for i in range(n)] + [f'"=&v"(q[{i}])' for i in range(n)] + ['"=&s"(m)'])
    ins = [f'"v"(a[{i}])' for i in range(n)] + [f'"v"(b[{i}])' for i in range(n)] + [f'"v"(p[{i}])' for i in range(n)]
    Q = lambda i: f"%{n + i}"  # noqa: E731
    M = f"%{2 * n}"
    A = lambda i: f"%{2 * n + 1 + i}"  # noqa: E731
    B = lambda i: f"%{3 * n + 1 + i}"  # noqa: E731
    P = lambda i: f"%{4 * n + 1 + i}"  # noqa: E731
    lines = [f"v_sub_co_u32 %0, {M}, {A(0)}, {B(0)}"]
    lines += [f"v_subb_co_u32 %{i}, {M}, {A(i)}, {B(i)}, {M}" for i in range(1, n)]
    lines += [f"v_cndmask_b32 {Q(i)}, 0, {P(i)}, {M}" for i in range(n)]
    lines += [f"v_add_co_u32 %0, vcc, %0, {Q(0)}"]
    lines += [f"v_addc_co_u32 %{i}, vcc, %{i}, {Q(i)}, vcc" for i in range(1, n)]
    return (f"template <>\n__device__ __forceinline__ void fsub_n<{n}>(uint32_t *r, const uint32_t *a, const uint32_t *b, "
            f"const uint32_t *p) {{\n    uint32_t q[{n}];\n    uint64_t m;\n" + asm_block(lines, outs, ins) + "}\n")


def gen_col(k):
    # one product-scan column: (hi:lo) = lo + sum x[j] * y[j], hi from the carries alone
    outs = ['"+v"(lo)', '"=&v"(hi)']
    ins = [f'"v"(x[{j}])' for j in range(k)] + [f'"v"(y[{j}])' for j in range(k)]
    X = lambda j: f"%{2 + j}"  # noqa: E731
    Y = lambda j: f"%{2 + k + j}"  # noqa: E731
    lines = []
    for j in range(k):
        lines.append(f"v_mad_u64_u32 %0, vcc, {X(j)}, {Y(j)}, %0")
        lines.append(f"v_addc_co_u32 %1, vcc, 0, {'0' if j == 0 else '%1'}, vcc")
    return (f"template <>\n__device__ __forceinline__ void mac_col<{k}>(uint64_t &lo, uint32_t &hi, const uint32_t *x, "
            f"const uint32_t *y) {{\n" + asm_block(lines, outs, ins) + "}\n")


def main():
    print("// ecc_chains.hpp -- GENERATED by gen_chains.py; do not edit.")
    print("// Multi-limb carry chains for k_ecdh.hip as single asm blocks (see gen_chains.py).")
    print("#pragma once\n")
    # primary templates: only the generated sizes exist (a missing one fails to compile)
    nosize = '{\n    static_assert(N < 0, "ecc_chains.hpp: size not generated (gen_chains.py)");\n}'
    print("template <int N>\n__device__ __forceinline__ uint32_t add_n(uint32_t *r, const uint32_t *a, const uint32_t *b) "
          + nosize)
    print("template <int N>\n__device__ __forceinline__ uint32_t sub_n(uint32_t *r, const uint32_t *a, const uint32_t *b) "
          + nosize)
    print("template <int N>\n__device__ __forceinline__ void reduce_n(uint32_t *r, const uint32_t *t, uint32_t top, "
          "const uint32_t *p) " + nosize)
    print("template <int N>\n__device__ __forceinline__ void fsub_n(uint32_t *r, const uint32_t *a, const uint32_t *b, "
          "const uint32_t *p) " + nosize)
    print("template <int N>\n__device__ __forceinline__ void mac_col(uint64_t &lo, uint32_t &hi, const uint32_t *x, "
          "const uint32_t *y) " + nosize + "\n")
    for k in range(1, 9):
        print(gen_col(k))
    for n in SIZES:
        print(gen_add(n))
        print(gen_sub(n))
        if n <= 8:
            print(gen_reduce(n))
            print(gen_fsub(n))


if __name__ == "__main__":
    main()
