#!/usr/bin/env python3
"""Generates fisco-bcos_amd/csrc/fe_asm.h: 256-bit carry chains as single inline-asm blocks.

On gfx950 the compiler pads every dependent VCC carry step with `s_nop 1` (it models a VALU-writes-
VCC -> VALU-reads-VCC hazard).  tools/carrybench.hip checked 1.7e10 unpadded dependent carry steps
on MI355X with zero mismatches, so the hot chains are emitted unpadded, each in one asm block (VCC
never has to survive between asm statements).  All operands are VGPRs: VOP2 carry ops read VCC
implicitly, and an SGPR source would be a second constant-bus read.
"""
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "csrc", "fe_asm.h")


class Ops:
    """Operand numbering for one asm statement: outputs first, then inputs."""

    def __init__(self):
        self.outs, self.ins = [], []

    def out(self, name, n=8):
        base = len(self.outs)
        self.outs += [(name, i if n > 1 else None) for i in range(n)]
        return base

    def inp(self, name, n=8):
        base = len(self.ins)
        self.ins += [(name, i if n > 1 else None) for i in range(n)]
        return base

    def ref(self, kind, base, i=0):
        return "%" + str(base + i + (len(self.outs) if kind == "in" else 0))

    def constraints(self):
        def c(lst, tag):
            return ", ".join(f'"{tag}"({n}[{i}])' if i is not None else f'"{tag}"({n})' for n, i in lst)
        return c(self.outs, "=&v"), c(self.ins, "v")


def chain(first, rest, dst, a, b):
    lines = [f"{first} {dst[0]}, vcc, {a[0]}, {b[0]}"]
    lines += [f"{rest} {dst[i]}, vcc, {a[i]}, {b[i]}, vcc" for i in range(1, 8)]
    return lines


def render(sig, locals_, ops, body, doc, clobbers='"vcc"'):
    outs, ins = ops.constraints()
    s = [f"// {doc}", f"__device__ __forceinline__ void {sig} {{"]
    if locals_:
        s.append(f"    {locals_}")
    s.append("    asm(")
    for i, ln in enumerate(body):
        s.append(f'        "{ln}' + ('\\n\\t"' if i + 1 < len(body) else '"'))
    s.append(f"        : {outs}")
    s.append(f"        : {ins}")
    s.append(f'        : {clobbers});')
    s.append("}")
    return "\n".join(s) + "\n"


def k1_addsub(sub):
    ops = Ops()
    r, t0, t1 = ops.out("r"), ops.out("t0", 1), ops.out("t1", 1)
    a, b, k = ops.inp("a"), ops.inp("b"), ops.inp("k977", 1)
    R = [ops.ref("out", r, i) for i in range(8)]
    A = [ops.ref("in", a, i) for i in range(8)]
    B = [ops.ref("in", b, i) for i in range(8)]
    T0, T1, K = ops.ref("out", t0), ops.ref("out", t1), ops.ref("in", k)
    f, c, prop = (("v_sub_co_u32_e32", "v_subb_co_u32_e32", "v_subbrev_co_u32_e32") if sub else
                  ("v_add_co_u32_e32", "v_addc_co_u32_e32", "v_addc_co_u32_e32"))
    body = chain(f, c, R, A, B)
    # fold the carry/borrow out of 2^256: 2^256 == 2^32 + 977 (mod p).  The fold touches words 0-1;
    # it propagates into words 2-7 (and then needs a second fold) only when word 1 over/underflows,
    # probability ~2^-32 per lane, so that tail is branched over unless some lane of the wave needs it
    # (it adds each lane's own carry, 0 for the others).  s_nop covers the VALU-writes-VCC ->
    # SALU-reads-VCC latency.
    def fold():
        return [f"v_cndmask_b32_e64 {T0}, 0, {K}, vcc", f"v_cndmask_b32_e64 {T1}, 0, 1, vcc",
                f"{f} {R[0]}, vcc, {R[0]}, {T0}", f"{c} {R[1]}, vcc, {R[1]}, {T1}, vcc"]
    body += fold()
    body += ["s_nop 4", "s_cmp_eq_u64 vcc, 0", "s_cbranch_scc1 2f"]
    body += [f"{prop} {R[i]}, vcc, 0, {R[i]}, vcc" for i in range(2, 8)]
    body += fold()
    body += [f"{prop} {R[i]}, vcc, 0, {R[i]}, vcc" for i in range(2, 8)]
    body += ["2:"]
    name = "k1_sub_asm" if sub else "k1_add_asm"
    return render(f"{name}(uint32_t r[8], const uint32_t a[8], const uint32_t b[8])",
                  "uint32_t t0, t1; const uint32_t k977 = 977u;", ops, body,
                  f"secp256k1 base field: r = a {'-' if sub else '+'} b (mod p), values in [0, 2^256)",
                  clobbers='"vcc", "scc"')


def k1_shl_fold(K, R, T, M0):
    """R (8 words) + T * 2^256 -> R + T * (2^32 + 977) (mod p), T < 2^24: words 0-1 inline, the
    carry tail (probability ~2^-32 per lane) branched over unless some lane of the wave needs it."""
    add, addc = "v_add_co_u32_e32", "v_addc_co_u32_e32"
    b = [f"v_mul_u32_u24_e32 {M0}, {K}, {T}", f"{add} {R[0]}, vcc, {R[0]}, {M0}", f"{addc} {R[1]}, vcc, {R[1]}, {T}, vcc"]
    b += ["s_nop 4", "s_cmp_eq_u64 vcc, 0", "s_cbranch_scc1 2f"]
    b += [f"{addc} {R[i]}, vcc, 0, {R[i]}, vcc" for i in range(2, 8)]
    # a carry out of 2^256 here leaves R < T * (2^32 + 977) < 2^57 - fold it once more (no further carry)
    b += [f"v_cndmask_b32_e64 {M0}, 0, {K}, vcc", f"v_cndmask_b32_e64 {T}, 0, 1, vcc",
          f"{add} {R[0]}, vcc, {R[0]}, {M0}", f"{addc} {R[1]}, vcc, {R[1]}, {T}, vcc"]
    b += [f"{addc} {R[i]}, vcc, 0, {R[i]}, vcc" for i in range(2, 8)]
    b += ["2:"]
    return b


def shifted(X, k, dst):
    """dst[0..7] = low 256 bits of X << k (k in 1..3); returns the instructions (top word separate)."""
    b = [f"v_lshlrev_b32_e32 {dst[0]}, {k}, {X[0]}"]
    b += [f"v_alignbit_b32 {dst[i]}, {X[i]}, {X[i - 1]}, {32 - k}" for i in range(1, 8)]
    return b


def k1_shl(k):
    ops = Ops()
    r, t, m0 = ops.out("r"), ops.out("t", 1), ops.out("m0", 1)
    a, kk = ops.inp("a"), ops.inp("k977", 1)
    R = [ops.ref("out", r, i) for i in range(8)]
    A = [ops.ref("in", a, i) for i in range(8)]
    T, M0, K = ops.ref("out", t), ops.ref("out", m0), ops.ref("in", kk)
    body = shifted(A, k, R) + [f"v_lshrrev_b32_e32 {T}, {32 - k}, {A[7]}"]
    body += k1_shl_fold(K, R, T, M0)
    return render(f"k1_shl{k}_asm(uint32_t r[8], const uint32_t a[8])", "uint32_t t, m0; const uint32_t k977 = 977u;",
                  ops, body, f"secp256k1 base field: r = 2^{k} a (mod p), values in [0, 2^256)",
                  clobbers='"vcc", "scc"')


def k1_add_shl(k):
    ops = Ops()
    r, bs, t, m0 = ops.out("r"), ops.out("bs"), ops.out("t", 1), ops.out("m0", 1)
    a, bb, kk = ops.inp("a"), ops.inp("b"), ops.inp("k977", 1)
    R = [ops.ref("out", r, i) for i in range(8)]
    BS = [ops.ref("out", bs, i) for i in range(8)]
    A = [ops.ref("in", a, i) for i in range(8)]
    B = [ops.ref("in", bb, i) for i in range(8)]
    T, M0, K = ops.ref("out", t), ops.ref("out", m0), ops.ref("in", kk)
    body = shifted(B, k, BS) + [f"v_lshrrev_b32_e32 {T}, {32 - k}, {B[7]}"]
    body += chain("v_add_co_u32_e32", "v_addc_co_u32_e32", R, A, BS)
    body += [f"v_addc_co_u32_e32 {T}, vcc, 0, {T}, vcc"]
    body += k1_shl_fold(K, R, T, M0)
    return render(f"k1_add_shl{k}_asm(uint32_t r[8], const uint32_t a[8], const uint32_t b[8])",
                  "uint32_t bs[8], t, m0; const uint32_t k977 = 977u;", ops, body,
                  f"secp256k1 base field: r = a + 2^{k} b (mod p), values in [0, 2^256)", clobbers='"vcc", "scc"')


def k1_normalize():
    ops = Ops()
    r, t = ops.out("r"), ops.out("t")
    a, k = ops.inp("a"), ops.inp("k977", 1)
    R = [ops.ref("out", r, i) for i in range(8)]
    T = [ops.ref("out", t, i) for i in range(8)]
    A = [ops.ref("in", a, i) for i in range(8)]
    K = ops.ref("in", k)
    body = [f"v_add_co_u32_e32 {T[0]}, vcc, {A[0]}, {K}", f"v_addc_co_u32_e32 {T[1]}, vcc, 1, {A[1]}, vcc"]
    body += [f"v_addc_co_u32_e32 {T[i]}, vcc, 0, {A[i]}, vcc" for i in range(2, 8)]
    body += [f"v_cndmask_b32_e32 {R[i]}, {A[i]}, {T[i]}, vcc" for i in range(8)]  # a >= p <=> a + c carries
    return render("k1_normalize_asm(uint32_t r[8], const uint32_t a[8])", "uint32_t t[8]; const uint32_t k977 = 977u;",
                  ops, body, "secp256k1: canonical residue of a in [0, 2^256)")


def mod_add():
    ops = Ops()
    r, t, cc = ops.out("r"), ops.out("t"), ops.out("c", 1)
    a, b, m = ops.inp("a"), ops.inp("b"), ops.inp("m")
    R = [ops.ref("out", r, i) for i in range(8)]
    T = [ops.ref("out", t, i) for i in range(8)]
    C = ops.ref("out", cc)
    A = [ops.ref("in", a, i) for i in range(8)]
    B = [ops.ref("in", b, i) for i in range(8)]
    M = [ops.ref("in", m, i) for i in range(8)]
    body = chain("v_add_co_u32_e32", "v_addc_co_u32_e32", R, A, B)
    body += [f"v_cndmask_b32_e64 {C}, 0, 1, vcc"]
    body += chain("v_sub_co_u32_e32", "v_subb_co_u32_e32", T, R, M)
    body += [f"v_subbrev_co_u32_e32 {C}, vcc, 0, {C}, vcc", f"v_cmp_gt_i32_e32 vcc, 0, {C}"]
    body += [f"v_cndmask_b32_e32 {R[i]}, {T[i]}, {R[i]}, vcc" for i in range(8)]  # keep a+b only if it was < m
    return render("mod_add_asm(uint32_t r[8], const uint32_t a[8], const uint32_t b[8], const uint32_t m[8])",
                  "uint32_t t[8], c;", ops, body, "r = a + b mod m (a, b < m)")


def mod_sub():
    ops = Ops()
    r, t, cc = ops.out("r"), ops.out("t"), ops.out("c", 1)
    a, b, m = ops.inp("a"), ops.inp("b"), ops.inp("m")
    R = [ops.ref("out", r, i) for i in range(8)]
    T = [ops.ref("out", t, i) for i in range(8)]
    C = ops.ref("out", cc)
    A = [ops.ref("in", a, i) for i in range(8)]
    B = [ops.ref("in", b, i) for i in range(8)]
    M = [ops.ref("in", m, i) for i in range(8)]
    body = chain("v_sub_co_u32_e32", "v_subb_co_u32_e32", R, A, B)
    body += [f"v_cndmask_b32_e64 {C}, 0, -1, vcc"]
    body += [f"v_and_b32_e32 {T[i]}, {C}, {M[i]}" for i in range(8)]
    body += chain("v_add_co_u32_e32", "v_addc_co_u32_e32", R, R, T)
    return render("mod_sub_asm(uint32_t r[8], const uint32_t a[8], const uint32_t b[8], const uint32_t m[8])",
                  "uint32_t t[8], c;", ops, body, "r = a - b mod m (a, b < m)")


def k1_reduce():
    """T = L + H 2^256  ->  L + H*977 + H*2^32 (mod p), three folds, result in [0, 2^256)."""
    ops = Ops()
    o = ops.out("o")
    u8, u9, cc, m0, m1 = (ops.out(n, 1) for n in ("u8", "u9", "c", "m0", "m1"))
    t, lo, hi, k = ops.inp("t", 16), ops.inp("lo"), ops.inp("hi"), ops.inp("k977", 1)
    O = [ops.ref("out", o, i) for i in range(8)]
    U8, U9, C, M0, M1 = (ops.ref("out", x) for x in (u8, u9, cc, m0, m1))
    Tt = [ops.ref("in", t, i) for i in range(16)]
    LO = [ops.ref("in", lo, i) for i in range(8)]
    HI = [ops.ref("in", hi, i) for i in range(8)]
    K = ops.ref("in", k)
    add, addc = "v_add_co_u32_e32", "v_addc_co_u32_e32"
    b = chain(add, addc, O, Tt[:8], LO)                     # L + lo
    b += [f"v_cndmask_b32_e64 {U8}, 0, 1, vcc"]
    b += [f"{add} {O[1]}, vcc, {O[1]}, {HI[0]}"]            # + hi << 32
    b += [f"{addc} {O[i]}, vcc, {O[i]}, {HI[i - 1]}, vcc" for i in range(2, 8)]
    b += [f"{addc} {U8}, vcc, {U8}, {HI[7]}, vcc", f"v_cndmask_b32_e64 {U9}, 0, 1, vcc"]
    b += [f"{add} {O[1]}, vcc, {O[1]}, {Tt[8]}"]            # + H << 32
    b += [f"{addc} {O[i]}, vcc, {O[i]}, {Tt[7 + i]}, vcc" for i in range(2, 8)]
    b += [f"{addc} {U8}, vcc, {U8}, {Tt[15]}, vcc", f"{addc} {U9}, vcc, 0, {U9}, vcc"]
    # second fold: top = u8 + u9 2^32 (< 2^34): + top*977 + top*2^32
    b += [f"v_mul_lo_u32 {M0}, {U8}, {K}", f"v_mul_hi_u32 {M1}, {U8}, {K}", f"v_mad_u32_u24 {M1}, {U9}, {K}, {M1}"]
    b += [f"{add} {O[0]}, vcc, {O[0]}, {M0}", f"{addc} {O[1]}, vcc, {O[1]}, {M1}, vcc",
          f"{addc} {O[2]}, vcc, {O[2]}, {U9}, vcc"]
    b += [f"{addc} {O[i]}, vcc, 0, {O[i]}, vcc" for i in range(3, 8)]
    b += [f"v_cndmask_b32_e64 {C}, 0, 1, vcc"]
    b += [f"{add} {O[1]}, vcc, {O[1]}, {U8}"]
    b += [f"{addc} {O[i]}, vcc, 0, {O[i]}, vcc" for i in range(2, 8)]
    b += [f"{addc} {C}, vcc, 0, {C}, vcc"]
    # third fold of the (at most one) wrap: + c*(2^32 + 977); cannot carry again
    b += [f"v_mul_u32_u24 {M0}, {C}, {K}", f"{add} {O[0]}, vcc, {O[0]}, {M0}", f"{addc} {O[1]}, vcc, {O[1]}, {C}, vcc"]
    b += [f"{addc} {O[i]}, vcc, 0, {O[i]}, vcc" for i in range(2, 8)]
    return render("k1_reduce_asm(uint32_t o[8], const uint32_t t[16], const uint32_t lo[8], const uint32_t hi[8])",
                  "uint32_t u8, u9, c, m0, m1; const uint32_t k977 = 977u;", ops, b,
                  "secp256k1: reduce a 512-bit product (lo/hi = H*977 split by v_mul_lo/hi) to [0, 2^256)")


def main():
    parts = ["// fe_asm.h -- GENERATED by tools/gen_fe_asm.py; do not edit by hand.",
             "// 256-bit carry chains as single inline-asm blocks, without the s_nop padding the compiler",
             "// inserts between dependent VCC carry steps on gfx950 (validated by tools/carrybench.hip).",
             "#pragma once", "#include <stdint.h>", "", "namespace bcosgpu {", "",
             k1_addsub(False), k1_addsub(True), k1_shl(1), k1_shl(2), k1_shl(3), k1_add_shl(1),
             k1_normalize(), k1_reduce(), mod_add(), mod_sub(), "}  // namespace bcosgpu", ""]
    with open(OUT, "w") as f:
        f.write("\n".join(parts))
    print("wrote", os.path.normpath(OUT))


if __name__ == "__main__":
    main()
