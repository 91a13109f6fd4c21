#!/usr/bin/env python3
"""Generates fisco-bcos_amd/csrc/fe_asm.h: the 256-bit field primitives as single inline-asm blocks.

Why asm: each partial product is one v_mad_u64_u32 whose carry-out (an SGPR pair) feeds one
v_addc_co_u32, and each 256-bit add / sub is one VCC carry chain; the compiler's own lowering uses
compare-and-select carry detection instead.

Hazard: on gfx940+ a VALU write of an SGPR / VCC must be followed by two wait states before a VALU
reads it (carry-in, v_cndmask mask, SGPR source).  The hardware does not interlock it, LLVM pads its
own code (s_nop 1) but never looks inside an asm string.  Every block below is therefore run through
`schedule()`: a list scheduler over the block's dependence graph that interleaves independent
instructions (the lagged carry additions of a Comba column, the next column's products, the parallel
carry chains of the secp256k1 fold) between each SGPR writer and its reader and emits `s_nop` only
where nothing independent is left.  tools/hazard_check.py verifies the rule on the disassembly of the
built library (tests/test_hazards.py).

Pair halves: a 64-bit accumulator must be an aligned VGPR pair, and inline asm cannot name half of a
pair operand, so the product blocks use the fixed pairs v[0:1] and v[2:3] (declared clobbered).
"""
import os
import re

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "csrc", "fe_asm.h")
NEED = 2  # wait states between a VALU SGPR write and a VALU read of it

_PH = re.compile(r"%\[(\w+)\]")
_PHYS_V = re.compile(r"^v(\d+)$")
_PHYS_VP = re.compile(r"^v\[(\d+):(\d+)\]$")


def keys(x):
    """Dependence keys of one operand string."""
    m = _PH.fullmatch(x)
    if m:
        return [m.group(1)]
    if x == "vcc":
        return ["vcc"]
    m = _PHYS_V.match(x)
    if m:
        return [x]
    m = _PHYS_VP.match(x)
    if m:
        return ["v%d" % i for i in range(int(m.group(1)), int(m.group(2)) + 1)]
    return []


class Op:
    def __init__(self, text, vd=(), vu=(), sd=(), su=(), valu=True, cost=1, barrier=False, sjunk=()):
        self.text, self.valu, self.cost, self.barrier = text, valu, cost, barrier
        self.vd = [k for x in vd for k in keys(x)]
        self.vu = [k for x in vu for k in keys(x)]
        self.sd = [k for x in sd for k in keys(x)]
        self.su = [k for x in su for k in keys(x)]
        # SGPRs written but never read in the block (a discarded carry-out): no ordering constraint,
        # but their write time still counts for the exit pad
        self.sj = [k for x in sjunk for k in keys(x)]


def isv(x):
    return x.startswith("%[") or (x.startswith("v") and x != "vcc")


# ------------------------------------------------------------------ instruction helpers
def add(d, x, y, co):
    if co == "vcc" and isv(y):
        return Op(f"v_add_co_u32_e32 {d}, vcc, {x}, {y}", [d], [x, y], [co])
    return Op(f"v_add_co_u32_e64 {d}, {co}, {x}, {y}", [d], [x, y], [co])


def addc(d, x, y, ci, co):
    if co == "vcc" and ci == "vcc" and isv(y):
        return Op(f"v_addc_co_u32_e32 {d}, vcc, {x}, {y}, vcc", [d], [x, y], [co], [ci])
    return Op(f"v_addc_co_u32_e64 {d}, {co}, {x}, {y}, {ci}", [d], [x, y], [co], [ci])


def sub(d, x, y, co):
    if co == "vcc" and isv(y):
        return Op(f"v_sub_co_u32_e32 {d}, vcc, {x}, {y}", [d], [x, y], [co])
    return Op(f"v_sub_co_u32_e64 {d}, {co}, {x}, {y}", [d], [x, y], [co])


def subb(d, x, y, ci, co):
    if co == "vcc" and ci == "vcc" and isv(y):
        return Op(f"v_subb_co_u32_e32 {d}, vcc, {x}, {y}, vcc", [d], [x, y], [co], [ci])
    return Op(f"v_subb_co_u32_e64 {d}, {co}, {x}, {y}, {ci}", [d], [x, y], [co], [ci])


def subbrev(d, x, y, ci, co):  # d = y - x - ci
    if co == "vcc" and ci == "vcc" and isv(y):
        return Op(f"v_subbrev_co_u32_e32 {d}, vcc, {x}, {y}, vcc", [d], [x, y], [co], [ci])
    return Op(f"v_subbrev_co_u32_e64 {d}, {co}, {x}, {y}, {ci}", [d], [x, y], [co], [ci])


def mad(dp, co, x, y, acc):
    """dp (pair) = x * y + acc (pair or 0); co = carry-out of the 64-bit addition."""
    return Op(f"v_mad_u64_u32 {dp}, {co}, {x}, {y}, {acc}", [dp], [x, y, acc], [co], cost=2)


def madj(dp, junk, x, y, acc):
    """dp (pair) = x * y + acc with the carry-out discarded into `junk` (never read)."""
    return Op(f"v_mad_u64_u32 {dp}, {junk}, {x}, {y}, {acc}", [dp], [x, y, acc], cost=2, sjunk=[junk])


def mov(d, x):
    return Op(f"v_mov_b32_e32 {d}, {x}", [d], [x])


def cndmask(d, x, y, m):  # d = m ? y : x
    if m == "vcc" and isv(y):
        return Op(f"v_cndmask_b32_e32 {d}, {x}, {y}, vcc", [d], [x, y], [], [m])
    return Op(f"v_cndmask_b32_e64 {d}, {x}, {y}, {m}", [d], [x, y], [], [m])


def valu(text, d, *srcs, cost=1):
    return Op(text, [d], list(srcs), cost=cost)


def cmp_vcc(text, *srcs):
    return Op(text, [], list(srcs), ["vcc"])


def salu(text, sd=(), su=()):
    return Op(text, [], [], sd, su, valu=False)


def branch(text):
    return Op(text, valu=False, barrier=True)


def label(name):
    return Op(name + ":", valu=False, barrier=True)


# ------------------------------------------------------------------ scheduler
def schedule_segment(ops, wtime, t0):
    """List-schedule one straight-line segment.  wtime: key -> issue time of its last VALU SGPR write
    (carried in and out); returns (lines, end time)."""
    n = len(ops)
    preds = [set() for _ in range(n)]
    last_def, readers = {}, {}
    for i, o in enumerate(ops):
        for k in o.vu + o.su:
            if k in last_def:
                preds[i].add(last_def[k])
            readers.setdefault(k, []).append(i)
        for k in o.vd + o.sd:
            if k in last_def:
                preds[i].add(last_def[k])
            for r in readers.get(k, []):
                if r != i:
                    preds[i].add(r)
            last_def[k] = i
            readers[k] = []
    succs = [[] for _ in range(n)]
    for i in range(n):
        for p in preds[i]:
            succs[p].append(i)
    prio = [0] * n
    for i in reversed(range(n)):
        prio[i] = ops[i].cost + max((prio[s] for s in succs[i]), default=0)
    npred = [len(p) for p in preds]
    ready = [i for i in range(n) if npred[i] == 0]
    lines, t = [], t0

    def stall(i):  # wait states still missing before op i may issue
        o = ops[i]
        if not o.valu:
            return 0
        return max([0] + [wtime[k] + NEED + 1 - t for k in o.su if k in wtime])

    done = 0
    while done < n:
        ok = [i for i in ready if stall(i) == 0]
        if ok:
            i = max(ok, key=lambda j: (prio[j], -j))
        else:
            i = max(ready, key=lambda j: (prio[j], -j))
            w = stall(i)
            lines.append("s_nop %d" % (w - 1))
            t += w
        o = ops[i]
        lines.append(o.text)
        if o.valu:
            for k in o.sd + o.sj:
                wtime[k] = t
        else:
            for k in o.sd:
                wtime.pop(k, None)
        t += 1
        ready.remove(i)
        done += 1
        for s in succs[i]:
            npred[s] -= 1
            if npred[s] == 0:
                ready.append(s)
    return lines, t


def exit_pad(wtime, t):
    """Wait states still owed at the end of a block: code after the asm (hipcc's, or the next asm
    block) is not padded against writes inside it."""
    return max([0] + [v + NEED + 1 - t for v in wtime.values()])


def schedule(ops, s_inputs=()):
    """Schedule a block; branches and labels split it into segments kept in order.  The hazard state
    at a label is the merge (latest write) of the fall-through and every branch to it.  SGPR inputs
    count as written by a VALU just before the block (hipcc does not pad for the asm's reads), and
    the block ends with every SGPR write at least two wait states old."""
    lines, t = [], 2
    wtime = {k: 1 for x in s_inputs for k in keys(x)}
    pending = {}  # label -> [(time after the branch, wtime)] of the branches to it
    seg = []
    for pos, o in enumerate(ops + [None]):
        if o is None or o.barrier:
            out, t = schedule_segment(seg, wtime, t)
            lines += out
            seg = []
            if o is None:
                break
            if o.text.endswith(":"):
                if pos == len(ops) - 1:  # the block's last label: settle the fall-through path first
                    w = exit_pad(wtime, t)
                    if w:
                        lines.append("s_nop %d" % (w - 1))
                        t += w
                name = o.text[:-1]
                for tb, w in pending.pop(name, []):
                    for k, v in w.items():  # same age on the branch path as at its branch
                        wtime[k] = max(wtime.get(k, -99), t - (tb - v))
                lines.append(o.text)
            else:
                tgt = o.text.split()[-1].rstrip("f").rstrip("b")
                lines.append(o.text)
                t += 1
                pending.setdefault(tgt, []).append((t, dict(wtime)))
        else:
            seg.append(o)
    w = exit_pad(wtime, t)
    if w:
        lines.append("s_nop %d" % (w - 1))
    return lines


# ------------------------------------------------------------------ rendering
class Block:
    """One asm statement: operands (name -> (constraint, C++ expression)), locals, ops."""

    def __init__(self, sig, doc, locals_=""):
        self.sig, self.doc, self.locals = sig, doc, locals_
        self.outs, self.ins = [], []
        self.ops = []
        self.clobbers = []

    def vout(self, name, n=None, expr=None):
        return self._reg(self.outs, name, n, "=&v", expr)

    def sout(self, name, n=None, expr=None):
        return self._reg(self.outs, name, n, "=&s", expr)

    def vin(self, name, n=None, expr=None):
        return self._reg(self.ins, name, n, "v", expr)

    def sin(self, name, n=None, expr=None):
        return self._reg(self.ins, name, n, "s", expr)

    def _reg(self, lst, name, n, con, expr):
        if n is None:
            lst.append((name, con, expr or name))
            return "%[" + name + "]"
        res = []
        for i in range(n):
            nm = "%s%d" % (name, i)
            lst.append((nm, con, (expr or name) + "[%d]" % i))
            res.append("%[" + nm + "]")
        return res

    def emit(self, *ops):
        for o in ops:
            self.ops.append(o)

    def render(self):
        number = {}
        for i, (nm, _, _) in enumerate(self.outs + self.ins):
            number[nm] = i
        body = schedule(self.ops, ["%[" + nm + "]" for nm, c, _ in self.ins if c == "s"])
        body = [_PH.sub(lambda m: "%" + str(number[m.group(1)]), ln) for ln in body]
        s = ["// " + self.doc, "__device__ __forceinline__ void %s {" % self.sig]
        if self.locals:
            s.append("    " + self.locals)
        s.append("    asm volatile(")
        for i, ln in enumerate(body):
            s.append('        "%s%s' % (ln, '\\n\\t"' if i + 1 < len(body) else '"'))
        s.append("        : " + ", ".join('"%s"(%s)' % (c, e) for _, c, e in self.outs))
        s.append("        : " + ", ".join('"%s"(%s)' % (c, e) for _, c, e in self.ins))
        s.append("        : " + ", ".join('"%s"' % c for c in self.clobbers) + ");")
        s.append("}")
        nops = sum(1 for ln in body if ln.startswith("s_nop"))
        ninst = sum(1 for ln in body if not ln.endswith(":"))
        return "\n".join(s) + "\n", ninst, nops


# ------------------------------------------------------------------ 512-bit products
PA, PB = ("v[0:1]", "v0", "v1"), ("v[2:3]", "v2", "v3")


def comba_columns(blk, prods_of, skip_carry, ccs, junk, outs, first_col, last_col):
    """Column-wise (Comba) accumulation.  prods_of(k) = list of (x, y) operand pairs of column k.
    Column k accumulates in pair P (PA for even k, PB for odd); each product's carry-out is added
    into Q.hi (the other pair's high word = the next column's carry word) by a v_addc that the
    scheduler lags behind later products (rotating carry registers).  After the column: out[k] =
    P.lo, Q.lo = P.hi.  Returns the pair holding the last column."""
    n = 0
    for k in range(first_col, last_col + 1):
        P, Q = (PA, PB) if k % 2 == 0 else (PB, PA)
        prods = prods_of(k)
        qhi_init = False
        for idx, (x, y) in enumerate(prods):
            cc = ccs[n % len(ccs)]
            n += 1
            acc = "0" if (k == first_col and idx == 0) else P[0]
            if skip_carry(k, idx):
                blk.emit(mad(P[0], junk, x, y, acc))
                continue
            blk.emit(mad(P[0], cc, x, y, acc))
            blk.emit(addc(Q[2], Q[2] if qhi_init else "0", "0", cc, junk))
            qhi_init = True
        blk.emit(mov(outs[k], P[1]))
        if k < last_col:
            if not qhi_init:
                blk.emit(mov(Q[2], "0"))
            blk.emit(mov(Q[1], P[2]))
    return (PA, PB)[last_col % 2]


def gen_mul512():
    blk = Blk("mul_512_asm(uint32_t r[16], const uint32_t a[8], const uint32_t b[8])",
              "r = a * b (512-bit product), Comba order with lagged carry additions",
              "uint64_t c0, c1, c2, cj;")
    R = blk.vout("r", 16)
    cc = [blk.sout("c0"), blk.sout("c1"), blk.sout("c2")]
    cj = blk.sout("cj")
    A, B = blk.vin("a", 8), blk.vin("b", 8)
    blk.clobbers = ["v0", "v1", "v2", "v3"]

    def prods(k):
        return [(A[i], B[k - i]) for i in range(8) if 0 <= k - i < 8]

    # no carry out of 2^64 for: column 0 (acc = 0), the first product of column 1 (acc < 2^32), and
    # column 14 (its accumulator is the top 64 bits of the product)
    def skip(k, idx):
        return k == 0 or k == 14 or (k == 1 and idx == 0)

    last = comba_columns(blk, prods, skip, cc, cj, R, 0, 14)
    blk.emit(mov(R[15], last[2]))
    return blk


def gen_sqr512():
    blk = Blk("sqr_512_asm(uint32_t r[16], const uint32_t a[8])",
              "r = a^2 (512-bit): off-diagonal products once (Comba), doubled, plus the diagonal",
              "uint32_t t[16]; uint64_t c0, c1, c2, cj;")
    R = blk.vout("r", 16)
    T = blk.vout("t", 16)
    cc = [blk.sout("c0"), blk.sout("c1"), blk.sout("c2")]
    cj = blk.sout("cj")
    A = blk.vin("a", 8)
    blk.clobbers = ["v0", "v1", "v2", "v3", "vcc"]

    def prods(k):
        return [(A[i], A[k - i]) for i in range(8) if i < k - i < 8]

    # column 1: acc = 0; column 2: acc < 2^32 (no carry from its single product)
    def skip(k, idx):
        return k in (1, 2) and idx == 0

    last = comba_columns(blk, prods, skip, cc, cj, T, 1, 13)
    # t[14] = last.hi, t[15] = carry word of column 13 (the other pair's high word)
    other = PA if last is PB else PB
    blk.emit(mov(T[14], last[2]), mov(T[15], other[2]))
    # 2 t (t < 2^511): shifted words; t[0] = 0
    D = T  # doubled in place, high word first
    for k in range(15, 1, -1):
        blk.emit(valu(f"v_alignbit_b32 {D[k]}, {T[k]}, {T[k - 1]}, 31", D[k], T[k], T[k - 1]))
    blk.emit(valu(f"v_lshlrev_b32_e32 {D[1]}, 1, {T[1]}", D[1], T[1]))
    # + diagonal squares a_i^2 at words 2i, 2i+1 (one VCC chain); the squares alternate the pairs
    for i in range(8):
        P = PA if i % 2 == 0 else PB
        blk.emit(mad(P[0], cj, A[i], A[i], "0"))
        if i == 0:
            blk.emit(mov(R[0], P[1]))
            blk.emit(add(R[1], P[2], D[1], "vcc"))
        else:
            blk.emit(addc(R[2 * i], P[1], D[2 * i], "vcc", "vcc"))
            blk.emit(addc(R[2 * i + 1], P[2], D[2 * i + 1], "vcc", "vcc"))
    return blk


Blk = Block


# ------------------------------------------------------------------ secp256k1 reduction and add/sub
def gen_k1_reduce():
    """T = L + H 2^256 -> L + H 977 + H 2^32 (mod p) in [0, 2^256).  The products H_k * 977 go to the
    fixed pairs v[0:1] / v[2:3] in turn; three carry chains (L + lo; + hi << 32; + H << 32) on three
    carry registers, lagged by the scheduler; then top = u8 + u9 2^32 (< 2^34) is folded into words
    0-2 and the carry tail into words 3-7 (and a last fold of 2^256), probability ~2^-30 per lane, is
    branched over."""
    blk = Blk("k1_reduce_asm(uint32_t o[8], const uint32_t t[16])",
              "secp256k1: reduce a 512-bit product to [0, 2^256)",
              "uint32_t u8, u9, f0, f1, f2; uint64_t cx, cy, cj; uint32_t k977 = 977u;")
    O = blk.vout("o", 8)
    U8, U9, F0, F1, F2 = (blk.vout(x) for x in ("u8", "u9", "f0", "f1", "f2"))
    CX, CY, CJ = blk.sout("cx"), blk.sout("cy"), blk.sout("cj")
    Tt = blk.vin("t", 16)
    K = blk.vin("k977")
    blk.clobbers = ["v0", "v1", "v2", "v3", "vcc", "scc"]
    X, Y, Z = "vcc", CX, CY
    LO, HI = [], []
    for k in range(8):  # H_k * 977 < 2^42
        P = PA if k % 2 == 0 else PB
        LO.append(P[1])
        HI.append(P[2])
    # program order interleaves each product with its consumers, so the WAR edges on the two pairs
    # are explicit and the scheduler may only reorder within them
    for k in range(8):
        P = PA if k % 2 == 0 else PB
        blk.emit(mad(P[0], CJ, Tt[8 + k], K, "0"))
        blk.emit(add(O[0], Tt[0], LO[0], X) if k == 0 else addc(O[k], Tt[k], LO[k], X, X))
        if k == 0:
            pass
        elif k == 1:
            blk.emit(add(O[1], O[1], HI[0], Y))
        else:
            blk.emit(addc(O[k], O[k], HI[k - 1], Y, Y))
    blk.emit(addc(U8, "0", "0", X, X))                      # u8 = carry of L + lo
    blk.emit(addc(U8, U8, HI[7], Y, Y))                     # + hi_7 (word 8)
    blk.emit(addc(U9, "0", "0", Y, Y))
    blk.emit(add(O[1], O[1], Tt[8], Z))                      # + H << 32
    for i in range(2, 8):
        blk.emit(addc(O[i], O[i], Tt[7 + i], Z, Z))
    blk.emit(addc(U8, U8, Tt[15], Z, Z))
    blk.emit(addc(U9, U9, "0", Z, Z))
    # fold top = u8 + u9 2^32: top*977 + top*2^32 = f0 + f1 2^32 + f2 2^64
    blk.emit(valu(f"v_mul_lo_u32 {F0}, {U8}, {K}", F0, U8, K))
    blk.emit(valu(f"v_mul_hi_u32 {F1}, {U8}, {K}", F1, U8, K))
    blk.emit(valu(f"v_mad_u32_u24 {F1}, {U9}, {K}, {F1}", F1, U9, K, F1))  # + u9*977 (< 2^12)
    blk.emit(add(F1, F1, U8, Y))
    blk.emit(addc(F2, U9, "0", Y, Y))  # f2 = u9 + carry, <= 4
    blk.emit(add(O[0], O[0], F0, X))
    blk.emit(addc(O[1], O[1], F1, X, X))
    blk.emit(addc(O[2], O[2], F2, X, X))
    blk.emit(salu("s_cmp_eq_u64 vcc, 0", [], ["vcc"]))
    blk.emit(branch("s_cbranch_scc1 2f"))
    # rare tail: propagate into words 3-7; a carry out of 2^256 folds once more (cannot carry again)
    for i in range(3, 8):
        blk.emit(addc(O[i], "0", O[i], X, X))
    blk.emit(cndmask(F0, "0", K, X))
    blk.emit(cndmask(F1, "0", "1", X))
    blk.emit(add(O[0], O[0], F0, X))
    blk.emit(addc(O[1], O[1], F1, X, X))
    for i in range(2, 8):
        blk.emit(addc(O[i], "0", O[i], X, X))
    blk.emit(label("2"))
    return blk


def k1_fold_tail(blk, R, T0, T1, K, C, sub_):
    """After a 256-bit add (sub) whose carry (borrow) out of 2^256 is in C: fold +- C (2^32 + 977)
    into words 0-1, branch over the carry tail into words 2-7 unless some lane of the wave needs it."""
    f, c, prop = ((sub, subb, subbrev) if sub_ else (add, addc, addc))

    def fold():
        blk.emit(cndmask(T0, "0", K, C))
        blk.emit(cndmask(T1, "0", "1", C))
        blk.emit(f(R[0], R[0], T0, "vcc"))
        blk.emit(c(R[1], R[1], T1, "vcc", "vcc"))

    fold()
    blk.emit(salu("s_cmp_eq_u64 vcc, 0", [], ["vcc"]))
    blk.emit(branch("s_cbranch_scc1 2f"))
    for i in range(2, 8):
        blk.emit(prop(R[i], "0", R[i], "vcc", "vcc") if not sub_ else subbrev(R[i], "0", R[i], "vcc", "vcc"))
    fold()
    for i in range(2, 8):
        blk.emit(prop(R[i], "0", R[i], "vcc", "vcc") if not sub_ else subbrev(R[i], "0", R[i], "vcc", "vcc"))
    blk.emit(label("2"))


def gen_k1_addsub(sub_):
    name = "k1_sub_asm" if sub_ else "k1_add_asm"
    blk = Blk(f"{name}(uint32_t r[8], const uint32_t a[8], const uint32_t b[8])",
              f"secp256k1 base field: r = a {'-' if sub_ else '+'} b (mod p), values in [0, 2^256)",
              "uint32_t t0, t1; uint32_t k977 = 977u;")
    R = blk.vout("r", 8)
    T0, T1 = blk.vout("t0"), blk.vout("t1")
    A, B = blk.vin("a", 8), blk.vin("b", 8)
    K = blk.vin("k977")
    blk.clobbers = ["vcc", "scc"]
    f, c = (sub, subb) if sub_ else (add, addc)
    blk.emit(f(R[0], A[0], B[0], "vcc"))
    for i in range(1, 8):
        blk.emit(c(R[i], A[i], B[i], "vcc", "vcc"))
    k1_fold_tail(blk, R, T0, T1, K, "vcc", sub_)
    return blk


def shifted(blk, X, k, dst):
    blk.emit(valu(f"v_lshlrev_b32_e32 {dst[0]}, {k}, {X[0]}", dst[0], X[0]))
    for i in range(1, 8):
        blk.emit(valu(f"v_alignbit_b32 {dst[i]}, {X[i]}, {X[i - 1]}, {32 - k}", dst[i], X[i], X[i - 1]))


def k1_shl_fold(blk, R, T, M0, K):
    """R + T * 2^256 -> R + T (2^32 + 977) (mod p), T < 2^24: words 0-1 inline, the carry tail
    (probability ~2^-32 per lane) branched over unless some lane of the wave needs it."""
    blk.emit(valu(f"v_mul_u32_u24_e32 {M0}, {K}, {T}", M0, K, T))
    blk.emit(add(R[0], R[0], M0, "vcc"))
    blk.emit(addc(R[1], R[1], T, "vcc", "vcc"))
    blk.emit(salu("s_cmp_eq_u64 vcc, 0", [], ["vcc"]))
    blk.emit(branch("s_cbranch_scc1 2f"))
    for i in range(2, 8):
        blk.emit(addc(R[i], "0", R[i], "vcc", "vcc"))
    # a carry out of 2^256 here leaves R < T (2^32 + 977) < 2^57: fold once more (no further carry)
    blk.emit(cndmask(M0, "0", K, "vcc"))
    blk.emit(cndmask(T, "0", "1", "vcc"))
    blk.emit(add(R[0], R[0], M0, "vcc"))
    blk.emit(addc(R[1], R[1], T, "vcc", "vcc"))
    for i in range(2, 8):
        blk.emit(addc(R[i], "0", R[i], "vcc", "vcc"))
    blk.emit(label("2"))


def gen_k1_shl(k):
    blk = Blk(f"k1_shl{k}_asm(uint32_t r[8], const uint32_t a[8])",
              f"secp256k1 base field: r = 2^{k} a (mod p), values in [0, 2^256)",
              "uint32_t t, m0; uint32_t k977 = 977u;")
    R = blk.vout("r", 8)
    T, M0 = blk.vout("t"), blk.vout("m0")
    A = blk.vin("a", 8)
    K = blk.vin("k977")
    blk.clobbers = ["vcc", "scc"]
    shifted(blk, A, k, R)
    blk.emit(valu(f"v_lshrrev_b32_e32 {T}, {32 - k}, {A[7]}", T, A[7]))
    k1_shl_fold(blk, R, T, M0, K)
    return blk


def gen_k1_add_shl(k):
    blk = Blk(f"k1_add_shl{k}_asm(uint32_t r[8], const uint32_t a[8], const uint32_t b[8])",
              f"secp256k1 base field: r = a + 2^{k} b (mod p), values in [0, 2^256)",
              "uint32_t bs[8], t, m0; uint32_t k977 = 977u;")
    R = blk.vout("r", 8)
    BS = blk.vout("bs", 8)
    T, M0 = blk.vout("t"), blk.vout("m0")
    A, B = blk.vin("a", 8), blk.vin("b", 8)
    K = blk.vin("k977")
    blk.clobbers = ["vcc", "scc"]
    shifted(blk, B, k, BS)
    blk.emit(valu(f"v_lshrrev_b32_e32 {T}, {32 - k}, {B[7]}", T, B[7]))
    blk.emit(add(R[0], A[0], BS[0], "vcc"))
    for i in range(1, 8):
        blk.emit(addc(R[i], A[i], BS[i], "vcc", "vcc"))
    blk.emit(addc(T, "0", T, "vcc", "vcc"))
    k1_shl_fold(blk, R, T, M0, K)
    return blk


def gen_k1_normalize():
    blk = Blk("k1_normalize_asm(uint32_t r[8], const uint32_t a[8])", "secp256k1: canonical residue of a in [0, 2^256)",
              "uint32_t t[8]; uint32_t k977 = 977u;")
    R = blk.vout("r", 8)
    T = blk.vout("t", 8)
    A = blk.vin("a", 8)
    K = blk.vin("k977")
    blk.clobbers = ["vcc"]
    blk.emit(add(T[0], A[0], K, "vcc"))
    blk.emit(addc(T[1], "1", A[1], "vcc", "vcc"))
    for i in range(2, 8):
        blk.emit(addc(T[i], "0", A[i], "vcc", "vcc"))
    for i in range(8):  # a >= p <=> a + (2^32 + 977) carries
        blk.emit(cndmask(R[i], A[i], T[i], "vcc"))
    return blk


def gen_mod_add():
    blk = Blk("mod_add_asm(uint32_t r[8], const uint32_t a[8], const uint32_t b[8], const uint32_t m[8])",
              "r = a + b mod m (a, b < m): a + b and a + b - m as two lagged carry chains",
              "uint32_t t[8], c; uint64_t cs;")
    R = blk.vout("r", 8)
    T = blk.vout("t", 8)
    C = blk.vout("c")
    CS = blk.sout("cs")
    A, B, M = blk.vin("a", 8), blk.vin("b", 8), blk.vin("m", 8)
    blk.clobbers = ["vcc"]
    blk.emit(add(R[0], A[0], B[0], "vcc"))
    for i in range(1, 8):
        blk.emit(addc(R[i], A[i], B[i], "vcc", "vcc"))
    blk.emit(addc(C, "0", "0", "vcc", "vcc"))
    blk.emit(sub(T[0], R[0], M[0], CS))
    for i in range(1, 8):
        blk.emit(subb(T[i], R[i], M[i], CS, CS))
    blk.emit(subbrev(C, "0", C, CS, CS))      # c - borrow: < 0 iff a + b < m
    blk.emit(cmp_vcc(f"v_cmp_gt_i32_e32 vcc, 0, {C}", C))
    for i in range(8):  # keep a + b only if it was < m
        blk.emit(cndmask(R[i], T[i], R[i], "vcc"))
    return blk


def gen_mod_sub():
    blk = Blk("mod_sub_asm(uint32_t r[8], const uint32_t a[8], const uint32_t b[8], const uint32_t m[8])",
              "r = a - b mod m (a, b < m)", "uint32_t t[8], c;")
    R = blk.vout("r", 8)
    T = blk.vout("t", 8)
    C = blk.vout("c")
    A, B, M = blk.vin("a", 8), blk.vin("b", 8), blk.vin("m", 8)
    blk.clobbers = ["vcc"]
    blk.emit(sub(R[0], A[0], B[0], "vcc"))
    for i in range(1, 8):
        blk.emit(subb(R[i], A[i], B[i], "vcc", "vcc"))
    blk.emit(cndmask(C, "0", "-1", "vcc"))
    for i in range(8):
        blk.emit(valu(f"v_and_b32_e32 {T[i]}, {C}, {M[i]}", T[i], C, M[i]))
    blk.emit(add(R[0], R[0], T[0], "vcc"))
    for i in range(1, 8):
        blk.emit(addc(R[i], R[i], T[i], "vcc", "vcc"))
    return blk


# ------------------------------------------------------------------ 10 x 26-bit secp256k1 field
def gen_fe26(square):
    """fe26_mul / fe26_sqr (fe26.h): 19 product columns as two v_mad_u64_u32 chains the scheduler
    interleaves -- the high chain (columns 10..18, pair v[0:1]) carries into 26-bit limbs H0..H8 and
    H9; the low chain (columns 0..9, pair v[2:3]) adds H_j * R0 and H_(j-1) * 2^10 (2^260 = 2^36 + R0)
    to column j before cutting limb j -- then the carry x out of bit 256 and the H9 terms fold into
    limbs 0..3.  Carries enter each column as the accumulator the first product adds to, so a column
    costs its products plus one v_and and one 64-bit shift."""
    name = "fe26_sqr_asm(uint32_t r[10], const uint32_t a[10])" if square else \
        "fe26_mul_asm(uint32_t r[10], const uint32_t a[10], const uint32_t b[10])"
    blk = Blk(name, "r = a^2 mod p (fe26, inputs m <= 16, output m = 1)" if square else
              "r = a * b mod p (fe26, inputs m <= 16, output m = 1)",
              "uint32_t h[10], d[9]; uint64_t jh, jl; uint32_t kR0 = 0x3d10u, k1024 = 1024u, "
              "kR0x = 0x3d10u << 10, k20 = 1u << 20, k977 = 977u;" if square else
              "uint32_t h[10]; uint64_t jh, jl; uint32_t kR0 = 0x3d10u, k1024 = 1024u, "
              "kR0x = 0x3d10u << 10, k20 = 1u << 20, k977 = 977u;")
    R = blk.vout("r", 10)
    H = blk.vout("h", 10)
    D = blk.vout("d", 9) if square else None
    JH, JL = blk.sout("jh"), blk.sout("jl")
    A = blk.vin("a", 10)
    B = A if square else blk.vin("b", 10)
    kR0, k1024, kR0x, k20, k977 = (blk.sin(x) for x in ("kR0", "k1024", "kR0x", "k20", "k977"))
    blk.clobbers = ["v0", "v1", "v2", "v3"]
    HP, LP = ("v[0:1]", "v0", "v1"), ("v[2:3]", "v2", "v3")
    M26, M22 = "0x3ffffff", "0x3fffff"
    if square:
        for i in range(9):
            blk.emit(valu(f"v_lshlrev_b32_e32 {D[i]}, 1, {A[i]}", D[i], A[i]))

    def prods(k):
        if not square:
            return [(A[i], B[k - i]) for i in range(10) if 0 <= k - i < 10]
        out = [(D[i], A[k - i]) for i in range(10) if i < k - i < 10]
        if k % 2 == 0:
            out.append((A[k // 2], A[k // 2]))
        return out

    def column(P, junk, k, first):
        ps = prods(k)
        for idx, (x, y) in enumerate(ps):
            blk.emit(madj(P[0], junk, x, y, "0" if (first and idx == 0) else P[0]))

    # both chains in one stream; the scheduler interleaves them
    for j in range(10):
        if j < 9:  # high column 10 + j -> H_j
            column(HP, JH, 10 + j, j == 0)
            blk.emit(valu(f"v_and_b32_e32 {H[j]}, {M26}, {HP[1]}", H[j], HP[1]))
            blk.emit(valu(f"v_lshrrev_b64 {HP[0]}, 26, {HP[0]}", HP[0], HP[0]))
            if j == 8:
                blk.emit(mov(H[9], HP[1]))  # H9 < 2^27
        column(LP, JL, j, j == 0)
        blk.emit(madj(LP[0], JL, H[j], kR0, LP[0]))
        if j >= 1:
            blk.emit(madj(LP[0], JL, H[j - 1], k1024, LP[0]))
        if j < 9:
            blk.emit(valu(f"v_and_b32_e32 {R[j]}, {M26}, {LP[1]}", R[j], LP[1]))
            blk.emit(valu(f"v_lshrrev_b64 {LP[0]}, 26, {LP[0]}", LP[0], LP[0]))
        else:
            blk.emit(valu(f"v_and_b32_e32 {R[9]}, {M22}, {LP[1]}", R[9], LP[1]))
            blk.emit(valu(f"v_lshrrev_b64 {LP[0]}, 22, {LP[0]}", LP[0], LP[0]))  # x < 2^42
    # limb 0 += x 977 + H9 R0 2^10;  limb 1 += x 2^6 + H9 2^20;  carries through limb 3
    blk.emit(madj(HP[0], JH, H[9], kR0x, "0"))
    blk.emit(madj(HP[0], JH, LP[1], k977, HP[0]))
    blk.emit(valu(f"v_mad_u32_u24 {HP[2]}, {LP[2]}, {k977}, {HP[2]}", HP[2], LP[2], k977, HP[2]))
    blk.emit(madj(HP[0], JH, R[0], "1", HP[0]))
    blk.emit(valu(f"v_and_b32_e32 {R[0]}, {M26}, {HP[1]}", R[0], HP[1]))
    blk.emit(valu(f"v_lshrrev_b64 {HP[0]}, 26, {HP[0]}", HP[0], HP[0]))
    # (v_lshl_add_u64 takes shift amounts 0..4 only: shift x first)
    blk.emit(valu(f"v_lshlrev_b64 {LP[0]}, 6, {LP[0]}", LP[0], LP[0]))
    blk.emit(valu(f"v_lshl_add_u64 {HP[0]}, {LP[0]}, 0, {HP[0]}", HP[0], LP[0], HP[0]))
    blk.emit(madj(HP[0], JH, H[9], k20, HP[0]))
    blk.emit(madj(HP[0], JH, R[1], "1", HP[0]))
    blk.emit(valu(f"v_and_b32_e32 {R[1]}, {M26}, {HP[1]}", R[1], HP[1]))
    blk.emit(valu(f"v_alignbit_b32 {HP[1]}, {HP[2]}, {HP[1]}, 26", HP[1], HP[2], HP[1]))  # < 2^23
    blk.emit(valu(f"v_add_u32_e32 {HP[1]}, {R[2]}, {HP[1]}", HP[1], R[2], HP[1]))
    blk.emit(valu(f"v_and_b32_e32 {R[2]}, {M26}, {HP[1]}", R[2], HP[1]))
    blk.emit(valu(f"v_lshrrev_b32_e32 {HP[1]}, 26, {HP[1]}", HP[1], HP[1]))
    blk.emit(valu(f"v_add_u32_e32 {R[3]}, {R[3]}, {HP[1]}", R[3], R[3], HP[1]))
    return blk


def gen_fp26(square):
    """fp26_mul / fp26_sqr (fp26.h, SM2, Montgomery R = 2^286): the 19 product columns in the fixed
    pairs v[2k:2k+1] (column k), then eleven Montgomery digits, each m = low 26 bits of its column, the
    column's floor-carry (64-bit arithmetic shift) into the next, and m's four shifted multiply-adds
    (+2^12 at k+2, -2^18 at k+3, -2^16 at k+8, +2^22 at k+9) as signed / unsigned v_mad; the result is
    columns 11..20 carried into 26-bit limbs.  Physical registers because inline asm cannot name half of a
    64-bit operand; v0..v47 are declared clobbered."""
    name = "fp26_sqr_asm(uint32_t r[10], const uint32_t a[10])" if square else \
        "fp26_mul_asm(uint32_t r[10], const uint32_t a[10], const uint32_t b[10])"
    blk = Blk(name, "r = a^2 R^-1 mod p (SM2, fp26: inputs m <= 15, output m = 1)" if square else
              "r = a b R^-1 mod p (SM2, fp26: inputs m <= 15, output m = 1)",
              ("uint32_t d[9]; " if square else "") + "uint64_t jp, jr; uint32_t k12 = 1u << 12, kn18 = 0xfffc0000u, "
              "kn16 = 0xffff0000u, k22 = 1u << 22;")
    R = blk.vout("r", 10)
    D = blk.vout("d", 9) if square else None
    JP, JR = blk.sout("jp"), blk.sout("jr")
    A = blk.vin("a", 10)
    B = A if square else blk.vin("b", 10)
    k12, kn18, kn16, k22 = (blk.sin(x) for x in ("k12", "kn18", "kn16", "k22"))
    blk.clobbers = ["v%d" % i for i in range(48)]
    C = [("v[%d:%d]" % (2 * k, 2 * k + 1), "v%d" % (2 * k), "v%d" % (2 * k + 1)) for k in range(21)]
    MT = ["v42", "v43"]
    TT = ["v[44:45]", "v[46:47]"]
    M26, M22 = "0x3ffffff", "0x3fffff"
    if square:
        for i in range(9):
            blk.emit(valu(f"v_lshlrev_b32_e32 {D[i]}, 1, {A[i]}", D[i], A[i]))

    def prods(k):
        if not square:
            return [(A[i], B[k - i]) for i in range(10) if 0 <= k - i < 10]
        out = [(D[i], A[k - i]) for i in range(10) if i < k - i < 10]
        if k % 2 == 0:
            out.append((A[k // 2], A[k // 2]))
        return out

    for k in range(19):
        for idx, (x, y) in enumerate(prods(k)):
            blk.emit(madj(C[k][0], JP, x, y, "0" if idx == 0 else C[k][0]))
    started = set(range(19))

    def acc_into(k, x, const, signed):
        op = "v_mad_i64_i32" if signed else "v_mad_u64_u32"
        src = C[k][0] if k in started else "0"
        started.add(k)
        blk.emit(Op(f"{op} {C[k][0]}, {JR}, {x}, {const}, {src}", [C[k][0]], [x, const] + ([] if src == "0" else [src]),
                    cost=2, sjunk=[JR]))

    for i in range(11):
        m, t = MT[i % 2], TT[i % 2]
        blk.emit(valu(f"v_and_b32_e32 {m}, {M26}, {C[i][1]}", m, C[i][1]))
        blk.emit(valu(f"v_ashrrev_i64 {t}, 26, {C[i][0]}", t, C[i][0]))
        blk.emit(valu(f"v_lshl_add_u64 {C[i + 1][0]}, {t}, 0, {C[i + 1][0]}", C[i + 1][0], t, C[i + 1][0]))
        acc_into(i + 2, m, k12, False)
        acc_into(i + 3, m, kn18, True)
        acc_into(i + 8, m, kn16, True)
        acc_into(i + 9, m, k22, False)
    for j in range(11, 20):
        t = TT[j % 2]
        blk.emit(valu(f"v_and_b32_e32 {R[j - 11]}, {M26}, {C[j][1]}", R[j - 11], C[j][1]))
        blk.emit(valu(f"v_ashrrev_i64 {t}, 26, {C[j][0]}", t, C[j][0]))
        if j < 19:
            blk.emit(valu(f"v_lshl_add_u64 {C[j + 1][0]}, {t}, 0, {C[j + 1][0]}", C[j + 1][0], t, C[j + 1][0]))
        else:
            blk.emit(mov(R[9], t.replace("v[44:45]", "v44").replace("v[46:47]", "v46")))  # c20 = the carry, < 2^23
    return blk


def main():
    parts = ["// fe_asm.h -- GENERATED by tools/gen_fe_asm.py; do not edit by hand.",
             "// 256-bit field primitives as single inline-asm blocks, scheduled so that every VALU read of",
             "// an SGPR / VCC comes at least two wait states after the VALU write of it (the gfx940+ hazard",
             "// hipcc pads in its own code but not inside asm); checked on the built library by",
             "// tools/hazard_check.py.  Per block: instructions / s_nop count.",
             "#pragma once", "#include <stdint.h>", "", "namespace bcosgpu {", ""]
    stats = []
    for g in (gen_mul512, gen_sqr512, gen_k1_reduce, lambda: gen_k1_addsub(False), lambda: gen_k1_addsub(True),
              lambda: gen_k1_shl(1), lambda: gen_k1_shl(2), lambda: gen_k1_shl(3), lambda: gen_k1_add_shl(1),
              gen_k1_normalize, gen_mod_add, gen_mod_sub, lambda: gen_fe26(False), lambda: gen_fe26(True), lambda: gen_fp26(False), lambda: gen_fp26(True)):
        blk = g()
        text, ninst, nops = blk.render()
        name = blk.sig.split("(")[0]
        stats.append((name, ninst, nops))
        parts.append("// %d instructions, %d s_nop" % (ninst, nops))
        parts.append(text)
    parts += ["}  // namespace bcosgpu", ""]
    with open(OUT, "w") as f:
        f.write("\n".join(parts))
    for s in stats:
        print("%-20s %4d instructions %3d s_nop" % s)
    print("wrote", os.path.normpath(OUT))


if __name__ == "__main__":
    main()
