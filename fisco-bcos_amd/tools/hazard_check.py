#!/usr/bin/env python3
"""Static check of the gfx950 manually-inserted wait-state hazards over the built code.

CDNA3/CDNA4 (gfx940+) do not interlock these dependencies; the program must put enough independent
instructions or s_nop wait states between producer and consumer.  LLVM's hazard recognizer pads
compiler-generated code, but it does not look inside inline asm, and our field arithmetic
(csrc/fe_asm.h), the lane-trio DPP routing (csrc/ec26_trio.h, ecp26_trio.h) and the cooperative Keccak
(csrc/hash_device.h) are inline asm.  Checked rules (wait states between producer and consumer):

  sgpr     VALU writes an SGPR or VCC (the carry-out of v_add_co / v_addc_co / v_sub*_co /
           v_mad_u64_u32, a v_cmp result, v_readlane / v_readfirstlane)
           -> a VALU reads it (carry-in, v_cndmask mask, any SGPR source)                      2
  lanesel  VALU writes an SGPR -> v_readlane / v_writelane uses it as the lane select           4
  dpp      VALU writes a VGPR -> a DPP instruction (..._dpp) reads that VGPR                   2
  dppexec  VALU writes EXEC (v_cmpx) -> a DPP instruction                                      5
  permlane VALU writes a VGPR -> v_permlane16_swap / v_permlane32_swap reads it (both
           operands are read)                                                                  2
  readlane VALU writes a VGPR -> v_readlane / v_readfirstlane reads it                         1

SALU reads of a VALU-written SGPR are interlocked by the hardware and are not reported; VMEM / LDS
results are ordered by s_waitcnt, not wait states, and are not tracked.

This tool disassembles the gfx950 code object of each object file / shared library given, follows
every function's control flow (fall-through, conditional and unconditional branches, the
s_getpc/s_setpc long-branch idiom) and reports each consumer fewer wait states after its producer
than its rule needs.  Wait states: one per instruction, N + 1 for s_nop N.

usage: hazard_check.py [--quiet] FILE...   (exit status 1 when a violation is found)
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
NEED = 2  # wait states required between the VALU SGPR write and the VALU read
RULES = {"sgpr": 2, "lanesel": 4, "dpp": 2, "dppexec": 5, "permlane": 2, "readlane": 1}
HORIZON = max(RULES.values())  # a write older than this many wait states can no longer matter
EXEC = ("x",)

# VALU instructions whose SECOND operand is an SGPR (pair) destination (VOP3b / VOP2 carry-out forms)
_SDST2 = re.compile(r"^v_(add|sub|subrev|addc|subb|subbrev)_co_u32|^v_mad_[iu]64_[iu]32|^v_div_scale")
# VALU instructions whose FIRST operand is an SGPR destination
_SDST1 = re.compile(r"^v_cmp_|^v_readlane_b32|^v_readfirstlane_b32")
_SREG = re.compile(r"^(?:s(\d+)|s\[(\d+):(\d+)\]|(vcc)|(vcc_lo)|(vcc_hi))$")
_VREG = re.compile(r"^v(?:(\d+)|\[(\d+):(\d+)\])$")
_FUNC = re.compile(r"^([0-9a-f]+) <(.+)>:$")
_INST = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):(.*)$")
_TGT = re.compile(r"<(.+)\+0x([0-9a-f]+)>")


_TOK = {}


def _regs(tok):
    """(SGPR indices, VGPR indices) named by an operand token (vcc = 106/107); DPP / SDWA controls and
    VOP3 modifiers are ignored ('-|v3| row_shr:1' -> v3).  Memoised: tokens repeat across millions of
    instructions."""
    r = _TOK.get(tok)
    if r is not None:
        return r
    t = tok.strip()
    t = t.split(" ")[0].strip("-|") if t else ""
    sg, vg = (), ()
    m = _SREG.match(t)
    if m:
        if m.group(1):
            sg = (int(m.group(1)),)
        elif m.group(2):
            sg = tuple(range(int(m.group(2)), int(m.group(3)) + 1))
        elif m.group(4):
            sg = (106, 107)
        else:
            sg = (106,) if m.group(5) else (107,)
    else:
        m = _VREG.match(t)
        if m:
            vg = (int(m.group(1)),) if m.group(1) else tuple(range(int(m.group(2)), int(m.group(3)) + 1))
    _TOK[tok] = r = (sg, vg)
    return r


def sregs(tok):
    """SGPR indices named by an operand token (vcc = 106/107), or an empty tuple."""
    return _regs(tok)[0]


def vregs(tok):
    """VGPR indices named by an operand token, or an empty tuple."""
    return _regs(tok)[1]


def operands(s):
    return [t.strip() for t in s.split(",")] if s else []


def valu_defs_uses(mn, ops):
    """(SGPRs written, SGPRs read) by a VALU instruction."""
    if mn.startswith("v_cmpx"):
        return (), tuple(r for t in ops for r in sregs(t))
    if _SDST2.match(mn):
        defs = sregs(ops[1]) if len(ops) > 1 else ()
        uses = tuple(r for t in ops[2:] for r in sregs(t))
        return defs, uses
    if _SDST1.match(mn):
        defs = sregs(ops[0]) if ops else ()
        return defs, tuple(r for t in ops[1:] for r in sregs(t))
    return (), tuple(r for t in ops[1:] for r in sregs(t))


def valu_vgpr_defs_uses(mn, ops):
    """(VGPRs written, VGPRs read) by a VALU instruction."""
    if mn.startswith("v_permlane"):  # swaps: both operands read and written
        regs = tuple(r for t in ops for r in vregs(t))
        return regs, regs
    if mn.startswith("v_cmp") or _SDST1.match(mn) or mn.startswith("v_nop"):
        return (), tuple(r for t in ops for r in vregs(t))
    defs = vregs(ops[0]) if ops else ()
    uses = tuple(r for t in ops[1:] for r in vregs(t))
    if "_dpp" in mn:  # the destination is also read (the "old" value kept in masked-off lanes), as LLVM counts it
        uses += defs
    return defs, uses


_DISASM = {}


def functions(path):
    """Every function of a file's gfx950 code objects, disassembled (memoised per path and mtime)."""
    key = (os.path.abspath(path), os.path.getmtime(path))
    if key not in _DISASM:
        funcs = []
        with tempfile.TemporaryDirectory() as td:
            for co in extract_code_objects(path, td):
                funcs += disassemble(co)
        _DISASM.clear()
        _DISASM[key] = funcs
    return _DISASM[key]


def dpp_mnemonics(path):
    """Counter of the DPP / permlane mnemonics in a library's gfx950 code."""
    import collections
    return collections.Counter(mn for _, _, insts in functions(path) for _, mn, _ in insts
                               if "_dpp" in mn or "permlane" in mn)


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def extract_code_objects(path, tmpdir):
    """The gfx950 code objects inside a HIP host object / shared library: its .hip_fatbin section
    holds one clang offload bundle per linked translation unit."""
    fat = os.path.join(tmpdir, os.path.basename(path) + ".fatbin")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fat, path, os.devnull],
                   check=True, capture_output=True)
    blob = open(fat, "rb").read()
    out, pos = [], 0
    while True:
        pos = blob.find(MAGIC, pos)
        if pos < 0:
            return out
        n = struct.unpack_from("<Q", blob, pos + len(MAGIC))[0]
        q = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, q)
            triple = blob[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if triple == TARGET:
                co = os.path.join(tmpdir, "%d.co" % len(out))
                with open(co, "wb") as f:
                    f.write(blob[pos + off:pos + off + size])
                out.append(co)
        pos += len(MAGIC)


def disassemble(co):
    out = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co],
                         check=True, capture_output=True, text=True).stdout
    funcs, cur = [], None
    for line in out.splitlines():
        m = _FUNC.match(line)
        if m:
            cur = (m.group(2), int(m.group(1), 16), [])
            funcs.append(cur)
            continue
        m = _INST.match(line)
        if m and cur is not None:
            ops = m.group(2)
            t = _TGT.search(m.group(4))
            if t:  # branch target annotation follows the encoding comment
                ops += " <%s+0x%s>" % (t.group(1), t.group(2))
            cur[2].append((int(m.group(3), 16), m.group(1), ops))
    return funcs


_MNEM = {}


def _mclass(mn):
    """Per-mnemonic facts (memoised): (is VALU, SGPR-dest operand index or -1, VGPR-dest operand index
    or -1, permlane, dpp, readlane-like, writes exec)."""
    c = _MNEM.get(mn)
    if c is None:
        valu = mn.startswith("v_")
        perm = mn.startswith("v_permlane")
        sdst = 1 if _SDST2.match(mn) else 0 if (_SDST1.match(mn) and not mn.startswith("v_cmpx")) else -1
        vdst = -1 if (not valu or perm or mn.startswith("v_cmp") or _SDST1.match(mn) or mn.startswith("v_nop")) else 0
        lane = mn.startswith("v_readlane") or mn.startswith("v_readfirstlane")
        c = _MNEM[mn] = (valu, sdst, vdst, perm, "_dpp" in mn, lane, mn.startswith("v_cmpx"),
                         mn.startswith("v_readlane") or mn.startswith("v_writelane"))
    return c


def _parse(mn, ops):
    """([(state key, rule)] this instruction reads, [state keys] it writes) -- VALU only."""
    valu, sdst, vdst, perm, dpp, lane, cmpx, lanesel_op = _mclass(mn)
    if not valu:
        return (), ()
    toks = ops.split(",") if ops else []
    reads, writes = [], []
    lanesel = _regs(toks[-1])[0] if lanesel_op and toks else ()
    for k, tok in enumerate(toks):
        sg, vg = _regs(tok)
        if sg:
            if k == sdst:
                writes += [("s", r) for r in sg]
            else:
                reads += [(("s", r), "lanesel" if r in lanesel else "sgpr") for r in sg]
        if vg:
            if perm:
                reads += [(("v", r), "permlane") for r in vg]
                writes += [("v", r) for r in vg]
            elif k == vdst:
                writes += [("v", r) for r in vg]
                if dpp:  # the destination is also read (the "old" value of masked-off lanes), as LLVM counts it
                    reads += [(("v", r), "dpp") for r in vg]
            elif dpp:
                reads += [(("v", r), "dpp") for r in vg]
            elif lane:
                reads += [(("v", r), "readlane") for r in vg]
    if dpp:
        reads.append((EXEC, "dppexec"))
    if cmpx:
        writes.append(EXEC)
    return reads, writes


def _reads(mn, ops):
    return _parse(mn, ", ".join(ops))[0]


def _writes(mn, ops):
    return _parse(mn, ", ".join(ops))[1]


def check_function(name, start, insts):
    """Forward dataflow of {register: wait states since its VALU write (< HORIZON)} over the CFG.
    Violations: (function, offset, mnemonic, operands, register, wait states, rule)."""
    n = len(insts)
    index = {a: i for i, (a, _, _) in enumerate(insts)}
    succ = [None] * n
    for i, (a, mn, ops) in enumerate(insts):
        nxt = [i + 1] if i + 1 < n else []
        if mn in ("s_endpgm", "s_setpc_b64", "s_trap") or mn.startswith("s_endpgm"):
            succ[i] = []  # long branches: >= 3 SALU instructions precede the jump, nothing is in flight
        elif mn.startswith("s_branch") or mn.startswith("s_cbranch"):
            m = _TGT.search(ops)
            tgt = [index[start + int(m.group(2), 16)]] if m and start + int(m.group(2), 16) in index else []
            succ[i] = tgt if mn.startswith("s_branch") else nxt + tgt
        else:
            succ[i] = nxt
    parsed = [_parse(mn, ops) + (int(ops, 0) + 1 if mn == "s_nop" else 1,) for _, mn, ops in insts]
    targets = {s_ for i, nx in enumerate(succ) for s_ in nx if s_ != i + 1}
    entry = [None] * n
    entry[0] = {}
    work = [0]
    violations = []
    seen = set()
    while work:
        i = min(work)
        work.remove(i)
        # absolute time along this straight-line run: wt[r] = time its last VALU write completed
        t = 0
        wt = {r: -age for r, age in entry[i].items()}
        while True:
            reads, writes, ws = parsed[i]
            for key, rule in reads:
                w = wt.get(key)
                if w is not None and t - w < RULES[rule]:
                    a = insts[i][0]
                    if (a, key) not in seen:
                        seen.add((a, key))
                        reg = "exec" if key == EXEC else ("vcc" if key[0] == "s" and key[1] >= 106 else "%s%d" % key)
                        violations.append((name, a - start, insts[i][1], insts[i][2], reg, t - w, rule))
            t += ws
            for r in writes:
                wt[r] = t
            if len(wt) > 64:
                wt = {r: w for r, w in wt.items() if t - w < HORIZON}
            nxt = succ[i]
            if len(nxt) == 1 and nxt[0] == i + 1 and i + 1 not in targets:
                i += 1
                entry[i] = True  # reached only by this fall-through
                continue
            state = {r: t - w for r, w in wt.items() if t - w < HORIZON}
            for s_ in nxt:
                old = entry[s_]
                if old is None:
                    entry[s_] = dict(state)
                    if s_ not in work:
                        work.append(s_)
                else:
                    merged = dict(old)
                    for r, e in state.items():
                        if r not in merged or e < merged[r]:
                            merged[r] = e
                    if merged != old:
                        entry[s_] = merged
                        if s_ not in work:
                            work.append(s_)
            break
    return violations


def check_file(path, quiet=False):
    funcs = functions(path)
    total = 0
    report = []
    for name, start, insts in funcs:
        if not insts:
            continue
        v = check_function(name, start, insts)
        total += len(v)
        report.extend(v)
    if not quiet:
        for name, off, mn, ops, reg, e, rule in report[:50]:
            print("%s+0x%x: %s %s  reads %s %d wait state(s) after a VALU write (%s needs %d)" % (
                name, off, mn, ops, reg, e, rule, RULES[rule]))
        print("%s: %d functions, %d hazard(s)" % (os.path.basename(path), len(funcs), total))
    return total, len(funcs)


def _vmem_store(mn):
    return mn.startswith(("global_store", "buffer_store", "flat_store", "scratch_store"))


def fused_publish_order(path, kernel="merkle_fused_kernel"):
    """The ISA facts the one-launch Merkle kernel's cross-wave hand-off rests on (hash_kernels.hip,
    merkle_fused_kernel: relaxed agent-scope atomics, no cache-wide fence), per instance of `kernel`:
      (1) every counter atomic (global_atomic_*) is reached from the preceding node stores only through an
          `s_waitcnt vmcnt(0)`: scanning back from the atomic, that wait comes before any vector store, so
          the published node's write-through stores have been acknowledged before the counter moves;
      (2) the published nodes are written with sc1 stores (write-through past the XCD's L2) and the
          children are gathered with sc1 loads (missing the non-coherent L2), so the reader of a completed
          group sees memory, not a stale line.
    Returns (instances checked, list of (function, offset, problem))."""
    bad, seen = [], 0
    for name, start, insts in functions(path):
        if kernel not in name:
            continue
        seen += 1
        atomics = [i for i, (_, mn, _) in enumerate(insts) if mn.startswith("global_atomic")]
        if not atomics:
            bad.append((name, 0, "no counter atomic"))
        for i in atomics:
            j = i - 1
            while j >= 0 and not (insts[j][1] == "s_waitcnt" and "vmcnt(0)" in insts[j][2]):
                if _vmem_store(insts[j][1]):
                    bad.append((name, insts[i][0], "vector store %s at 0x%x reaches the atomic without "
                                "s_waitcnt vmcnt(0)" % (insts[j][1], insts[j][0])))
                    break
                j -= 1
            if j < 0:
                bad.append((name, insts[i][0], "no s_waitcnt vmcnt(0) before the atomic"))
        if not any(_vmem_store(mn) and "sc1" in ops for _, mn, ops in insts):
            bad.append((name, 0, "no sc1 (write-through) node store"))
        if not any(mn.startswith("global_load") and "sc1" in ops for _, mn, ops in insts):
            bad.append((name, 0, "no sc1 (coherent) child load"))
    return seen, bad


def main(argv):
    quiet = "--quiet" in argv
    files = [a for a in argv if not a.startswith("--")]
    bad = 0
    for f in files:
        t, _ = check_file(f, quiet)
        bad += t
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
