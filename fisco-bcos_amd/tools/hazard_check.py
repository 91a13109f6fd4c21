#!/usr/bin/env python3
"""Static check of the gfx950 "VALU writes SGPR -> VALU reads that SGPR" hazard over the built code.

CDNA3/CDNA4 (gfx940+) require two wait states between a VALU instruction that writes an SGPR or VCC
(the carry-out of v_add_co / v_addc_co / v_sub*_co / v_mad_u64_u32, a v_cmp result, v_readlane /
v_readfirstlane) and a later VALU instruction that reads it (a carry-in, a v_cndmask lane mask, or
any SGPR source operand).  The hardware does not interlock this dependency.  LLVM's hazard
recognizer pads compiler-generated code itself (s_nop 1 directly after the writer, s_nop 0 when one
instruction sits in between; `llc -mcpu=gfx950 -run-pass=post-RA-hazard-rec` on a two-instruction
MIR test shows it, and gfx90a gets no pad), but it does not look inside inline asm, so every carry
chain written as asm (csrc/fe_asm.h) must carry its own wait states.

This tool disassembles the gfx950 code object of each object file / shared library given, follows
every function's control flow (fall-through, conditional and unconditional branches, the
s_getpc/s_setpc long-branch idiom) and reports each VALU read of an SGPR fewer than two wait states
after a VALU write of it.  Wait states: one per instruction, N + 1 for s_nop N.  SALU reads of a
VALU-written SGPR are interlocked by the hardware and are not reported.

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

# VALU instructions whose SECOND operand is an SGPR (pair) destination (VOP3b / VOP2 carry-out forms)
_SDST2 = re.compile(r"^v_(add|sub|subrev|addc|subb|subbrev)_co_u32|^v_mad_[iu]64_[iu]32|^v_div_scale")
# VALU instructions whose FIRST operand is an SGPR destination
_SDST1 = re.compile(r"^v_cmp_|^v_readlane_b32|^v_readfirstlane_b32")
_SREG = re.compile(r"^(?:s(\d+)|s\[(\d+):(\d+)\]|(vcc)|(vcc_lo)|(vcc_hi))$")
_FUNC = re.compile(r"^([0-9a-f]+) <(.+)>:$")
_INST = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):(.*)$")
_TGT = re.compile(r"<(.+)\+0x([0-9a-f]+)>")


def sregs(tok):
    """SGPR indices named by an operand token (vcc = 106/107), or an empty tuple."""
    m = _SREG.match(tok)
    if not m:
        return ()
    if m.group(1):
        return (int(m.group(1)),)
    if m.group(2):
        return tuple(range(int(m.group(2)), int(m.group(3)) + 1))
    if m.group(4):
        return (106, 107)
    return (106,) if m.group(5) else (107,)


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


def check_function(name, start, insts):
    """Forward dataflow of {sgpr: wait states since its VALU write (< NEED)} over the CFG."""
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
    entry = [None] * n
    entry[0] = {}
    work = [0]
    violations = []
    seen = set()
    while work:
        i = min(work)
        work.remove(i)
        state = dict(entry[i])
        while True:
            a, mn, ops = insts[i]
            ws = 1
            if mn == "s_nop":
                ws = int(ops, 0) + 1
            defs = ()
            if mn.startswith("v_"):
                defs, uses = valu_defs_uses(mn, operands(ops))
                for r in uses:
                    if r in state and (a, r) not in seen:
                        seen.add((a, r))
                        violations.append((name, a - start, mn, ops, r, state[r]))
            # advance time, then record this instruction's writes
            state = {r: e + ws for r, e in state.items() if e + ws < NEED}
            for r in defs:
                state[r] = 0
            nxt = succ[i]
            if len(nxt) == 1 and nxt[0] == i + 1 and entry[i + 1] is None:
                i += 1
                entry[i] = dict(state)
                continue
            for s in nxt:
                old = entry[s]
                if old is None:
                    entry[s] = dict(state)
                    work.append(s)
                else:
                    merged = dict(old)
                    for r, e in state.items():
                        if r not in merged or e < merged[r]:
                            merged[r] = e
                    if merged != old:
                        entry[s] = merged
                        if s not in work:
                            work.append(s)
            break
    return violations


def check_file(path, quiet=False):
    funcs = []
    with tempfile.TemporaryDirectory() as td:
        for co in extract_code_objects(path, td):
            funcs += disassemble(co)
    total = 0
    report = []
    for name, start, insts in funcs:
        if not insts:
            continue
        v = check_function(name, start, insts)
        total += len(v)
        report.extend(v)
    if not quiet:
        for name, off, mn, ops, r, e in report[:50]:
            reg = "vcc" if r >= 106 else "s%d" % r
            print("%s+0x%x: %s %s  reads %s %d wait state(s) after a VALU write" % (name, off, mn, ops, reg, e))
        print("%s: %d functions, %d hazard(s)" % (os.path.basename(path), len(funcs), total))
    return total, len(funcs)


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
