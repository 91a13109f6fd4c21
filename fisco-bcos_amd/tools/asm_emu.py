#!/usr/bin/env python3
"""A small emulator for the straight-line integer VALU subset the generated fe_asm.h blocks use, one
lane at a time: lets the CPU suite run a generated block on known inputs (tests/test_fe26.py) without a
GPU.  Blocks are read from the header text: the asm string lines, then the output / input operand lists
give %N -> (kind, C++ expression)."""
import re

M32 = (1 << 32) - 1
M64 = (1 << 64) - 1


def parse_block(header_text, func):
    """-> (instructions, outs, ins): operand i is outs[i] for i < len(outs), else ins[i - len(outs)]."""
    i = header_text.index("void %s(" % func)
    body = header_text[i:header_text.index("\n}\n", i)]
    lines = re.findall(r'^\s*"(.*?)(?:\\n\\t)?"\s*$', body, re.M)
    ops = re.findall(r"^\s*: (.*)$", body, re.M)
    outs = re.findall(r'"(=&?[vs])"\(([^)]*)\)', ops[0])
    ins = re.findall(r'"([vs])"\(([^)]*)\)', ops[1])
    return [ln for ln in lines if ln], outs, ins


class Lane:
    def __init__(self, operands):
        self.r = {}  # register name -> 32-bit value
        self.operands = operands  # %N -> register name

    def _name(self, x):
        x = x.strip()
        if x.startswith("%"):
            return self.operands[int(x[1:])]
        return x

    def get(self, x):
        x = x.strip()
        m = re.fullmatch(r"v\[(\d+):(\d+)\]", x)
        if m:
            lo = int(m.group(1))
            return self.r.get("v%d" % lo, 0) | (self.r.get("v%d" % (lo + 1), 0) << 32)
        if re.fullmatch(r"-?(0x[0-9a-f]+|\d+)", x):
            return int(x, 0) & M64
        return self.r[self._name(x)]

    def get64(self, x):
        x = x.strip()
        if x.startswith("%"):
            nm = self.operands[int(x[1:])]
            return self.r[nm]
        return self.get(x)

    def set(self, x, v):
        x = x.strip()
        m = re.fullmatch(r"v\[(\d+):(\d+)\]", x)
        if m:
            lo = int(m.group(1))
            self.r["v%d" % lo] = v & M32
            self.r["v%d" % (lo + 1)] = (v >> 32) & M32
            return
        self.r[self._name(x)] = v & M64 if x.startswith("%") and self._name(x).startswith("s64") else v & M32

    def run(self, lines):
        for ln in lines:
            op, _, rest = ln.partition(" ")
            a = [t.strip() for t in rest.split(",")] if rest else []
            if op == "s_nop":
                continue
            if op == "v_mad_u64_u32":
                acc = self.get(a[4])
                self.set(a[0], ((self.get(a[2]) & M32) * (self.get(a[3]) & M32) + acc) & M64)
            elif op == "v_mad_i64_i32":
                def s32(v):
                    v &= M32
                    return v - (1 << 32) if v >> 31 else v
                acc = self.get(a[4]) & M64
                acc = acc - (1 << 64) if acc >> 63 else acc
                self.set(a[0], (s32(self.get(a[2])) * s32(self.get(a[3])) + acc) & M64)
            elif op == "v_ashrrev_i64":
                v = self.get(a[2]) & M64
                v = v - (1 << 64) if v >> 63 else v
                self.set(a[0], (v >> int(a[1], 0)) & M64)
            elif op == "v_mad_u32_u24":
                self.set(a[0], ((self.get(a[1]) & 0xFFFFFF) * (self.get(a[2]) & 0xFFFFFF) + self.get(a[3])) & M32)
            elif op == "v_and_b32_e32":
                self.set(a[0], self.get(a[1]) & self.get(a[2]))
            elif op == "v_lshrrev_b64":
                self.set(a[0], self.get(a[2]) >> int(a[1], 0))
            elif op == "v_lshrrev_b32_e32":
                self.set(a[0], (self.get(a[2]) & M32) >> int(a[1], 0))
            elif op == "v_lshlrev_b32_e32":
                self.set(a[0], (self.get(a[2]) << int(a[1], 0)) & M32)
            elif op == "v_lshl_add_u64":
                sh = int(a[2], 0)
                if sh > 4:  # the hardware takes shift amounts 0..4 only
                    raise ValueError("v_lshl_add_u64 shift %d unsupported: %s" % (sh, ln))
                self.set(a[0], ((self.get(a[1]) << sh) + self.get(a[3])) & M64)
            elif op == "v_lshlrev_b64":
                self.set(a[0], (self.get(a[2]) << int(a[1], 0)) & M64)
            elif op == "v_alignbit_b32":
                v = ((self.get(a[1]) & M32) << 32) | (self.get(a[2]) & M32)
                self.set(a[0], (v >> int(a[3], 0)) & M32)
            elif op in ("v_add_u32_e32", "v_add_u32_e64"):
                self.set(a[0], (self.get(a[1]) + self.get(a[2])) & M32)
            elif op == "v_mov_b32_e32":
                self.set(a[0], self.get(a[1]) & M32)
            else:
                raise NotImplementedError(ln)


def run_block(header_text, func, values):
    """values: C++ expression -> integer for every input operand; returns expression -> value for
    every output operand (32-bit VGPR outputs)."""
    lines, outs, ins = parse_block(header_text, func)
    operands = {}
    lane = Lane(operands)
    for i, (_, expr) in enumerate(outs):
        operands[i] = "o:" + expr
    for j, (_, expr) in enumerate(ins):
        operands[len(outs) + j] = "i:" + expr
        lane.r["i:" + expr] = values[expr]
    lane.run(lines)
    return {expr: lane.r.get("o:" + expr) for _, expr in outs}
