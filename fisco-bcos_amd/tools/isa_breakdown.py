#!/usr/bin/env python3
"""Static instruction breakdown of a kernel's loops in the built gfx950 code (tools/hazard_check.py's
disassembler): every backward branch closes a loop; per loop, the instructions of its body by category --
field-product multiply-adds (v_mad_u64_u32, v_mul_*), routing (DPP moves and DPP-folded selects,
permlanes, ds_bpermute / swizzle), selects (v_cndmask without DPP), other VALU (adds, shifts, bitops:
carries, reductions, subtractions, small multiples), LDS, global / scratch memory, SALU, s_nop and
waitcnt.  Used for the C2 lane-trio kernel's window loop: which of its instructions are
products and which only move operands between the lanes of a trio.

usage: isa_breakdown.py LIB_OR_OBJECT KERNEL_SUBSTRING [--top N]   (one JSON object)"""
import collections
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import hazard_check  # noqa: E402


def category(mn, ops):
    if mn.startswith("s_nop"):
        return "s_nop"
    if mn.startswith("s_waitcnt"):
        return "waitcnt"
    if mn.startswith("v_mad_u64_u32") or mn.startswith("v_mad_i64_i32") or mn.startswith("v_mul_"):
        return "product_mad_mul"
    if "_dpp" in mn or "row_" in ops or "quad_perm" in ops or "permlane" in mn:
        return "routing_dpp_permlane"
    if mn.startswith("ds_bpermute") or mn.startswith("ds_swizzle"):
        return "routing_lds_permute"
    if mn.startswith("v_cndmask"):
        return "select"
    if mn.startswith("ds_"):
        return "lds"
    if mn.startswith("global_") or mn.startswith("buffer_") or mn.startswith("scratch_") or mn.startswith("flat_"):
        return "vmem"
    if mn.startswith("v_"):
        return "valu_other"
    if mn.startswith("s_"):
        return "salu_branch"
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 6
    funcs = [f for f in hazard_check.functions(path) if sub in f[0]]
    if not funcs:
        print(json.dumps({"error": "no function matching %r" % sub}))
        return 1
    out = {}
    for name, base, insts in funcs:
        addr_idx = {a: i for i, (a, _, _) in enumerate(insts)}
        loops = []
        for i, (a, mn, ops) in enumerate(insts):
            if mn.startswith("s_cbranch") or mn == "s_branch":
                m = re.search(r"<.+\+0x([0-9a-f]+)>", ops)
                if not m:
                    continue
                tgt = base + int(m.group(1), 16)
                j = addr_idx.get(tgt)
                if j is not None and j <= i:
                    loops.append((j, i))
        total = collections.Counter(category(mn, ops) for _, mn, ops in insts)
        rec = {"instructions": len(insts), "by_category": dict(total.most_common()), "loops": []}
        for j, i in sorted(loops, key=lambda x: -(x[1] - x[0]))[:top]:
            body = insts[j:i + 1]
            c = collections.Counter(category(mn, ops) for _, mn, ops in body)
            valu = sum(v for k, v in c.items() if k in ("product_mad_mul", "routing_dpp_permlane", "select",
                                                        "valu_other"))
            rec["loops"].append({"start": "0x%x" % insts[j][0], "end": "0x%x" % insts[i][0], "instructions": len(body),
                                 "valu": valu, "by_category": dict(c.most_common()),
                                 "valu_share": {k: round(c[k] / valu, 3) for k in
                                                ("product_mad_mul", "routing_dpp_permlane", "select", "valu_other")}
                                 if valu else {}})
        out[name] = rec
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
