#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel-trace --stats and --pmc passes) into one JSON per workload.

usage: prof_summary.py OUT.json TRACE_DIR [PMC_DIR ...]

  kernels[name] = {calls, avg_ns (kernel_stats), <COUNTER>: mean per dispatch, vgpr, sgpr, scratch, lds}
FETCH_SIZE / WRITE_SIZE are rocprofv3's KB per dispatch; per MI355X_MICROARCH.md ("On gfx950
FETCH_SIZE reports exactly 1/2 of the bytes of a wide coalesced streaming read") consumers double
FETCH_SIZE (bench.py does: traffic = (2 FETCH_SIZE + WRITE_SIZE) KiB).
"""
import collections
import csv
import glob
import json
import os
import sys


def _short(name):
    return name.split("(")[0].strip()


def kernel_stats(d):
    out = {}
    for path in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                out[_short(row["Name"])] = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                                            "min_ns": float(row["MinNs"]), "max_ns": float(row["MaxNs"]),
                                            "percent": float(row["Percentage"])}
    return out


def counters(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, dispatch) -> counter -> sum
    meta = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = _short(row["Kernel_Name"])
                per[(k, row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
                meta[k] = {"vgpr": int(row.get("VGPR_Count") or 0), "agpr": int(row.get("Accum_VGPR_Count") or 0),
                           "sgpr": int(row.get("SGPR_Count") or 0), "scratch": int(row.get("Scratch_Size") or 0),
                           "lds": int(row.get("LDS_Block_Size") or 0), "grid": int(row.get("Grid_Size") or 0),
                           "workgroup": int(row.get("Workgroup_Size") or 0)}
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, _), cs in per.items():
        for c, v in cs.items():
            acc[k][c].append(v)
    return {k: dict({c: sum(v) / len(v) for c, v in cs.items()}, **meta.get(k, {}), dispatches=max(len(v) for v in cs.values()))
            for k, cs in acc.items()}


def main():
    out, trace, pmcs = sys.argv[1], sys.argv[2], sys.argv[3:]
    ks = kernel_stats(trace)
    for d in pmcs:
        for k, cs in counters(d).items():
            ks.setdefault(k, {}).update(cs)
    for k, c in ks.items():
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            c["hbm_bytes_per_dispatch"] = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
    for k, c in ks.items():
        if c.get("GRBM_GUI_ACTIVE") and c.get("avg_ns"):
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back)
            cyc = c["GRBM_GUI_ACTIVE"] / 8.0
            c["eff_clock_ghz"] = cyc / c["avg_ns"]
            if c.get("SQ_INSTS_VALU"):
                # On gfx950 SQ_ACTIVE_INST_VALU reads equal to SQ_INSTS_VALU (an instruction count, not
                # quad-cycles), so VALU pressure is stated as kernel cycles per wave-instruction per SIMD:
                # 4.0 = one wave64 VALU instruction every 4 cycles on every one of the 1,024 SIMDs.
                c["valu_cycles_per_instr_per_simd"] = cyc * 1024.0 / c["SQ_INSTS_VALU"]
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
    import bench
    with open(out, "w") as f:
        json.dump({"source": "rocprofv3 --kernel-trace --stats + separate --pmc passes", "trace_dir": trace,
                   "pmc_dirs": pmcs, "kernel_source_sha": bench.kernel_source_sha(), "kernels": ks}, f,
                  indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
