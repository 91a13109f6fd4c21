#!/usr/bin/env python3
"""Per-leg rocprofv3 summary of tools/leg_run.py passes (the bench's Merkle and hash legs).

usage: leg_prof.py OUT.json --trace DIR RUN.json [--pmc DIR RUN.json ...]

DIR is a rocprofv3 output directory, RUN.json the leg_run.py line of that pass (leg order, reps).  A leg's
dispatches are the library kernels between its two separator fills (torch FillFunctor kernels); every
counter is summed over them and divided by the pass's reps, i.e. stated PER ROOT / PER BATCH.  From the
trace pass: the kernels' summed duration per root and each kernel's dispatch count.  FETCH_SIZE /
WRITE_SIZE stay in rocprofv3's KiB (bench.leg_pmc doubles FETCH_SIZE: MI355X_MICROARCH.md's gfx950
correction)."""
import collections
import csv
import glob
import json
import os
import sys


def _short(name):
    return name.split("(")[0].replace("void ", "").replace("bcosgpu::", "").strip()


def _is_sep(name):
    return "FillFunctor" in name


def _legs(rows, order):
    """rows: [(dispatch_id, kernel, payload)] -> {leg: [(kernel, payload), ...]} by separator pairs (the last
    2 x len(order) fills: an earlier fill -- a torch.zeros -- is not a separator)."""
    rows.sort(key=lambda r: r[0])
    fills = [i for i, r in enumerate(rows) if _is_sep(r[1])]
    if len(fills) > 2 * len(order):
        rows = rows[fills[len(fills) - 2 * len(order)]:]
    out, cur, nsep = {}, None, 0
    for _, k, pay in rows:
        if _is_sep(k):
            if nsep % 2 == 0:
                cur = order[nsep // 2] if nsep // 2 < len(order) else None
                if cur is not None:
                    out[cur] = []
            else:
                cur = None
            nsep += 1
        elif cur is not None and "at::" not in k:
            out[cur].append((k, pay))
    return out


def counters(d, order, reps):
    per = collections.defaultdict(lambda: [None, collections.defaultdict(float)])
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                e = per[int(row["Dispatch_Id"])]
                e[0] = _short(row["Kernel_Name"])
                e[1][row["Counter_Name"]] += float(row["Counter_Value"])
    legs = _legs([(i, k, c) for i, (k, c) in per.items()], order)
    res = {}
    for leg, ds in legs.items():
        tot = collections.defaultdict(float)
        for _, c in ds:
            for name, v in c.items():
                tot[name] += v
        res[leg] = {name: v / reps for name, v in tot.items()}
    return res


def trace(d, order, reps):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                rows.append((int(row["Dispatch_Id"]), _short(row["Kernel_Name"]),
                             int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
    legs = _legs(rows, order)
    res = {}
    for leg, ds in legs.items():
        ks = collections.Counter(k for k, _ in ds)
        res[leg] = {"kernel_ns_per_unit": sum(ns for _, ns in ds) / reps,
                    "kernels": {k: v / reps for k, v in ks.items()}}
    return res


def _run(path):
    with open(path) as f:
        lines = [ln for ln in f.read().splitlines() if ln.startswith("{")]
    return json.loads(lines[-1])


def main():
    out, args = sys.argv[1], sys.argv[2:]
    legs = collections.defaultdict(dict)
    ms = {}
    srcs = []
    while args:
        kind, d, runf = args[0], args[1], args[2]
        args = args[3:]
        run = _run(runf)
        srcs.append({"kind": kind, "dir": d, "reps": run["reps"]})
        if kind == "--trace":
            ms = run["ms"]
            for leg, v in trace(d, run["order"], run["reps"]).items():
                legs[leg].update(v)
        else:
            for leg, v in counters(d, run["order"], run["reps"]).items():
                legs[leg].update(v)
    for leg, v in legs.items():
        if leg in ms:
            v["event_ms_per_unit"] = ms[leg]
        if v.get("SQ_INSTS_VALU") and v.get("GRBM_GUI_ACTIVE"):
            v["valu_issue"] = v["SQ_INSTS_VALU"] * 4.0 / 1024.0 / (v["GRBM_GUI_ACTIVE"] / 8.0)
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
    import bench
    with open(out, "w") as f:
        json.dump({"source": "rocprofv3 passes of tools/leg_run.py (kernel trace; separate --pmc passes), per root / batch",
                   "passes": srcs, "kernel_source_sha": bench.kernel_source_sha(), "legs": legs}, f,
                  indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
