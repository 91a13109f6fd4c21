"""Timeline of the last repetition in a rocprofv3 --kernel-trace --memory-copy-trace CSV output directory:
kernels and copies (start / end / duration in us from the repetition's first event, stream / queue),
repetitions split at idle gaps of more than 10 ms.  usage: trace_timeline.py DIR"""
import csv
import glob
import os
import sys


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main():
    d = sys.argv[1]
    ev = []
    for r in rows(d, "*kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:60], r.get("Stream_Id", "")))
    for r in rows(d, "*memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", r.get("Direction", "")[:18], r.get("Stream_Id", "")))
    ev.sort()
    last = 0
    for i in range(1, len(ev)):
        if ev[i][0] - max(e[1] for e in ev[:i]) > 10_000_000:
            last = i
    rep = ev[last:]
    t0 = rep[0][0]
    for s, e, k, name, st in rep:
        print("%9.1f %9.1f %8.1f  %s %-60s stream %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, k, name, st))
    print("span %.1f us" % ((max(e for _, e, *_ in rep) - t0) / 1e3))


if __name__ == "__main__":
    main()
