"""Single-call latency tail A/B (tools/callbench.cpp over the coalesced C ABI): the same T-thread single-call
run per suite under environment variants of the coalescer and kernel choice, each in its own process, with
callbench's tail record (p90 / p95 / p99 / p99.9 and the calls slower than 4 x p50 by the tenth of the run
they started in).  GPU tool; one JSON line per (suite, variant).

usage: tail_ab.py OUT_DIR THREADS VARIANT [VARIANT ...]   (VARIANT: "default" or NAME=VALUE[,NAME=VALUE])"""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from callbench_sweep import EXE, write_data  # noqa: E402


def main():
    out_dir, threads, variants = sys.argv[1], int(sys.argv[2]), sys.argv[3:] or ["default"]
    for suite in (1, 0):
        path = os.path.join(out_dir, "callbench_%d.bin" % suite)
        write_data(path, suite)
        for rep in range(2):
            for v in variants:
                env = dict(os.environ)
                if v != "default":
                    env.update(kv.split("=", 1) for kv in v.split(","))
                r = subprocess.run([EXE, path, str(threads), "1000"], capture_output=True, text=True, timeout=120,
                                   env=env)
                res = json.loads(r.stdout.strip().splitlines()[-1]) if r.stdout.strip() else {}
                res.update(variant=v, rep=rep, rc=r.returncode)
                print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
