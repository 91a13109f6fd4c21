"""The bench's device-set legs (bench.devset_legs: C4 through bcosgpu_block_verify_multi, C5 through
bcosgpu_blocks_verify_multi, host buffers in and out) on a given device list, for A/B runs of the
pipeline's environment hooks (BCOSGPU_PIPE_HEAD, BCOSGPU_PIPE_CHUNK, BCOSGPU_PIPE_STREAMS: read once per
process, so one variant per process).  GPU tool; prints one JSON object.

usage: devset_probe.py [DEVICES, default 0,0] [MIN_SECONDS, default 2]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "fisco-bcos_amd"), ROOT]

import bench  # noqa: E402
import bcos_gpu  # noqa: E402


def main():
    devs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,0").split(",")]
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
    bcos_gpu.ensure_device(0)
    out = bench.devset_legs(devs, min_seconds=secs)
    out["env"] = {k: v for k, v in os.environ.items() if k.startswith("BCOSGPU_PIPE")}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
