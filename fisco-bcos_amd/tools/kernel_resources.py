#!/usr/bin/env python3
"""Print per-kernel register / spill / scratch usage of the gfx950 code objects inside a hipcc
object or shared library (parses the clang offload bundle, then llvm-readelf --notes).

usage: kernel_resources.py fisco-bcos_amd/build/ecc_kernels.o [name-filter]
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def bundles(blob):
    pos = 0
    while True:
        pos = blob.find(MAGIC, pos)
        if pos < 0:
            return
        n = struct.unpack_from("<Q", blob, pos + len(MAGIC))[0]
        q = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, q)
            triple = blob[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if "gfx950" in triple:
                yield triple, blob[pos + off:pos + off + size]
        pos += len(MAGIC)


def main():
    path, filt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    blob = open(path, "rb").read()
    for triple, co in bundles(blob):
        with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
            f.write(co)
        notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", f.name], capture_output=True,
                               text=True).stdout
        os.unlink(f.name)
        recs, cur = [], None
        for line in notes.splitlines():
            if re.match(r"^  - \.", line):  # a kernel's record (its fields at 4 spaces, in any order)
                cur = {}
                recs.append(cur)
                line = "    " + line[4:]
            m = re.match(r"^    \.(name|vgpr_count|agpr_count|vgpr_spill_count|sgpr_spill_count|"
                         r"private_segment_fixed_size|sgpr_count|group_segment_fixed_size):\s+(\S+)", line)
            if m and cur is not None:
                cur[m.group(1)] = m.group(2)
        for r in recs:
            if r.get("name") and not r["name"].endswith(".kd") and filt in r["name"]:
                print(dict(sorted(r.items(), key=lambda kv: kv[0] != "name")))


if __name__ == "__main__":
    main()
