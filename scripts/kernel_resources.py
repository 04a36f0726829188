#!/usr/bin/env python3
"""Register / LDS / spill usage of the gfx950 kernels inside a built object or library
(development tool): extracts the offload bundle, reads the code object's AMDGPU metadata.
usage: kernel_resources.py <.o|.so> [name-substring ...]"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")


def main():
    src = sys.argv[1]
    pats = sys.argv[2:]
    with tempfile.TemporaryDirectory() as d:
        fb = Path(d) / "fatbin"
        subprocess.run([LLVM / "llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", src, Path(d) / "junk"], check=True)
        co = Path(d) / "co"
        subprocess.run([LLVM / "clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([LLVM / "llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    cur = {}
    rows = []
    for line in notes.splitlines():
        line = line.strip()
        m = re.match(r"-?\s*\.(\w+):\s+(.*)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "name" and cur.get("name") is None:
            cur["name"] = v
        elif k in ("vgpr_count", "sgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_spill_count",
                   "group_segment_fixed_size", "private_segment_fixed_size"):
            cur[k] = v
        if k == "wavefront_size":
            pass
        if len(cur) >= 8:
            rows.append(cur)
            cur = {}
    for r in rows:
        n = r.get("name", "?")
        if pats and not any(p in n for p in pats):
            continue
        print(f"vgpr {r.get('vgpr_count'):>4} agpr {r.get('agpr_count'):>3} sgpr {r.get('sgpr_count'):>4} "
              f"spill v/s {r.get('vgpr_spill_count')}/{r.get('sgpr_spill_count')} lds {r.get('group_segment_fixed_size'):>6} "
              f"scratch {r.get('private_segment_fixed_size'):>4}  {n}")


if __name__ == "__main__":
    main()
