#!/usr/bin/env python3
"""Register / scratch / LDS use of the kernels in a hipcc object or .so
(reads the gfx950 code object's AMDGPU metadata with llvm-readelf).

    python tools/kres.py FILE [name-regex]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_object(path, tmp):
    fb = os.path.join(tmp, "fb.bin")
    subprocess.run([LLVM + "/llvm-objcopy", "--dump-section=.hip_fatbin=" + fb, path], check=True,
                   capture_output=True)
    out = os.path.join(tmp, "co.elf")
    subprocess.run([LLVM + "/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + fb,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + out], check=True)
    return out


def main():
    path, pat = sys.argv[1], re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    with tempfile.TemporaryDirectory() as tmp:
        notes = subprocess.run([LLVM + "/llvm-readelf", "--notes", code_object(path, tmp)], check=True,
                               capture_output=True, text=True).stdout
    kern, cur = [], None
    for line in notes.splitlines():
        m = re.match(r"\s+- \.agpr_count:\s+(\d+)", line)
        if m:
            cur = {"agpr": int(m.group(1))}
            kern.append(cur)
            continue
        m = re.match(r"\s+\.(name|vgpr_count|sgpr_count|private_segment_fixed_size|group_segment_fixed_size|"
                     r"vgpr_spill_count|sgpr_spill_count):\s+(\S+)", line)
        if m and cur is not None:
            cur[m.group(1)] = m.group(2)
    for k in kern:
        if pat.search(k.get("name", "")):
            print("vgpr %4s agpr %3d sgpr %3s spill v%s s%s scratch %5s lds %6s  %s" % (
                k.get("vgpr_count"), k["agpr"], k.get("sgpr_count"), k.get("vgpr_spill_count"),
                k.get("sgpr_spill_count"), k.get("private_segment_fixed_size"), k.get("group_segment_fixed_size"),
                k.get("name")))


if __name__ == "__main__":
    main()
