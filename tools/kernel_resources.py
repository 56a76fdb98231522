#!/usr/bin/env python3
"""Register, LDS and scratch use of the gfx950 kernels in a built library (from the code objects'
AMDGPU metadata notes): `python tools/kernel_resources.py [lib] [name-filter]`."""
import re
import struct
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects(lib: Path, tmp: Path):
    fatbin = tmp / "fatbin.bin"
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fatbin}", str(lib),
                    str(tmp / "stripped.so")], check=True)
    data = fatbin.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    at, k = data.find(magic), 0
    while at >= 0:
        count = struct.unpack_from("<Q", data, at + 24)[0]
        p = at + 32
        for _ in range(count):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple:
                co = tmp / f"co{k}.o"
                co.write_bytes(data[at + off:at + off + size])
                k += 1
                yield co
        at = data.find(magic, at + 1)


def resources(lib: Path):
    rows = []
    with tempfile.TemporaryDirectory() as t:
        for co in code_objects(lib, Path(t)):
            meta = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)], check=True,
                                  capture_output=True, text=True).stdout
            for blk in re.split(r"\n\s*- \.agpr_count", meta)[1:]:
                def get(key):
                    m = re.search(rf"\.{key}:\s+(\S+)", blk)
                    return m.group(1) if m else "?"
                rows.append((get("name"), get("vgpr_count"), get("sgpr_count"),
                             get("private_segment_fixed_size"), get("group_segment_fixed_size"),
                             get("vgpr_spill_count"), get("sgpr_spill_count")))
    return rows


if __name__ == "__main__":
    lib = Path(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1] else ROOT / "metropolis-hastings-gpgpu_amd" / "libmhgpu.so"
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    print(f"{'kernel':70s} vgpr sgpr scratch lds vspill sspill")
    for r in sorted(resources(lib)):
        if flt in r[0]:
            print(f"{r[0][:70]:70s} {r[1]:>4s} {r[2]:>4s} {r[3]:>7s} {r[4]:>4s} {r[5]:>6s} {r[6]:>6s}")
