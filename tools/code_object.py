#!/usr/bin/env python3
"""Register budget of every gfx950 kernel in a built library, from its code
objects (not from the profiler's granule-encoded VGPR_Count field).

The library's .hip_fatbin section holds one clang offload bundle per HIP
translation unit; each gfx950 entry is an ELF code object whose AMDGPU
metadata note lists per kernel .vgpr_count, .agpr_count, .sgpr_count, the
spill counts and the private (scratch) segment size.

    python tools/code_object.py [compton2d_amd/libcompton2d.so] [--kernel NAME]
"""
from __future__ import annotations

import argparse
import os
import re
import struct
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path(os.environ.get("ROCM_PATH", "/opt/rocm")) / "lib" / "llvm" / "bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
FIELDS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
          ".private_segment_fixed_size", ".group_segment_fixed_size")


def gfx950_objects(lib: Path):
    """The gfx950 code objects (bytes) of every offload bundle in `lib`."""
    with tempfile.TemporaryDirectory() as td:
        fb = Path(td) / "fatbin"
        subprocess.run([str(LLVM / "llvm-objcopy"), "--dump-section", ".hip_fatbin=%s" % fb, str(lib),
                        str(Path(td) / "lib.copy")], check=True, capture_output=True)
        data = fb.read_bytes()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + len(MAGIC))[0]
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple and size:
                out.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, pos + 1)
    return out


def kernel_registers(lib: Path) -> dict:
    """{kernel symbol: {field: int}} over all gfx950 code objects of `lib`."""
    res = {}
    for co in gfx950_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            txt = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", f.name], check=True,
                                 capture_output=True, text=True).stdout
        # the metadata is YAML-like: one "- .args:" block per kernel
        for blk in re.split(r"\n\s+- \.args:|\n\s+- \.agpr_count:", txt)[1:]:
            m = re.search(r"\.name:\s+(\S+)", blk)
            if not m:
                continue
            d = {}
            for k in FIELDS:
                v = re.search(re.escape(k) + r":\s+(\d+)", blk)
                if v:
                    d[k[1:]] = int(v.group(1))
            res[m.group(1)] = d
    return res


def disassemble(lib: Path, pattern: str) -> str:
    """llvm-objdump of the gfx950 code object holding a kernel whose name contains `pattern`."""
    for co in gfx950_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            syms = subprocess.run([str(LLVM / "llvm-readelf"), "-s", f.name], check=True,
                                  capture_output=True, text=True).stdout
            if pattern in syms:
                return subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", f.name],
                                      check=True, capture_output=True, text=True).stdout
    return ""


def describe(lib: Path, pattern: str = "") -> str:
    lines = []
    for name, d in sorted(kernel_registers(lib).items()):
        if pattern and pattern not in name:
            continue
        lines.append("%-48s VGPR %3s AGPR %3s SGPR %3s spills v/s %s/%s scratch %s B LDS %s B" % (
            name[:48], d.get("vgpr_count"), d.get("agpr_count"), d.get("sgpr_count"),
            d.get("vgpr_spill_count"), d.get("sgpr_spill_count"), d.get("private_segment_fixed_size"),
            d.get("group_segment_fixed_size")))
    return "\n".join(lines)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=str(Path(__file__).resolve().parents[1] /
                                                  "compton2d_amd" / "libcompton2d.so"))
    ap.add_argument("--kernel", default="")
    ap.add_argument("--disasm", action="store_true", help="print the ISA of the code object with --kernel")
    a = ap.parse_args(argv)
    if a.disasm:
        print(disassemble(Path(a.lib), a.kernel))
        return 0
    print(describe(Path(a.lib), a.kernel))
    return 0


if __name__ == "__main__":
    sys.exit(main())
