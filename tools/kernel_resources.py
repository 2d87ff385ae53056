"""VGPR / SGPR / spill / LDS counts of every gfx950 kernel in the built library (tools only):
the offload bundles in the .so's fat binary are split out and their AMDGPU metadata notes
read with llvm-readelf.  Usage: python tools/kernel_resources.py [lib.so] [name-filter]"""
import os
import re
import struct
import subprocess
import sys
import tempfile

lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
    "monst3r-slam_amd", "monst3r_slam_amd", "libmonst3r_slam_amd.so")
flt = sys.argv[2] if len(sys.argv) > 2 else ""
data = open(lib, "rb").read()
magic = b"__CLANG_OFFLOAD_BUNDLE__"
rows = []
pos = data.find(magic)
while pos >= 0:
    n = struct.unpack_from("<Q", data, pos + 24)[0]
    p = pos + 32
    for _ in range(n):
        off, size, tl = struct.unpack_from("<QQQ", data, p)
        triple = data[p + 24:p + 24 + tl].decode()
        p += 24 + tl
        if "gfx950" in triple and size:
            with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
                f.write(data[pos + off:pos + off + size])
            out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", f.name],
                                 capture_output=True, text=True).stdout
            os.unlink(f.name)
            for blk in out.split("\n  - .agpr_count")[1:]:
                def g(k):
                    m = re.search(r"\." + k + r":\s+(\S+)", blk)
                    return m.group(1) if m else "?"
                agpr = blk.split()[1] if blk.split() else "?"
                rows.append((g("name"), g("vgpr_count"), agpr, g("sgpr_count"),
                             g("vgpr_spill_count"), g("sgpr_spill_count"),
                             g("group_segment_fixed_size")))
    pos = data.find(magic, pos + 1)
for r in sorted(set(rows)):
    if flt in r[0]:
        print(f"vgpr {r[1]:>4} agpr {r[2]:>3} sgpr {r[3]:>3} vspill {r[4]:>3} sspill {r[5]:>3} "
              f"lds {r[6]:>6}  {r[0]}")
