"""Register / scratch / LDS use of the gfx950 kernels in a built library.

  python tools/kernel_resources.py [lib.so] [name-substring]

Extracts the gfx950 code object from the library's clang offload bundle and
prints, per kernel, the AMDGPU metadata that decides occupancy and spilling:
VGPRs, AGPRs, SGPRs, spill counts, scratch (private segment) bytes, static LDS.
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib):
    data = open(lib, "rb").read()
    pos = 0
    while True:
        pos = data.find(MAGIC, pos)
        if pos < 0:
            return
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        off = pos + 32
        for _ in range(n):
            o, size, tlen = struct.unpack_from("<QQQ", data, off)
            triple = data[off + 24:off + 24 + tlen].decode()
            off += 24 + tlen
            if "gfx" in triple:
                yield triple, data[pos + o:pos + o + size]
        pos += len(MAGIC)


def kernels(co):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        txt = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True).stdout
    out, cur = [], None
    for line in txt.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s+(.*)$", line)
        if not m:
            continue
        key, val = m.group(1), m.group(2).strip()
        if key == "agpr_count" or (key == "args" and cur is None):
            cur = {}
            out.append(cur)
        if cur is not None:
            cur[key] = val
    return [k for k in out if "name" in k]


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "openkite_amd/lib/libkite_nmpc.so")
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    for triple, co in code_objects(lib):
        print(triple)
        print(f"{'kernel':60s} {'vgpr':>5s} {'agpr':>5s} {'sgpr':>5s} {'vspill':>6s} {'sspill':>6s} "
              f"{'scratch':>7s} {'lds':>6s}")
        for k in kernels(co):
            name = k["name"]
            if pat and pat not in name:
                continue
            print(f"{name[:60]:60s} {k.get('vgpr_count', '?'):>5s} {k.get('agpr_count', '?'):>5s} "
                  f"{k.get('sgpr_count', '?'):>5s} {k.get('vgpr_spill_count', '?'):>6s} "
                  f"{k.get('sgpr_spill_count', '?'):>6s} {k.get('private_segment_fixed_size', '?'):>7s} "
                  f"{k.get('group_segment_fixed_size', '?'):>6s}")


if __name__ == "__main__":
    main()
