"""Static instruction mix of kernels in gfx950 device assembly (hipcc
--cuda-device-only -S), one column per (file, kernel) -- the before/after
counts DESIGN quotes for the QP kernels.
  python tools/asm_mix.py LABEL=file.s:kernel_substring [LABEL=file.s:kernel_substring ...]"""
import re
import sys
from collections import Counter

CATS = [
    ("total", lambda op: True),
    ("v_mfma (fp64 16x16x4)", lambda op: op.startswith("v_mfma")),
    ("fp64 VALU (v_*_f64)", lambda op: op.startswith("v_") and op.endswith("_f64") and not op.startswith("v_mfma")),
    ("v_cndmask", lambda op: op.startswith("v_cndmask")),
    ("exec-mask ops (s_*saveexec, s_*_exec)", lambda op: "saveexec" in op or op.endswith("_exec") or "exec_" in op),
    ("s_cbranch", lambda op: op.startswith("s_cbranch")),
    ("AGPR moves (v_accvgpr_*)", lambda op: op.startswith("v_accvgpr")),
    ("LDS (ds_*)", lambda op: op.startswith("ds_")),
    ("global/buffer memory", lambda op: op.startswith(("global_", "buffer_", "flat_"))),
    ("lane ops (readlane/permlane/bpermute)", lambda op: "readlane" in op or "permlane" in op or "bpermute" in op),
    ("s_waitcnt", lambda op: op.startswith("s_waitcnt")),
    ("scratch", lambda op: op.startswith("scratch_")),
]


def kernel_ops(path, sub):
    s = open(path).read()
    m = [x for x in re.finditer(r"^(_Z\S*?):", s, re.M) if sub in x.group(1)]
    if not m:
        raise SystemExit(f"{sub} not in {path}")
    start = m[0].end()
    end = s.index(".Lfunc_end", start)
    ops, dpp = Counter(), 0
    for line in s[start:end].splitlines():
        t = line.strip().split()
        if t and not t[0].startswith((".", ";")) and not t[0].endswith(":"):
            ops[t[0]] += 1
            if "row_" in line or "quad_perm" in line or "row_newbcast" in line:
                dpp += 1
    meta = re.search(r"\.vgpr_count:\s+(\d+)", s[end:end + 200000])
    return ops, dpp


cols = []
for arg in sys.argv[1:]:
    label, rest = arg.split("=", 1)
    path, sub = rest.rsplit(":", 1)
    cols.append((label, *kernel_ops(path, sub)))
w = max(len(c[0]) for c in cols) + 2
print(f"{'':40s}" + "".join(f"{c[0]:>{w}s}" for c in cols))
for name, pred in CATS:
    print(f"{name:40s}" + "".join(f"{sum(v for k, v in c[1].items() if pred(k)):>{w}d}" for c in cols))
print(f"{'DPP-modified VALU':40s}" + "".join(f"{c[2]:>{w}d}" for c in cols))
