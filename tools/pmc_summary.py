"""Summarise a tools/gpu_round.sh run into profiles/ files.

  python tools/pmc_summary.py gpurun_out/<tag> <tag>

writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats) and
profiles/<tag>_pmc_hbm.json: per kernel, the mean FETCH_SIZE / WRITE_SIZE per
launch (separate --pmc passes), in bytes, raw and corrected as
/opt/skills/guides/MI355X_MICROARCH.md prescribes for gfx950 (FETCH_SIZE reads
half the bytes of coalesced streaming reads: doubled; WRITE_SIZE exact).
"""
import collections
import csv
import json
import os
import shutil
import sys

src, tag = sys.argv[1], sys.argv[2]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(REPO, "profiles")
os.makedirs(prof, exist_ok=True)
shutil.copy(os.path.join(src, "prof", "ktrace_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
out = {}
for sub, name, ctr in [("pmc_fetch", "fetch", "FETCH_SIZE"), ("pmc_write", "write", "WRITE_SIZE")]:
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(src, sub, f"{name}_counter_collection.csv"))):
        vals[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)   # rocprofv3 reports kB
    for k, v in vals.items():
        if k.startswith("k_"):
            d = out.setdefault(k, {})
            d[f"{ctr}_bytes_raw"] = sum(v) / len(v)
            d["launches"] = len(v)
for k, d in out.items():
    d["read_bytes"] = 2.0 * d.get("FETCH_SIZE_bytes_raw", 0.0)
    d["write_bytes"] = d.get("WRITE_SIZE_bytes_raw", 0.0)
    d["traffic_bytes"] = d["read_bytes"] + d["write_bytes"]
json.dump({"tag": tag,
           "command": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate passes) -- python bench.py --steps 2 --warmup 1",
           "correction": "read = 2 x FETCH_SIZE (gfx950 coalesced-read rule), write = WRITE_SIZE; per launch",
           "kernels": out}, open(os.path.join(prof, f"{tag}_pmc_hbm.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
