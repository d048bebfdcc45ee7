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
# steady-state launch durations from the same trace: the profiled bench runs
# WARMUP untimed steps first (cold-start QPs iterate longer), so the stats
# mean over all launches sits above bench.py's HIP-event mean of the timed
# steps; this drops the first WARMUP launches of each RTI kernel
WARMUP = int(os.environ.get("KITE_PROF_WARMUP", "2"))
durs = collections.defaultdict(list)
for r in csv.DictReader(open(os.path.join(src, "prof", "ktrace_kernel_trace.csv"))):
    durs[r["Kernel_Name"].split("(")[0]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
steady = {}
for k, v in durs.items():
    if k.startswith("k_") and len(v) > WARMUP:
        st = v[WARMUP:]
        steady[k] = {"launches": len(v), "mean_ns_all": sum(v) / len(v), "warmup_dropped": WARMUP,
                     "mean_ns_steady": sum(st) / len(st), "min_ns": min(st), "max_ns": max(st)}
json.dump({"tag": tag, "source": "rocprofv3 --kernel-trace (ktrace_kernel_trace.csv)", "kernels": steady},
          open(os.path.join(prof, f"{tag}_kernel_steady.json"), "w"), indent=1)
out = {}
for sub, name, ctr in [("pmc_fetch", "fetch", "FETCH_SIZE"), ("pmc_write", "write", "WRITE_SIZE")]:
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(src, sub, f"{name}_counter_collection.csv"))):
        vals[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)   # rocprofv3 reports kB
    for k, v in vals.items():
        if k.startswith("k_"):
            d = out.setdefault(k, {})
            st = v[WARMUP:] if len(v) > WARMUP else v     # steady-state launches, as for the durations
            d[f"{ctr}_bytes_raw"] = sum(st) / len(st)
            d["launches"] = len(st)
for k, d in out.items():
    d["read_bytes"] = 2.0 * d.get("FETCH_SIZE_bytes_raw", 0.0)
    d["write_bytes"] = d.get("WRITE_SIZE_bytes_raw", 0.0)
    d["traffic_bytes"] = d["read_bytes"] + d["write_bytes"]
bench_config = None
algo_flops = None
try:                       # the bench line of the same session: which configuration was profiled
    line = json.loads(open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1])
    bench_config = line["run_config"]
    algo_flops = line.get("algorithmic_flops_per_launch")
except Exception:
    pass
json.dump({"tag": tag,
           "bench_config": bench_config,
           "command": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate passes) -- python bench.py --steps 30 --warmup 3",
           "warmup_launches_dropped": WARMUP,
           "correction": "read = 2 x FETCH_SIZE (gfx950 coalesced-read rule), write = WRITE_SIZE; per launch",
           "kernels": out}, open(os.path.join(prof, f"{tag}_pmc_hbm.json"), "w"), indent=1)
# SQ pass: wave-cycle breakdown and fp64 MFMA activity per launch (steady state)
sq_csv = os.path.join(src, "pmc_sq", "sq_counter_collection.csv")
if os.path.exists(sq_csv):
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    for r in csv.DictReader(open(sq_csv)):
        k = r["Kernel_Name"]
        if k.startswith("k_"):
            per[k][int(r.get("Dispatch_Id") or r.get("Correlation_Id"))][r["Counter_Name"]] = float(r["Counter_Value"])
    sq = {}
    SIMDS = 256 * 4
    XCDS = 8
    for k, disp in per.items():
        ids = sorted(disp)
        st = ids[WARMUP:] if len(ids) > WARMUP else ids
        avg = {c: sum(disp[i].get(c, 0.0) for i in st) / len(st) for c in disp[st[0]]}
        d = dict(avg, launches=len(st))
        wc = avg.get("SQ_WAVE_CYCLES", 0.0)
        if wc > 0:
            d["frac_wait_any"] = avg.get("SQ_WAIT_ANY", 0.0) / wc
            d["frac_wait_inst_any"] = avg.get("SQ_WAIT_INST_ANY", 0.0) / wc
            d["frac_active_inst_any"] = avg.get("SQ_ACTIVE_INST_ANY", 0.0) / wc
            d["frac_active_valu"] = avg.get("SQ_ACTIVE_INST_VALU", 0.0) / wc
        if avg.get("GRBM_GUI_ACTIVE", 0.0) > 0:
            # MFMA-busy cycles over GPU-busy cycles x SIMDs.  GRBM_GUI_ACTIVE is
            # summed over the 8 XCDs (MI355X_MICROARCH.md, GRBM row): one XCD's
            # busy cycles are GRBM_GUI_ACTIVE / 8 (27.08 M / 8 over 1.44 ms =
            # 2.35 GHz in the r02z trace), so the SIMD-cycle denominator is
            # (GRBM_GUI_ACTIVE / 8) x 1024 SIMDs
            d["gpu_busy_cycles_per_xcd"] = avg["GRBM_GUI_ACTIVE"] / XCDS
            d["mfma_util"] = avg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (avg["GRBM_GUI_ACTIVE"] / XCDS * SIMDS)
        d["mfma_f64_flops"] = avg.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) * 512.0
        alg = (algo_flops or {}).get(k)
        if alg:
            # executed MFMA flops (padding included) over the kernel's algorithmic flops per launch
            d["algorithmic_flops"] = alg
            d["mfma_executed_over_algorithmic"] = d["mfma_f64_flops"] / alg
        sq[k] = d
    json.dump({"tag": tag, "bench_config": bench_config,
               "command": "rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY "
                          "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 "
                          "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -- python bench.py --steps 30 --warmup 3",
               "note": "per launch, steady-state launches; WAVE/WAIT/ACTIVE in quad-cycles summed over waves; "
                       "mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs); "
                       "mfma_f64_flops = SQ_INSTS_VALU_MFMA_MOPS_F64 x 512",
               "kernels": sq}, open(os.path.join(prof, f"{tag}_sq_mfma.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
