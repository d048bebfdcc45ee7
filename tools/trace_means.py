"""Per-kernel steady mean durations from a rocprofv3 kernel-trace CSV (the
first 3 launches of each kernel dropped): python tools/trace_means.py TRACE.csv"""
import collections
import csv
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].split("(")[0].replace("kite::", "").split("<")[0]
    d[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for name, v in d.items():
    s = v[3:] if len(v) > 3 else v
    print(f"{name:34s} {len(v):4d} {sum(s) / len(s) / 1e3:10.2f} us")
