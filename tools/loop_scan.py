"""Per inner loop of one kernel in a gfx950 .s file: instruction count, global
loads, vmcnt waits, scratch, MFMA, LDS, readlane/writelane.
  python tools/loop_scan.py file.s kernel_regex"""
import re
import sys

s = open(sys.argv[1]).read()
name = re.findall(r"\n(" + sys.argv[2] + r"\w*):", s)[0]
st = s.index("\n" + name + ":") + 1
en = s.index(".Lfunc_end", st)
L = [l for l in s[st:en].splitlines() if l.strip() and not l.strip().startswith((".loc", ".cfi", ";"))]
print(name, len(L), "instructions")
loops = {}
for i, l in enumerate(L):
    m = re.search(r"in Loop: Header=(\S+) Depth=(\d)", l)
    if m and m.group(2) == "2":
        loops.setdefault(m.group(1), [i, i])[1] = i
for h, (a, b) in loops.items():
    seg = L[a:b + 1]
    c = lambda k: sum(k in x for x in seg)
    print(f"{h:12s} lines {a:6d}-{b:6d} n {b - a:5d} global_load {c('global_load'):3d} vmcnt(0) {c('vmcnt(0)'):3d} "
          f"vmcnt {c('vmcnt'):3d} scratch {c('scratch_'):3d} mfma {c('mfma'):3d} ds {c('ds_'):3d} "
          f"readlane {c('readlane'):3d} writelane {c('writelane'):3d} accvgpr {c('accvgpr'):3d}")
