"""Instruction mix of one kernel in a --save-temps / -S gfx950 assembly file.
  python tools/asm_count.py file.s kernel_substring [top]"""
import sys
from collections import Counter

src, name = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 50
s = open(src).read()
i = s.index(":", s.index("\n_", s.index(name) - 200) if False else s.index(name + ":") if (name + ":") in s else
            [k for k in range(len(s)) if s.startswith(name, k)][0])
begin = s.rfind("\n", 0, s.index(":", s.index(name))) + 1
start = s.index(":\n", s.index(name, s.index(".type\t" + name) if (".type\t" + name) in s else 0))
end = s.index(".Lfunc_end", start)
lines = s[start:end].splitlines()
c = Counter()
for l in lines:
    t = l.strip().split()
    if t and not t[0].startswith((".", ";")) and not t[0].endswith(":"):
        c[t[0]] += 1
print("instructions:", sum(c.values()))
for k, v in c.most_common(top):
    print(f"{k:32s} {v}")
