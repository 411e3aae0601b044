"""Instruction mix of one kernel in a hipcc --save-temps .s file."""
import re
import sys
from collections import Counter

path, pat = sys.argv[1], sys.argv[2]
txt = open(path).read().split("\n")
start = end = None
for i, l in enumerate(txt):
    if start is None and re.match(r"^_Z\S*" + pat + r"\S*:", l):
        start = i
    elif start is not None and (l.startswith(".Lfunc_end") or l.startswith("\t.size")):
        end = i
        break
body = txt[start:end]
ins = [l.strip() for l in body if l.startswith("\t") and not l.strip().startswith((".", ";"))]
print(txt[start].split(":")[0][:100], "instructions", len(ins))
c = Counter(l.split()[0] for l in ins)
for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40):
    print(f"{k:28s}{v}")
print("scratch:", [l for l in ins if "scratch" in l][:6])
