"""Instruction mix of a kernel in a hipcc --save-temps .s file (perf tooling).
usage: python tools/isa_stats.py FILE.s NAME_SUBSTRING"""
import re
import sys
from collections import Counter

src, pat = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
cur, body = None, []
for ln in lines:
    m = re.match(r"^(_Z\S+):", ln)
    if m:
        cur = m.group(1) if pat in m.group(1) else None
        continue
    if cur and ln.startswith(".Lfunc_end"):
        break
    if cur and ln.startswith("\t") and not ln.startswith("\t.") and ln.strip() and not ln.strip().startswith(";"):
        body.append(ln.split()[0])
c = Counter(body)
print("instructions", len(body))
print("alignbit (rotations; 20 per threefry block)", c["v_alignbit_b32"], "-> blocks", c["v_alignbit_b32"] / 20)
for k, v in c.most_common(25):
    print("%-28s %d" % (k, v))
