"""Static instruction counts per phase of the step kernel (perf tooling).
Build the ISA with phase markers, then split it:
  hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -std=c++17 --cuda-device-only -S \
      -DCOTIX_ASM_MARKERS -DCOTIX_EW=4 parallax_amd/csrc/cotix_step_kernel.hip -o /tmp/m.s
  python tools/isa_phases.py /tmp/m.s step_kernelILi4ELi1ELi0E"""
import re
import sys
from collections import Counter, defaultdict

NAMES = ["load", "save", "A", "T", "B", "C0", "C0b", "C1", "C2", "C3", "D", "E", "ret", "store", "restore", "G",
         "adj", "F", "K", "E1", "R", "trace", "B0", "B1", "F0", "F1", "F2", "F3",
         "TV0", "TV1", "TV2", "TV3"]
src, pat = sys.argv[1], sys.argv[2]
DUMP = sys.argv[3] if len(sys.argv) > 3 else None  # optional: print this phase's instructions
lines = open(src).read().split("\n")
body, cur = [], False
for ln in lines:
    m = re.match(r"^(_Z\S+):", ln)
    if m:
        cur = pat in m.group(1)
        continue
    if cur and ln.startswith(".Lfunc_end"):
        break
    if cur:
        body.append(ln)
sreg = {}
stack = []
cnt = defaultdict(Counter)
for ln in body:
    t = ln.strip()
    m = re.match(r"s_mov_b32\s+(s\d+),\s+(-?\d+)$", t)
    if m:
        sreg[m.group(1)] = int(m.group(2))
    m = re.match(r";#PHASE_BEGIN\s+(s\d+)", t)
    if m:
        stack.append(NAMES[sreg.get(m.group(1), 0)] if sreg.get(m.group(1), -1) >= 0 else "?")
        continue
    if t.startswith(";#PHASE_END"):
        if stack:
            stack.pop()
        continue
    if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
        continue
    op = t.split()[0]
    ph = stack[-1] if stack else "-"
    cnt[ph][op] += 1
    if DUMP is not None and ph == DUMP:
        print(t)
for ph, c in sorted(cnt.items(), key=lambda kv: -sum(kv[1].values())):
    tot = sum(c.values())
    v = sum(n for k, n in c.items() if k.startswith("v_"))
    s_ = sum(n for k, n in c.items() if k.startswith("s_"))
    ds = sum(n for k, n in c.items() if k.startswith("ds_"))
    top = ", ".join("%s %d" % kv for kv in c.most_common(6))
    print("%-6s total %5d  valu %5d  salu/branch %5d  lds %4d | %s" % (ph, tot, v, s_, ds, top))
