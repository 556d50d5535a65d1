"""Per-kernel register / scratch usage of the step kernel objects (perf
tooling): compiles cotix_step_kernel.hip for one envs-per-wave tiling with
-Rpass-analysis=kernel-resource-usage and prints one line per kernel.
  python tools/res_usage.py [EW] [filter]"""
import re
import subprocess
import sys

ew = sys.argv[1] if len(sys.argv) > 1 else "4"
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math", "-std=c++17",
       "--cuda-device-only", "-c", "-DCOTIX_EW=%s" % ew, "parallax_amd/csrc/cotix_step_kernel.hip", "-o", "/tmp/ru.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, {}
for ln in out.split("\n"):
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        n = re.search(r"step_kernelILi(\d+)ELi(\d+)ELi(\d+)E(?:Li(\d+)E)?", m.group(1))
        cur = "ew%s fn%s mode%s spec%s" % (n.group(1), n.group(2), n.group(3), n.group(4) or "0") if n else m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/lane\])?: (\d+)", ln)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    if flt in k:
        print("%-28s vgpr %3s sgpr %3s sgpr_spill %3s vgpr_spill %3s scratch %4s" % (
            k, v.get("VGPRs"), v.get("TotalSGPRs"), v.get("SGPRs Spill"), v.get("VGPRs Spill"), v.get("ScratchSize")))
