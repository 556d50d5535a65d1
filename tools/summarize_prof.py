"""Summarize a tools/gpu_profile.sh run (gpurun_out/prof) into profiles/<tag>_*.

Traffic per launch follows MI355X_MICROARCH.md "HBM": FETCH_SIZE/WRITE_SIZE are
in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so
the corrected figure doubles it (the guide calls other access widths
uncalibrated: both raw and corrected values are recorded)."""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
scen = sys.argv[2] if len(sys.argv) > 2 else "robocup"
src = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/prof_%s" % scen
out = "profiles"
K = "step_kernel"
# the fused step program's kernels: step_kernel, and the RoboCup step with its
# key-window helper wave (step_help_kernel); the config-5 backward may be the
# split tape backward (bwd_split_kernel)
STEP_KERNELS = ("step_kernel", "step_help_kernel")


def is_step(name):
    return any(k in name for k in STEP_KERNELS)


def last_dispatches(rows, n):
    """The step-kernel rows of the LAST n dispatches (the bench's timed launches:
    with --extras off nothing runs the kernel after them), so that warm-up
    launches of another regime (LunarLander falls before it settles) do not mix
    into the per-launch figures."""
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})[-n:]
    keep = set(ids)
    return [r for r in rows if int(r["Dispatch_Id"]) in keep]


def stall_fracs(s):
    """The stall pass's buckets as fractions of its own wave cycles."""
    if not s:
        return None
    w = s["SQ_WAVE_CYCLES"]
    return {"active_any": s["SQ_ACTIVE_INST_ANY"] / w, "active_valu": s["SQ_ACTIVE_INST_VALU"] / w,
            "active_lds": s["SQ_ACTIVE_INST_LDS"] / w, "wait_any": s["SQ_WAIT_ANY"] / w,
            "wait_inst_any": s["SQ_WAIT_INST_ANY"] / w, "wait_inst_lds": s["SQ_WAIT_INST_LDS"] / w,
            "lds_bank_conflict_cycles_per_lds_active": s["SQ_LDS_BANK_CONFLICT"] / max(s["SQ_ACTIVE_INST_LDS"], 1.0)}


def have(d):
    return os.path.exists(os.path.join(src, d, "run_counter_collection.csv"))


def pmc(d, n=None):
    rows = [r for r in csv.DictReader(open(os.path.join(src, d, "run_counter_collection.csv"))) if is_step(r["Kernel_Name"])]
    if n:
        rows = last_dispatches(rows, n)
    agg = defaultdict(list)
    for r in rows:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


if scen.startswith("grad"):
    # config 5: the forward (MODE 1) and backward (MODE 4 / 2) step kernels, per kernel
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    bench = json.load(open(os.path.join(src, "trace_bench.json")))

    def pmc_k(d, name):
        agg = defaultdict(list)
        for r in csv.DictReader(open(os.path.join(src, d, "run_counter_collection.csv"))):
            if r["Kernel_Name"] == name:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        return {k: sum(v) / len(v) for k, v in agg.items()}

    kernels = {}
    import re

    def mode_of(name):  # step_kernel<EW, FNSET, MODE[, SPEC]>
        m = re.search(r"step_kernel<\d+, \d+, (\d+)", name)
        return int(m.group(1)) if m else -1

    # the backward: the split tape backward, else MODE 4 (from the forward's
    # tape), else the re-play (MODE 2)
    split = [r for r in stats if "bwd_split_kernel" in r["Name"]]
    bmode = 4 if any(K in r["Name"] and mode_of(r["Name"]) == 4 for r in stats) else 2
    for part, mode in (("fwd", 1), ("bwd", bmode)):
        row = split[0] if part == "bwd" and split else [r for r in stats if K in r["Name"] and mode_of(r["Name"]) == mode][0]
        c = {}
        for d in ("pmc_fetch", "pmc_write", "pmc_sq"):
            c.update(pmc_k(d, row["Name"]))
        kernels[part] = {"kernel": row["Name"], "calls": int(row["Calls"]), "avg_launch_ns": float(row["AverageNs"]),
                         "counters_per_launch": c,
                         "hbm_bytes_per_launch_raw": (c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024,
                         "hbm_bytes_per_launch_corrected": (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024,
                         "valu_active_frac_of_wave_cycles": c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"],
                         "wait_frac_of_wave_cycles": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
                         "stall": stall_fracs(pmc_k("pmc_stall", row["Name"]) if have("pmc_stall") else None)}
    summary = {"tag": tag, "scenario": scen, "config": bench["config"], "library": bench["config"]["library"],
               "bench_value": bench["value"], "warmup": bench["warmup"], "steps": bench["steps"], "kernels": kernels}
    os.makedirs(out, exist_ok=True)
    json.dump(summary, open(os.path.join(out, "%s_%s_summary.json" % (tag, scen)), "w"), indent=1)
    json.dump(summary, open(os.path.join(out, "latest_pmc_%s.json" % scen), "w"), indent=1)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(out, "%s_%s_kernel_stats.csv" % (tag, scen)))
    print(json.dumps({p: {k: v for k, v in kk.items() if k != "counters_per_launch"} for p, kk in kernels.items()},
                     indent=1))
    sys.exit(0)

stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
row = [r for r in stats if is_step(r["Name"])][0]
bench = json.load(open(os.path.join(src, "trace_bench.json")))
nt = int(bench["steps"])  # the timed launches
trows = last_dispatches([r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv")))
                         if is_step(r["Kernel_Name"])], nt)
avg_ns = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trows) / len(trows)
c = {}
for d in ("pmc_fetch", "pmc_write", "pmc_sq"):
    c.update(pmc(d, nt))
raw = (c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
corr = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
summary = {
    "tag": tag,
    "scenario": scen,
    "kernel": row["Name"],
    "calls": int(row["Calls"]),
    "timed_launches": nt,
    "avg_launch_ns": avg_ns,  # over the timed launches (trace), like the counters
    "bench_event_launch_ms": bench["roofline"]["launch_ms"],
    "bench_value": bench["value"],
    "config": bench["config"],
    "warmup": bench["warmup"],
    "steps": bench["steps"],
    "hbm_bytes_per_launch_raw": raw,
    "hbm_bytes_per_launch_corrected": corr,
    "alg_bytes_per_launch": bench["roofline"].get("hbm", bench["roofline"]).get("alg_bytes_per_launch"),
    "counters_per_launch": c,
    "valu_active_frac_of_wave_cycles": c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"],
    "wait_frac_of_wave_cycles": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
    "stall": stall_fracs(pmc("pmc_stall", nt) if have("pmc_stall") else None),
}
os.makedirs(out, exist_ok=True)
json.dump(summary, open(os.path.join(out, "%s_%s_summary.json" % (tag, scen)), "w"), indent=1)
json.dump(summary, open(os.path.join(out, "latest_pmc_%s.json" % scen), "w"), indent=1)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(out, "%s_%s_kernel_stats.csv" % (tag, scen)))
for d in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_stall"):
    if have(d):
        shutil.copy(os.path.join(src, d, "run_counter_collection.csv"), os.path.join(out, "%s_%s_%s.csv" % (tag, scen, d)))
print(json.dumps({k: summary[k] for k in ("avg_launch_ns", "bench_event_launch_ms", "hbm_bytes_per_launch_raw",
                                          "hbm_bytes_per_launch_corrected", "valu_active_frac_of_wave_cycles",
                                          "wait_frac_of_wave_cycles", "stall")}, indent=1))
