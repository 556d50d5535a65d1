"""Does RCCL accept two ranks on one GPU?  (perf tooling)
Starts two child processes, ranks 0 and 1 of WORLD_SIZE=2 on cuda:0 with the
"nccl" (RCCL) backend, and all-gathers a small tensor; prints one JSON line
with each rank's outcome.  bench.py's two-ranks-on-one-GPU test uses gloo when
RCCL refuses."""
import json
import os
import socket
import subprocess
import sys


def child():
    import torch
    import torch.distributed as dist
    r = int(os.environ["RANK"])
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=r, world_size=2)
        x = torch.full((4,), float(r), device="cuda")
        out = [torch.empty_like(x) for _ in range(2)]
        dist.all_gather(out, x)
        torch.cuda.synchronize()
        ok = [float(o[0]) for o in out] == [0.0, 1.0]
        dist.destroy_process_group()
        print(json.dumps({"rank": r, "ok": ok}))
    except Exception as e:  # noqa: BLE001 -- the outcome is the measurement
        print(json.dumps({"rank": r, "ok": False, "error": "%s: %s" % (type(e).__name__, str(e)[:300])}))


def main():
    if os.environ.get("PROBE_CHILD"):
        return child()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    procs = [subprocess.Popen([sys.executable, __file__],
                              env=dict(os.environ, PROBE_CHILD="1", RANK=str(r), WORLD_SIZE="2",
                                       MASTER_ADDR="127.0.0.1", MASTER_PORT=port),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    res = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=120)
        except subprocess.TimeoutExpired:
            p.kill()
            o, e = p.communicate()
            res.append({"rc": None, "timeout": True, "stderr": e[-300:]})
            continue
        line = [ln for ln in o.splitlines() if ln.startswith("{")]
        res.append({"rc": p.returncode, **(json.loads(line[-1]) if line else {}), "stderr_tail": e[-300:]})
    print(json.dumps({"rccl_two_ranks_one_gpu": all(r.get("ok") for r in res), "ranks": res}))


if __name__ == "__main__":
    main()
