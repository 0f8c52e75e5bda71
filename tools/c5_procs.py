"""C5 from K separate processes over a common timed window (PHP-FPM workers making bulk check calls side by side):
every process runs `bench.py --workload c5 --start-at T`, and the node rate is the PMKs of all processes over the
union of their timed windows.  Prints one JSON line per K.

    python tools/c5_procs.py [--procs 1,2,4] [--steps 20] [--env KEY=VALUE ...]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", default="1,2,4")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--env", action="append", default=[])
    args = ap.parse_args()
    env = dict(os.environ, **dict(e.split("=", 1) for e in args.env))
    for k in [int(x) for x in args.procs.split(",")]:
        start = time.time() + 40.0  # every process has built its batch and warmed up before the window opens
        ps = [subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "c5", "--steps",
                                str(args.steps), "--warmup", "3", "--no-cpu-baseline", "--start-at", repr(start)],
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env) for _ in range(k)]
        outs = []
        for p in ps:
            o, e = p.communicate(timeout=600)
            if p.returncode != 0:
                raise SystemExit(f"c5 process failed (rc {p.returncode}): {e[-2000:]}")
            outs.append(json.loads(o.strip().splitlines()[-1]))
        t0 = min(o["window_unix"][0] for o in outs)
        t1 = max(o["window_unix"][1] for o in outs)
        pmks = sum(o["config"]["keys_per_step"] * o["steps"] for o in outs)
        print(json.dumps({"processes": k, "node_pmk_per_s": round(pmks / (t1 - t0), 1),
                          "per_process_ms_per_call": [o["ms_per_step"] for o in outs],
                          "mismatches": sum(o.get("mismatches", 0) for o in outs),
                          "tail_waves_last_call": [o.get("last_call", {}).get("tail_waves") for o in outs],
                          "env": args.env}), flush=True)


if __name__ == "__main__":
    main()
