# round 3, call o: C5 from 1, 2, 3 and 4 separate processes on one GPU (PHP-FPM workers, each its own library
# instance), timed over one common window (--start-at): node rate = all PMKs / (last end - first start).
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03o
mkdir -p $O
for np in 1 2 3 4; do
  at=$(python3 -c "import time; print(time.time() + 45)")
  pids=()
  for p in $(seq 1 $np); do
    timeout -k 10 300 python3 bench.py --workload c5 --steps $((30 * np)) --warmup 3 --no-cpu-baseline --start-at $at \
        > $O/c5_p${np}_$p.json 2> $O/c5_p${np}_$p.err &
    pids+=($!)
  done
  for pid in "${pids[@]}"; do wait $pid || { echo "process failed"; exit 1; }; done
  python3 - $O $np <<'PY'
import json, sys
o, n = sys.argv[1], int(sys.argv[2])
ds = [json.load(open(f"{o}/c5_p{n}_{p}.json")) for p in range(1, n + 1)]
lo = min(d["window_unix"][0] for d in ds); hi = max(d["window_unix"][1] for d in ds)
keys = sum(d["config"]["keys_per_step"] * d["steps"] for d in ds)
print(f"processes={n} node PMK/s {keys / (hi - lo):.0f} over {hi - lo:.2f} s; per process", [d["value"] for d in ds],
      "ms/call", [d["ms_per_step"] for d in ds], "starts", [round(d["window_unix"][0] - lo, 3) for d in ds],
      "ends", [round(hi - d["window_unix"][1], 3) for d in ds], "mismatches", [d["mismatches"] for d in ds])
PY
done
