# round 3, call n: C5 from 1, 2 and 4 separate processes on one GPU at once (PHP-FPM workers each load their own
# libdwpa22000.so: no head fencing between processes), against two callers in one process.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03n
mkdir -p $O
for np in 1 2 4; do
  pids=()
  for p in $(seq 1 $np); do
    timeout -k 10 300 python3 bench.py --workload c5 --steps 40 --warmup 3 --no-cpu-baseline \
        > $O/c5_p${np}_$p.json 2> $O/c5_p${np}_$p.err &
    pids+=($!)
  done
  for pid in "${pids[@]}"; do wait $pid || { echo "process failed"; exit 1; }; done
  python3 - $O $np <<'PY'
import json, sys
o, n = sys.argv[1], int(sys.argv[2])
ds = [json.load(open(f"{o}/c5_p{n}_{p}.json")) for p in range(1, n + 1)]
print(f"processes={n}", "per-process PMK/s", [d["value"] for d in ds], "sum", round(sum(d["value"] for d in ds)),
      "ms/call", [d["ms_per_step"] for d in ds], "mismatches", [d["mismatches"] for d in ds])
PY
done
timeout -k 10 300 python3 bench.py --workload c5 --callers 2 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5_k2.json 2> $O/c5_k2.err || exit 1
python3 -c "import json;d=json.load(open('$O/c5_k2.json'));print('callers=2', d['value'], d['ms_per_step'], d['mismatches'])"
