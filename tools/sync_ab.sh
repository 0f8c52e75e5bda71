#!/bin/bash
# End-of-call wait A/B (engine.cpp wait_done): DWPA_SYNC=sync (hipStreamSynchronize) vs poll (event query every
# ~20 us, the default), on C5 with one and two callers and on the small-call latency leg; interleaved twice.
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/sync_ab}
mkdir -p $OUT
guard() { case $1 in 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; esac; }
for rep in 1 2; do
  for m in sync poll; do
    for k in 1 2; do
      DWPA_SYNC=$m timeout -k 10 150 python3 bench.py --workload c5 --callers $k --steps 20 --warmup 3 --no-cpu-baseline \
          > $OUT/c5_${m}_k${k}_$rep.json 2> $OUT/c5_${m}_k${k}_$rep.err
      guard $?
      echo "$m callers=$k rep=$rep $(python3 -c "import json;d=json.load(open('$OUT/c5_${m}_k${k}_$rep.json'));print(d['value'], d['ms_per_step'], d['mismatches'])")"
    done
    DWPA_SYNC=$m timeout -k 10 150 python3 bench.py --workload c1lat --steps 9 > $OUT/c1lat_${m}_$rep.json 2> $OUT/c1lat_${m}_$rep.err
    guard $?
    echo "$m c1lat rep=$rep $(python3 -c "import json;d=json.load(open('$OUT/c1lat_${m}_$rep.json'));print([r['gpu_ms_per_call'] for r in d['rows']])")"
  done
done
echo done
