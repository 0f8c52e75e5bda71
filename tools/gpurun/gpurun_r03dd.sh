# round 3, call dd: C2 launch size A/B with the work-queue kernel -- 16.8M (default), 33.6M and 67.1M candidates per
# step (one launch each; the 100M dictionary is then 6 / 3 / 2 batches), interleaved.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03dd
mkdir -p $O
for rep in 1 2; do
  for b in 16777216 33554432 67108864; do
    st=$((100663296 / b)); [ $st -lt 1 ] && st=1
    timeout -k 10 300 python3 bench.py --batch $b --steps $st --warmup 1 --no-cpu-baseline > $O/c2_b${b}_$rep.json 2> $O/c2_b${b}_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$O/c2_b${b}_$rep.json'));r=d['roofline'];print('batch $b rep $rep', d['value'], d['ms_per_step'], r['kernel_pmk_per_s'], r['frac'], d['hits_verified'])"
  done
done
