# round 3, call aa: C2 with two batches in flight (--pipeline 2, own scan + stream each) against one, with the
# work-queue PBKDF2 kernel (round 1 measured +0.2 % with the grid kernel), interleaved.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03aa
mkdir -p $O
for rep in 1 2; do
  for p in 1 2; do
    timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --pipeline $p > $O/c2_p${p}_$rep.json 2> $O/c2_p${p}_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$O/c2_p${p}_$rep.json'));print('pipeline $p rep $rep', d['value'], d['ms_per_step'], d['hits_verified'])"
  done
done
