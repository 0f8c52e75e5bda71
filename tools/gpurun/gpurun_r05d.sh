# round 5, call d: (1) C5 with GPU_MAX_HW_QUEUES=1 against the default (the PHP-FPM sizing rule's cost for big
# batch calls); (2) VERDICT r4 item 5, spent once: is the C5 head's per-wave deficit against C2 (7.03 vs 6.50 ms per
# wave-time) occupancy (6 head waves per SIMD against C2's 8) or the kernels queued beside it?  C2's own kernel at a
# 196,608-PMK batch (exactly 6 waves per SIMD, nothing beside it) against the default 16M batch, then one PMC pass
# over C5 and one over the 6-wave C2 batch (SQ_WAVES, SQ_INSTS_VALU, SQ_BUSY_CYCLES, SQ_WAVE_CYCLES).
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05d}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for q in 4 1; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 180 python3 bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline \
      > $O/c5_hwq$q.json 2> $O/c5_hwq$q.err
  guard $?
  python3 -c "import json;d=json.load(open('$O/c5_hwq$q.json'));print('c5 hwq $q', d['value'], d['ms_per_step'], d['mismatches'])"
done
timeout -k 10 300 python3 bench.py --batch 196608 --steps 40 --warmup 2 --no-cpu-baseline --dict-words 10000000 \
    > $O/c2_b6w.json 2> $O/c2_b6w.err
guard $?
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --dict-words 60000000 \
    > $O/c2_b16m.json 2> $O/c2_b16m.err
guard $?
for f in c2_b6w c2_b16m; do
  python3 -c "import json;d=json.load(open('$O/$f.json'));r=d['roofline'];print('$f', d['value'], d['ms_per_step'], r.get('kernel'), r.get('kernel_ms'), r['frac'])"
done
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv \
    -d $O/pmc_c5 -o run -- python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_c5.json 2> $O/pmc_c5.err
guard $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv \
    -d $O/pmc_c2b6w -o run -- python3 bench.py --batch 196608 --steps 4 --warmup 1 --no-cpu-baseline \
    --dict-words 2000000 > $O/pmc_c2b6w.json 2> $O/pmc_c2b6w.err
guard $?
ls -R $O | head -30
