# round 3, call h: check-path TableBuilder kept per call context (A/B against ab/aes1g.so, the same code with a
# fresh builder per call), and the crack-path reader with reserved chunk capacity.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03h
mkdir -p $O
guard() { case $1 in 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -k "golden or c5 or random_batch or nc_windows or concurrent or chunked" \
    -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; guard $rc; echo "pytest rc=$rc $(tail -1 $O/pytest.txt)"; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for lib in ab/aes1g.so dwpa_amd/lib/libdwpa22000.so; do
    n=$(basename $lib .so)
    for k in 1 2; do
      DWPA_LIB=$PWD/$lib timeout -k 10 150 python3 bench.py --workload c5 --callers $k --steps 20 --warmup 3 \
          --no-cpu-baseline > $O/c5_${n}_k${k}_$rep.json 2> $O/c5_${n}_k${k}_$rep.err
      guard $?
      echo "$n callers=$k rep=$rep $(python3 -c "import json;d=json.load(open('$O/c5_${n}_k${k}_$rep.json'));print(d['value'], d['ms_per_step'], d['mismatches'])")"
    done
  done
done
THREADS=8 OUT=$O/reader_ab timeout -k 10 600 bash tools/reader_ab.sh > $O/reader_ab.log 2>&1 || exit $?
cat $O/reader_ab/c2_t8.json $O/reader_ab/list_t8.json
