# round 3, call f: keyver-3 AES address computation A/B (aes1f: LLVM's bfe + lshl_or; aes1g = default: shift +
# v_bitop3), the full C5 prefix oracle at this HEAD, and one LDS/VALU counter pass of the new default.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03f
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; esac; }
DWPA_FULL_ORACLE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py \
    -k "golden or c5 or random_batch or nc_windows" -x -v -s --timeout 360 --timeout-method thread > $O/pytest_full_oracle.log 2>&1
rc=$?; guard $rc; echo "pytest rc=$rc $(tail -1 $O/pytest_full_oracle.log)"; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for lib in aes1f aes1g; do
    for k in 1 2; do
      DWPA_LIB=$PWD/ab/$lib.so timeout -k 10 150 python3 bench.py --workload c5 --callers $k --steps 20 --warmup 3 \
          --no-cpu-baseline > $O/c5_${lib}_k${k}_$rep.json 2> $O/c5_${lib}_k${k}_$rep.err
      guard $?
      echo "$lib callers=$k rep=$rep $(python3 -c "import json;d=json.load(open('$O/c5_${lib}_k${k}_$rep.json'));print(d['value'], d['ms_per_step'], d['mismatches'])")"
    done
  done
done
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $C -d $O/pmc_aes1g -o run --output-format csv -- python3 bench.py --workload c5 \
    --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_aes1g.log 2>&1 || exit $?
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_aes1g -o run -- python3 bench.py \
    --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_aes1g.json 2> $O/prof_aes1g.err || exit $?
echo done
