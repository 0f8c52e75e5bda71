set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ab2
for v in 0 3 0 3; do
  export DWPA_LIB=$PWD/dwpa_amd/lib/ab/lib_v$v.so
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab2/c5_v$v -o run -- python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab2/c5_v$v.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab2/c2_v$v -o run -- python bench.py --dict-words 12000000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab2/c2_v$v.log 2>&1
done
