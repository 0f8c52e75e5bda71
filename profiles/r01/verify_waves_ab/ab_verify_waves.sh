set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/vab
mkdir -p $O
B=$PWD/dwpa_amd/lib/libdwpa22000_b.so
A=$PWD/dwpa_amd/lib/libdwpa22000.so
for r in 1 2; do
  for v in A B; do
    L=$A; [ $v = B ] && L=$B
    DWPA_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/c2_${v}$r -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 6 --warmup 1 > $O/c2_${v}$r.json 2> $O/c2_${v}$r.err
  done
done
for v in A B; do
  L=$A; [ $v = B ] && L=$B
  DWPA_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/c3_${v} -o run --output-format csv -- python3 bench.py --workload c3 --steps 2 --warmup 1 > $O/c3_${v}.json 2> $O/c3_${v}.err
done
