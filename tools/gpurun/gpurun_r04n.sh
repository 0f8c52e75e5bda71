# round 4, call n: why the head slows down beside the tail pieces (r04m: head 42.2 -> 48.3 ms with 8 pieces at
# priority 3).  Per variant one kernel-traced C5 run: the head's and the pieces' mean durations.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04n}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for v in "0 3" "8 0" "8 1" "8 2" "8 3"; do
  set -- $v
  DWPA_TAIL_PIECES=$1 DWPA_TAIL_PIECE_PRIO=$2 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$1_$2 -o run -- python3 bench.py --workload c5 --steps 8 --warmup 2 --no-cpu-baseline > $O/c5_p$1_$2.json 2> $O/c5_p$1_$2.err
  guard $?
  python3 - $O/p$1_$2/run_kernel_stats.csv $O/c5_p$1_$2.json "$1 $2" <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = json.load(open(sys.argv[2]))
out = {r["Name"][:34]: round(float(r["AverageNs"]) / 1e6, 3) for r in rows if "pbkdf2" in r["Name"] or "verify_att" in r["Name"]}
print("pieces/prio", sys.argv[3], "C5", d["value"], d["ms_per_step"], out)
PY
done
