# round 4, call za: C3's group kernel (k_pbkdf2_gfx950_mg_q) runs 2.6 % slower per PMK than C2's k_pbkdf2_gfx950_q
# with the same loop: VALU instructions, waves and busy cycles of both, one counter pass each.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04za}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/c3 -o run -- python3 bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > $O/c3.json 2> $O/c3.err
guard $?
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/c2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/c2.json 2> $O/c2.err
guard $?
python3 - $O <<'PY'
import csv, glob, sys, collections
for w in ("c2", "c3"):
    f = glob.glob(f"{sys.argv[1]}/{w}/*counter_collection.csv")[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:28]
        if "pbkdf2" not in k and "verify" not in k: continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in agg.items():
        print(w, k, {c: f"{v:.4g}" for c, v in d.items()})
PY
