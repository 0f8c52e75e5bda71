# round 5, call b (and c, the same script at O=r05c with the RSS stages and HW-queue variants): the server path as PHP-FPM runs it -- bench.py --workload c1cold: fresh
# worker processes (bare context x3, one worker at a time x3, then 4 and 16 concurrent workers, 16 also with
# DWPA_CALLS_PER_DEVICE=1 DWPA_HOST_THREADS=2).  The parent never touches the GPU; at most 16 children use it.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05c}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 900 python3 bench.py --workload c1cold --steps 20 > $O/c1cold.json 2> $O/c1cold.err
guard $?
python3 -c "
import json; d=json.load(open('$O/c1cold.json'))
print('value', d['value'], d['hits_verified'])
print(json.dumps(d['rows'], indent=1))
for c in d['concurrent']: print(json.dumps(c))"
