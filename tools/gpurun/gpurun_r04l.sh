# round 4, call l: placement of small launches beside a one-round head (tools/tail_placement.hip): would cutting
# C5's PBKDF2 tail into sequential pieces spread its work over more SIMDs?
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04l}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for cfg in "8 44 256" "8 176 64" "8 44 256" "16 44 256"; do
  set -- $cfg
  timeout -k 10 60 tools/bin/tail_placement $1 $2 $3 > $O/placement_$1_$2_$3.json
  guard $?
  cat $O/placement_$1_$2_$3.json
done
