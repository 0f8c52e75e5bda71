# round 5, call aq: VGPR source banks and VALU issue cost on gfx950 (tools/vgpr_bank.hip), lone wave and 8 waves.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05aq}
mkdir -p $O
timeout -k 10 60 ./tools/bin/vgpr_bank 4000 > $O/bank.json 2> $O/bank.err || { echo "rc $?"; exit 1; }
cat $O/bank.json
