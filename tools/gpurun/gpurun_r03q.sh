# round 3, call q: PBKDF2 loop list-scheduled again by the issue pass (sched=D: producers >= D VALU slots back where
# the dependences allow), raced in tools/bin/asm_lab against the product rule on 4M PMKs, outputs compared word for
# word with the first variant.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03q
mkdir -p $O
A=tools/bin/asm
V="$A/before_half.hsaco $A/sched_2_before_half.hsaco $A/sched_3_before_half.hsaco $A/sched_2:alt_before_half.hsaco $A/sched_4:alt_before_half.hsaco $A/sched_6_before_half.hsaco $A/sched_1_before_half.hsaco"
timeout -k 10 300 tools/bin/asm_lab 4194304 4 $V > $O/race1.json 2> $O/race1.err || exit 1
cat $O/race1.json
R=$(echo $V | tr ' ' '\n' | tac | tr '\n' ' ')
timeout -k 10 300 tools/bin/asm_lab 4194304 4 $A/before_half.hsaco $R > $O/race2.json 2> $O/race2.err || exit 1
cat $O/race2.json
