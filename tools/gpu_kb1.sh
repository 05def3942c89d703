set -o pipefail
cd $GRAFT_REPO_ROOT/tools/kbench/_build
export KB_COEF=1
S="2 16 512 512 16 5 2 2 1"
timeout -k 5 60 ./kbench fwd $S 50 && ISG_NO_S2K5=1 timeout -k 5 60 ./kbench fwd $S 50
timeout -k 5 60 ./kbench dgrad $S 50 && ISG_SUB2_DIRECT=1 timeout -k 5 60 ./kbench dgrad $S 50
timeout -k 5 60 ./kbench wgrad $S 50
H="2 16 256 256 16 1 1 0 1"
timeout -k 5 60 ./kbench headf $H 50 && timeout -k 5 60 ./kbench headb $H 50
cd $GRAFT_REPO_ROOT
OP=fwd SHAPE="$S" FILTER=s2k5 timeout -k 5 200 bash tools/kbench/pmc.sh s2k5
OP=headf SHAPE="$H" FILTER=head_fwd timeout -k 5 200 bash tools/kbench/pmc.sh headf
OP=headb SHAPE="$H" FILTER=head_bwd timeout -k 5 200 bash tools/kbench/pmc.sh headb
