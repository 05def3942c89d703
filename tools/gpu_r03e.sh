set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
H="2 16 256 256 16 1 1 0 1"; S="2 16 512 512 16 5 2 2 1"
export KB_COEF=1 CONFIG=2,20,1024
OP=headb SHAPE="$H" LABEL=d_out0 timeout -k 5 200 bash tools/kbench/traffic.sh headb | tail -c 300
OP=headf SHAPE="$H" LABEL=out0 timeout -k 5 200 bash tools/kbench/traffic.sh headf | tail -c 300
OP=dgrad SHAPE="$S" LABEL=dx_init_conv.layer2 timeout -k 5 200 bash tools/kbench/traffic.sh sub2 | tail -c 300
OP=fwd SHAPE="$S" LABEL=init_conv.layer2 timeout -k 5 200 bash tools/kbench/traffic.sh s2k5 | tail -c 300
OP=wgrad SHAPE="$S" LABEL=dw_init_conv.layer2 timeout -k 5 200 bash tools/kbench/traffic.sh twg | tail -c 300
unset KB_COEF CONFIG
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --profile-ops gpurun_out/ops_r3e.txt > gpurun_out/bench_r3e.log 2>&1; tail -1 gpurun_out/bench_r3e.log | cut -c1-1500
