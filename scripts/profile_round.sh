#!/bin/bash
# Full measurement pass on the GPU box (outputs under gpurun_out/prof):
#   bench      the default bench line (value, roofline, cpu baseline)
#   trace      rocprofv3 --kernel-trace --stats over a short bench run (hipGraph replays)
#   trace1s    the same with every step eager on one stream, the whole batch per launch
#              (bench.py --one-stream: the instrumented steps' schedule, per-launch times comparable)
#   fetch/write  rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate runs (HBM bytes, --one-stream)
#   trace5     the one-stream kernel trace of a cfg5 step (the booster batch)
#   cfg3/4/5   the other configs' bench lines
#   dist2      a 2-rank torchrun rehearsal of the bench on one GPU (gloo, ranks share the card)
# Each step under its own limit; a fault or time-out ends the script (gpu_steps.sh).
# usage: scripts/profile_round.sh [a|b|all]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$(pwd)
mkdir -p gpurun_out/prof
SHORT="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-epe"
exec_steps=(
  "bench:420:python3 $R/bench.py > $R/gpurun_out/prof/bench.log 2>&1; tail -n 1 $R/gpurun_out/prof/bench.log > $R/gpurun_out/prof/bench.json"
  "trace:300:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof/trace -o run --output-format csv -- $SHORT"
  "trace1s:300:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof/trace1s -o run --output-format csv -- $SHORT --one-stream"
  "fetch:300:cd /tmp && rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof/fetch -o run --output-format csv -- $SHORT --one-stream"
  "write:300:cd /tmp && rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof/write -o run --output-format csv -- $SHORT --one-stream"
  "trace5:400:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof/trace5 -o run --output-format csv -- python3 $R/bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline --no-epe --one-stream"
  "cfg3:300:python3 $R/bench.py --config cfg3 > $R/gpurun_out/prof/cfg3.log 2>&1; tail -n 1 $R/gpurun_out/prof/cfg3.log > $R/gpurun_out/prof/bench_cfg3.json"
  "cfg4:300:python3 $R/bench.py --config cfg4 > $R/gpurun_out/prof/cfg4.log 2>&1; tail -n 1 $R/gpurun_out/prof/cfg4.log > $R/gpurun_out/prof/bench_cfg4.json"
  "cfg5:420:python3 $R/bench.py --config cfg5 > $R/gpurun_out/prof/cfg5.log 2>&1; tail -n 1 $R/gpurun_out/prof/cfg5.log > $R/gpurun_out/prof/bench_cfg5.json"
  "dist2:300:cd $R && SA_DIST_BACKEND=gloo SA_DIST_SHARE_GPU=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config cfg4 --steps 2 --warmup 1 --no-epe > $R/gpurun_out/prof/dist2.log 2>&1"
)
# part a / b (one gpurun call each: a call is limited to 20 minutes): the first five steps / the rest
case "${1:-all}" in
  a) bash "$R/scripts/gpu_steps.sh" "${exec_steps[@]:0:5}" ;;
  b) bash "$R/scripts/gpu_steps.sh" "${exec_steps[@]:5}" ;;
  *) bash "$R/scripts/gpu_steps.sh" "${exec_steps[@]}" ;;
esac
