#!/bin/bash
# convf1 on the flow's x channel alone (round 6): the conv2d_small / model parity tests, then a bench
# line (conv2d_small's live per-launch time against the previous profile run's 39.1 us)
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/f1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_model.py -k "conv2d_small or forward or epe or reference" > gpurun_out/f1/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/f1/bench.log 2>&1 || exit 1
