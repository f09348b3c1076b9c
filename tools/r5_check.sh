#!/bin/bash
# round-5 check on the GPU box: the driver's bench form, then the focused GPU tests (each step under
# its own time limit, chained with &&)
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5/bench_k20.out 2> gpurun_out/r5/bench_k20.err && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_sharding_gpu.py \
    tests/test_rollout_gpu.py "tests/test_race_gpu.py::test_teacher_forced_step" \
    "tests/test_race_gpu.py::test_full_size_subset_vs_oracle" -s > gpurun_out/r5/tests.log 2>&1
