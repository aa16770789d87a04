#!/bin/bash
# deferred-tail0 tests, cfg3 bench and a kernel-trace profile (run on the GPU box)
set -u
scripts/gpu_step.sh defer_tests 400 python -u -m pytest tests/test_gpu_twostage_defer.py tests/test_gpu_crossfade_twostage.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "deferred or twostage or cfg3" -m gpu -q --timeout 120 --timeout-method thread || exit $?
grep -q "passed" gpurun_out/defer_tests.log && ! grep -q "failed" gpurun_out/defer_tests.log || exit 5
timeout -k 10 200 python scripts/bench_configs.py --configs 3 --no-cpu > gpurun_out/cfg3.log 2>&1 || exit 3
grep process_device_steps gpurun_out/cfg3.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg3 -o kt --output-format csv -- python3 scripts/bench_configs.py --configs 3 --no-cpu > gpurun_out/prof_cfg3.log 2>&1 || exit 4
find gpurun_out/prof_cfg3 -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-150 | head -9
