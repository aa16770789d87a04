#!/bin/bash
# Round-end measurement set (run on the GPU box): GPU tests, headline bench,
# rocprofv3 kernel stats + PMC passes of the bench, cfg3/cfg5 with cpu
# baselines and per-kernel PMC.  Usage: scripts/final_round.sh TAG
set -u
tag=$1
scripts/gpu_step.sh ${tag}_gputest 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread || exit $?
grep -q " passed" gpurun_out/${tag}_gputest.log && ! grep -q "failed" gpurun_out/${tag}_gputest.log || exit 5
scripts/gpu_step.sh ${tag}_bench 300 python bench.py || exit $?
scripts/gpu_step.sh ${tag}_bench1000 300 python bench.py --steps 1000 --warmup 200 --no-cpu-baseline --pmc off || exit $?
scripts/profile.sh $tag || exit $?
scripts/gpu_step.sh ${tag}_configs 600 python scripts/bench_configs.py --configs 3,5,2u,2m --pmc || exit $?
FFTCONV_LA_TRACE=16 FFTCONV_LA_TRACE_OUT=gpurun_out/${tag}_tl_cfg2 scripts/gpu_step.sh ${tag}_tl 200 python bench.py --steps 300 --warmup 100 --no-cpu-baseline --pmc off || exit $?
python scripts/la_timeline.py gpurun_out/${tag}_tl_cfg2.* > gpurun_out/${tag}_timeline_cfg2.txt 2>&1
