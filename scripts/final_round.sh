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
# kernel stats of cfg2u / cfg5 (the update's IR transform and window rebuild) and cfg3
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
scripts/gpu_step.sh ${tag}_kt_cfg25 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_cfg25 -o kt --output-format csv -- python3 scripts/bench_configs.py --configs 2u,5 --no-cpu || exit $?
python3 scripts/kstats.py gpurun_out/prof_${tag}_cfg25 14 > gpurun_out/${tag}_kstats_cfg25.txt
scripts/gpu_step.sh ${tag}_kt_cfg3 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_cfg3 -o kt --output-format csv -- python3 scripts/ab_cfg3.py fft-convolution_amd/libfftconv_amd.so --rounds 3 || exit $?
python3 scripts/kstats.py gpurun_out/prof_${tag}_cfg3 14 > gpurun_out/${tag}_kstats_cfg3.txt
