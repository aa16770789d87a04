#!/bin/bash
# kernel-trace stats of cfg3 for one library build (FFTCONV_AMD_LIB), run on the GPU box
set -u
lib=$1; tag=$2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
FFTCONV_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o kt --output-format csv -- python3 scripts/bench_configs.py --configs 3 --no-cpu > gpurun_out/prof_$tag.log 2>&1 || exit 4
find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1 | xargs grep tail0
