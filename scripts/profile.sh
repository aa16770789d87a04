#!/bin/bash
# Kernel-trace stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the
# bench workload; run on the GPU box from the repo root.  Usage:
#   scripts/profile.sh TAG [extra bench args...]
set -u
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/prof_$tag
mkdir -p "$out"
B="bench.py --no-cpu-baseline --pmc off $*"
scripts/gpu_step.sh "kt_$tag" 400 rocprofv3 --kernel-trace --stats -d "$out/kt" -o kt --output-format csv -- python3 $B --steps 1000 --warmup 200 &&
scripts/gpu_step.sh "fetch_$tag" 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex upols -d "$out/fetch" -o fetch --output-format csv -- python3 $B --steps 30 --warmup 5 &&
scripts/gpu_step.sh "write_$tag" 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex upols -d "$out/write" -o write --output-format csv -- python3 $B --steps 30 --warmup 5
