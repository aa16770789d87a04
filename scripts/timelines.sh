#!/bin/bash
# timelines.sh TAG LIB... -- FFTCONV_LA_TRACE launch timelines of cfg2 for each
# build (bench.py, 16 launches each) into gpurun_out/TAG_<name>.0
set -e
TAG=$1; shift
for L in "$@"; do
    n=$(basename "$(dirname "$L")")
    FFTCONV_AMD_LIB=$L FFTCONV_LA_TRACE=16 FFTCONV_LA_TRACE_OUT=gpurun_out/${TAG}_$n \
        timeout -k 10 120 python bench.py --steps 300 --warmup 100 --no-cpu-baseline --pmc off > gpurun_out/${TAG}_$n.log 2>&1
done
