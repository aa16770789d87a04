#!/bin/bash
# cfg2 launch-shape knobs read from the environment, back to back on one box
set -u
for spec in "X=0" "FFTCONV_LA_STEPS_FIRST=1" "FFTCONV_LA_MIDWG=1" "X=0" "FFTCONV_LA_STEPS_FIRST=1" "FFTCONV_LA_MIDWG=1"; do
  env $spec timeout -k 10 120 python bench.py --steps 2000 --no-cpu-baseline --pmc off > gpurun_out/envab.json 2>/dev/null || exit 3
  echo "$spec $(python -c "import json; d=json.load(open('gpurun_out/envab.json')); print(d['roofline']['launch_us'])")"
done
