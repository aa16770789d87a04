#!/bin/bash
# cfg3 side-stream CU share sweep + a kernel-trace profile (run on the GPU box)
set -u
for k in 2 3 4; do
  FFTCONV_TAIL_CU_DIV=$k timeout -k 10 200 python scripts/bench_configs.py --configs 3 --no-cpu > gpurun_out/cfg3_div$k.log 2>&1 || exit 3
  echo "div $k: $(grep process_device_steps gpurun_out/cfg3_div$k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["MSamples_s"], d["us_per_step"])')"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg3 -o kt --output-format csv -- python3 scripts/bench_configs.py --configs 3 --no-cpu > gpurun_out/prof_cfg3.log 2>&1 || exit 4
find gpurun_out/prof_cfg3 -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-160
