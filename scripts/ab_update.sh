#!/bin/bash
# cfg2u (update_device every 128 blocks) for two library builds, alternating
# processes, plus one rocprofv3 kernel trace of each (the update's IR
# transform and window rebuild).  usage: ab_update.sh LIB_A LIB_B TAG  (GPU box)
set -u
A=$1; Bl=$2; tag=$3
for rep in 1 2; do
  for L in $A $Bl; do
    FFTCONV_AMD_LIB=$L timeout -k 10 200 python3 scripts/bench_configs.py --configs 2u --no-cpu 2>/dev/null | \
      python3 -c "import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print('$L rep=$rep', d['MSamples_s'], d['us_per_step'])" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for L in $A $Bl; do
  n=$(echo $L | md5sum | cut -c1-6)
  FFTCONV_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_$n -o kt --output-format csv -- python3 scripts/bench_configs.py --configs 2u --no-cpu > /dev/null 2>&1 || exit 4
  echo "== $L"; python3 scripts/kstats.py gpurun_out/prof_${tag}_$n 4
done
