#!/bin/bash
# cfg3 with the tail's side stream on 1/k of the CUs (FFTCONV_TAIL_CU_DIV),
# alternating processes, one handle per process (bench_configs.py --configs 3)
for rep in 1 2; do
  for k in ${KS:-1 2 3 5 8}; do
    FFTCONV_TAIL_CU_DIV=$k timeout -k 10 120 python3 scripts/bench_configs.py --configs 3 --no-cpu 2>/dev/null | \
      python3 -c "import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print('k=$k rep=$rep', d.get('host_loop'), d['MSamples_s'], d['us_per_step'])" || exit 1
  done
done
