set -u
for p in 0 1 3 5 6 0; do
  FFTCONV_LA_TIMING_PROBE=$p timeout -k 10 120 python bench.py --steps 1000 --warmup 200 --no-cpu-baseline --pmc off > gpurun_out/p$p.json 2>/dev/null || exit 3
  python -c "import json,sys; d=json.load(open('gpurun_out/p$p.json')); print('probe $p', d['roofline']['launch_us'])"
done
FFTCONV_LA_TRACE=16 FFTCONV_LA_TRACE_OUT=gpurun_out/tr_cfg2 timeout -k 10 120 python bench.py --steps 300 --warmup 200 --no-cpu-baseline --pmc off > gpurun_out/tr.json 2>&1 || exit 4
ls gpurun_out
