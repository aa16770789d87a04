#!/bin/bash
# The lookahead, two-stage, crossfade, long-block, device-steps (run kernel)
# and Bluestein GPU tests against the debug build
# (make -C fft-convolution_amd debug-bounds): device bounds checks compiled in
# (FFTCONV_DEBUG_BOUNDS -- an out-of-range stream row, window row or state
# index prints "BOUNDS site ..." instead of touching memory) and UBSan on the
# host code.  Fails if any check fired.
set -uo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
export FFTCONV_AMD_LIB="$ROOT/fft-convolution_amd/libfftconv_amd_dbg.so"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
out=gpurun_out/debug_bounds.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_lookahead.py tests/test_gpu_twostage_defer.py \
    tests/test_gpu_crossfade_twostage.py tests/test_gpu_large.py tests/test_gpu_fullsize.py tests/test_gpu_windows.py \
    tests/test_gpu_device_steps.py tests/test_gpu_fft_any.py -v \
    --timeout 600 --timeout-method thread -s > "$out" 2>&1
rc=$?
echo "pytest rc=$rc"
if grep -q "BOUNDS site" "$out"; then echo "bounds checks fired:"; grep "BOUNDS site" "$out" | sort | uniq -c | head; exit 3; fi
if grep -q "runtime error" "$out"; then echo "UBSan reports:"; grep "runtime error" "$out" | head; exit 4; fi
tail -3 "$out"
exit $rc
