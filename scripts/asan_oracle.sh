#!/bin/bash
# The CPU test suite against the AddressSanitizer + UBSan build of the oracle
# (make -C oracle asan).  The ASan runtime must come first in the process, so
# it is preloaded into python; leak checking is off (the interpreter's own
# allocations are not ours), every other ASan / UBSan report aborts the run.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
make -s -C "$ROOT/oracle" asan
ASAN_RT="$(gcc -print-file-name=libasan.so)"
UBSAN_RT="$(gcc -print-file-name=libubsan.so)"
export LD_PRELOAD="$ASAN_RT:$UBSAN_RT"
export ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
export ORACLE_LIB="$ROOT/oracle/liboracle_asan.so"
cd "$ROOT"
python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
