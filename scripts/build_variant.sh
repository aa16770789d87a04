#!/bin/bash
# build_variant.sh NAME "-DMACRO=V ..." -- an A/B build of libfftconv_amd.so
# under build/var/NAME (scripts/ab_libs.py compares builds in one process)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
DEFS="$*"
OUT=$ROOT/build/var/$NAME
mkdir -p "$OUT"
make -s -C "$ROOT/fft-convolution_amd" OBJ="$OUT" LIB="$OUT/libfftconv_amd.so" \
    CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result $DEFS"
