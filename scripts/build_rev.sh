#!/bin/bash
# Build libfftconv_amd.so of git revision REV into build/rev/REV/ (for same-process A/B).
set -eu
rev=$1
root=$(cd "$(dirname "$0")/.." && pwd)
dst=$root/build/rev/$rev
rm -rf "$dst" && mkdir -p "$dst"
git -C "$root" archive "$rev" fft-convolution_amd include | tar -x -C "$dst"
make -s -C "$dst/fft-convolution_amd" >/dev/null
echo "$dst/fft-convolution_amd/libfftconv_amd.so"
