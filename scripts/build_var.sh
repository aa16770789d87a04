#!/bin/bash
# Build the working tree's libfftconv_amd.so with a sed patch applied to the
# kernels into build/var/NAME/ (for same-process or back-to-back A/B).
#   scripts/build_var.sh NAME 'sed-expression' [file]
set -eu
name=$1; expr=$2; file=${3:-csrc/kernels.hip}
root=$(cd "$(dirname "$0")/.." && pwd)
dst=$root/build/var/$name
rm -rf "$dst" && mkdir -p "$dst"
cp -r "$root/fft-convolution_amd" "$root/include" "$dst/"
rm -rf "$dst/fft-convolution_amd/build" "$dst/fft-convolution_amd/libfftconv_amd.so"
sed -i "$expr" "$dst/fft-convolution_amd/$file"
make -s -C "$dst/fft-convolution_amd" >/dev/null
echo "$dst/fft-convolution_amd/libfftconv_amd.so"
