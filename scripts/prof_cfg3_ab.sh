#!/bin/bash
# kernel-trace stats of cfg3 for one library build through ab_cfg3.py (plain
# ctypes: any build's exports), run on the GPU box.  usage: prof_cfg3_ab.sh LIB TAG
set -u
lib=$1; tag=$2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o kt --output-format csv -- python3 scripts/ab_cfg3.py $lib --rounds 3 > gpurun_out/prof_$tag.log 2>&1 || exit 4
python3 scripts/kstats.py gpurun_out/prof_$tag 14
grep -h "us/step" gpurun_out/prof_$tag.log
