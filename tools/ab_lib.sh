#!/bin/bash
# Same-box A/B of the headline: the production library against an alternative
# in-tree build (STG_CODEC_LIB), two benches each, then a kernel-stats profile of
# each.  Usage: bash tools/ab_lib.sh stellatrain_amd/libstg_codec_<variant>.so
set -o pipefail
ALT=$PWD/$1
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
    timeout -k 10 120 python bench.py --cpu-seconds 0 | tail -1 > gpurun_out/new$i.json || exit 1
    STG_CODEC_LIB=$ALT timeout -k 10 120 python bench.py --cpu-seconds 0 | tail -1 > gpurun_out/alt$i.json || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/p_new -o run -- \
    python3 bench.py --cpu-seconds 0 --steps 100 > /dev/null 2>&1 || exit 1
STG_CODEC_LIB=$ALT timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/p_alt \
    -o run -- python3 bench.py --cpu-seconds 0 --steps 100 > /dev/null 2>&1 || exit 1
