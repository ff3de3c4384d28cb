#!/bin/bash
# K1 (tv16_lscan) time attribution on the GPU box: the single-caller lone
# bench under rocprofv3 for the production library and the diagnostic builds
# libstg_codec_ld1.so (no per-chunk lists) / _ld2.so (plain stream).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in prod ld1 ld2; do
    dir=/tmp/lsd_$v; mkdir -p $dir
    if [ $v = prod ]; then cp stellatrain_amd/libstg_codec.so $dir/; else cp stellatrain_amd/libstg_codec_$v.so $dir/libstg_codec.so; fi
    LD_LIBRARY_PATH=$dir timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lsd_$v -o run \
        -- ./tools/lone_bench 0 96 > gpurun_out/lsd_$v.log 2>&1
    rc=$?; [ $rc -ge 124 ] && exit $rc  # the diagnostic builds fail stg_codec_check by design (wrong fills)
    echo "== $v" >> gpurun_out/lsd.txt
    grep single gpurun_out/lsd_$v.log >> gpurun_out/lsd.txt
    python3 tools/ktrace.py gpurun_out/lsd_$v | grep tv16 >> gpurun_out/lsd.txt
done
