#!/bin/bash
# One-bucket finish variants (GPU box): rocprof kernel traces of the
# single-bucket row under each env setting; per-kernel duration stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() {  # name env...
    local name=$1; shift
    env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/sw_$name" -o run \
        -- python3 tools/bench_configs.py --only single > "gpurun_out/sw_$name.log" 2>&1 || return 1
    echo "== $name $*" >> gpurun_out/sweep.txt
    grep single "gpurun_out/sw_$name.log" >> gpurun_out/sweep.txt
    python3 tools/ktrace.py "gpurun_out/sw_$name" | grep tv16 >> gpurun_out/sweep.txt
}
for v in ${SWEEP:-"default:STG_X=1" "shape1:STG_TV16_LSHAPE=1" "w32:STG_TV16_LFIN_WORKERS=32" "r16:STG_TV16_LFIN_RANKERS=16"}; do
    run "${v%%:*}" "${v#*:}" || break
done
