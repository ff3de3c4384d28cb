#!/bin/bash
# GPU-box driver: runs the named steps in order, each under its own time limit,
# and stops at the first step that ends in anything but success or an ordinary
# test failure (pytest rc 1).  Logs go to gpurun_out/<step>.log.
#   tools/gpu_run.sh tests bench breakdown prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp

step() {  # name limit cmd...
    local name=$1 limit=$2
    shift 2
    echo "[$(date +%T)] start $name" >> gpurun_out/summary.txt
    timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "[$(date +%T)] $name rc=$rc" >> gpurun_out/summary.txt
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after $name (rc=$rc)" >> gpurun_out/summary.txt
        exit $rc
    fi
}

for s in "$@"; do
    case $s in
        tests) step tests 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread ;;
        tests_all) step tests_all 900 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread ;;
        tests_tv16) step tests_tv16 600 python -u -m pytest tests/test_gpu_codecs.py tests/test_gpu_configs.py tests/test_gpu_coresidency.py tests/test_gpu_fill_modes.py -v -m gpu --timeout 120 --timeout-method thread ;;
        stale_ctl)  # negative control: the one-bucket count pairs pre-tagged as recycled memory would be
            STG_DEBUG_LDESC_STALE=1 step stale_ctl 300 python -u -m pytest tests/test_gpu_gather_fused.py -v -m gpu --timeout 120 --timeout-method thread ;;
        smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
        bench) step bench 400 python bench.py ;;
        bench_jitter) step bench_jitter 400 python bench.py --jitter 0.05 --no-cpu-baseline ;;
        prof_jitter) step prof_jitter 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_jitter" -o run \
                -- python3 bench.py --steps 100 --warmup 8 --no-cpu-baseline --c4-sweeps 0 --jitter 0.05 ;;
        prof_fresh) step prof_fresh 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_fresh" -o run \
                -- python3 bench.py --steps 100 --warmup 8 --no-cpu-baseline --c4-sweeps 0 ;;
        bench_short) step bench_short 300 python bench.py --steps 40 --warmup 8 --cpu-seconds 5 ;;
        breakdown) step breakdown 300 python tools/breakdown.py ;;
        breakdown_d3) step breakdown_d3 300 python tools/breakdown.py --dist 2 --param 9000 ;;
        prof) step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run \
                -- python3 bench.py --steps 50 --warmup 8 --no-cpu-baseline ;;
        pmc_fetch) step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
                -d "$R/gpurun_out/pmc_fetch" -o run -- python3 bench.py --steps 16 --warmup 4 --profile-steps 4 --no-cpu-baseline ;;
        pmc_write) step pmc_write 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv \
                -d "$R/gpurun_out/pmc_write" -o run -- python3 bench.py --steps 16 --warmup 4 --profile-steps 4 --no-cpu-baseline ;;
        prof_s1|prof_s3)  # scan work only (1) / plain streaming read (3): STG_DEBUG_TV16_STAGE
            export STG_DEBUG_TV16_STAGE=${s#prof_s}
            step $s 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$s" -o run \
                -- python3 bench.py --steps 50 --warmup 8 --no-cpu-baseline
            unset STG_DEBUG_TV16_STAGE ;;
        ubench) step ubench 300 python tools/ubench_read.py ;;
        configs) step configs 500 python tools/bench_configs.py ;;
        single) step single 200 python tools/bench_configs.py --only single ;;
        prof_single) step prof_single 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_single" -o run \
                -- python3 tools/bench_configs.py --only single ;;
        c2) step c2 300 python tools/bench_configs.py --only c2 ;;
        prof_topk) step prof_topk 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_topk" -o run -- python3 tools/bench_configs.py --only topk --cpu-seconds 0
            python3 tools/ktrace.py gpurun_out/prof_topk > gpurun_out/prof_topk.txt 2>&1 ;;
        prof_c5) step prof_c5 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_c5" -o run -- python3 tools/bench_configs.py --only c5
            python3 tools/ktrace.py gpurun_out/prof_c5 24 > gpurun_out/prof_c5.txt 2>&1 ;;
        prof_merge) step prof_merge 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_merge" -o run -- python3 tools/bench_configs.py --only merge
            python3 tools/ktrace.py gpurun_out/prof_merge 16 > gpurun_out/prof_merge.txt 2>&1 ;;
        scale_drop) step scale_drop 280 python tools/scale_drop.py 4 ${DROPS:-100,10,2,1.1} ;;
        fill_paths) step fill_paths 200 python tools/fill_paths.py --steps 400 ;;
        tiny) step tiny 120 python tools/tiny_probe.py
            STG_DEBUG_TV16_FILL=2 step tiny_literal 120 python tools/tiny_probe.py ;;
        tests_topk1) step tests_topk1 600 python -u -m pytest tests/test_gpu_topk1.py tests/test_gpu_codecs.py tests/test_gpu_configs.py -k "topk or c2 or hint" -v -m gpu --timeout 300 --timeout-method thread ;;
        tests_wide) step tests_wide 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_fill_modes.py -v -s -m gpu --timeout 300 --timeout-method thread ;;
        tests_topk) step tests_topk 400 python -u -m pytest tests/test_gpu_codecs.py tests/test_gpu_configs.py tests/test_gpu_api.py -k "topk or c2" -v -m gpu --timeout 120 --timeout-method thread ;;
        prof_c2) step prof_c2 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_c2" -o run -- python3 tools/bench_configs.py --only c2
            python3 tools/ktrace.py gpurun_out/prof_c2 > gpurun_out/prof_c2.txt 2>&1 ;;
        c3) step c3 300 python tools/bench_configs.py --only c3 ;;
        tests_tv) step tests_tv 400 python -u -m pytest tests -k "thresholdv and not thresholdv16 or c3 or tv_" -v -m gpu --timeout 120 --timeout-method thread ;;
        c4) step c4 300 python tools/bench_configs.py --only c4 ;;
        c5) step c5 300 python tools/bench_configs.py --only c5 ;;
        apply) step apply 300 python tools/bench_configs.py --only c5,apply ;;
        ef) step ef 300 python tools/bench_configs.py --only ef ;;
        gather) step gather 300 python tools/bench_configs.py --only gather ;;
        gfused) step gfused 300 python tools/bench_configs.py --only gfused,single ;;
        wfused) step wfused 300 python tools/bench_configs.py --only wfused ;;
        tests_wire) step tests_wire 600 python -u -m pytest tests/test_gpu_wire_fused.py tests/test_gpu_wire.py -v -m gpu --timeout 120 --timeout-method thread ;;
        prof_apply) step prof_apply 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_apply" -o run \
                -- python3 tools/bench_configs.py --only apply ;;
        lone_bench) step lone_bench 200 ./tools/lone_bench 16 96 ;;
        prof_lone_bench) step prof_lone_bench 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_lone_bench" -o run -- ./tools/lone_bench 16 96 ;;
        prof_lone)  # kernel durations of the single-caller lone bench (production library)
            step prof_lone 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_lone" -o run -- ./tools/lone_bench 0 96
            python3 tools/ktrace.py gpurun_out/prof_lone 12 > gpurun_out/prof_lone.txt 2>&1 ;;
        lfin_probe) step lfin_probe 200 python tools/lfin_probe.py ;;
        *) echo "unknown step $s" >> gpurun_out/summary.txt ;;
    esac
done
echo "[$(date +%T)] all done" >> gpurun_out/summary.txt
