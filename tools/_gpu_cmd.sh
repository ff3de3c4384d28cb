mkdir -p gpurun_out
STG_CODEC_LIB=$PWD/tools/variants/libstg_codec_lf2st.so LP_CALLS=30 timeout -k 10 120 python tools/lf2_probe.py > gpurun_out/lf2probe.log 2>&1 || exit $?
timeout -k 10 120 ./tools/lone_bench 16 96 > gpurun_out/lb.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pl -o run -- ./tools/lone_bench 0 96 > /dev/null 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_codecs.py tests/test_gpu_configs.py tests/test_gpu_wide.py tests/test_gpu_api.py tests/test_gpu_fill_modes.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
