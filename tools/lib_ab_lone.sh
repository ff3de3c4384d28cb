# tools/lone_bench single row + rocprof lscan time for the production library and each
# tools/variants/libstg_codec_<v>.so given (LD_LIBRARY_PATH picks the library lone_bench loads)
R=$(pwd)
PROD=prod; [ -n "${SKIP_PROD:-}" ] && PROD=
for v in $PROD "$@"; do
    d=$R/gpurun_out/ab_$v; mkdir -p $d
    if [ $v = prod ]; then cp stellatrain_amd/libstg_codec.so $d/; else cp tools/variants/libstg_codec_$v.so $d/libstg_codec.so; fi
    echo "== $v"
    LD_LIBRARY_PATH=$d timeout -k 10 120 ./tools/lone_bench 16 96 || exit $?
    LD_LIBRARY_PATH=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d/prof -o run -- ./tools/lone_bench 0 96 > $d/prof.log 2>&1 || exit $?
    python3 tools/kstats.py $d/prof | grep -E "lscan|fill"
    rm -f $d/libstg_codec.so
done
