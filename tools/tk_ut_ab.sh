# Top-k: TK2_UT = 32 tiles per unit (libstg_codec_ut32.so) against the default 16, several unit sizes
for U in 1536 3072; do
    for L in "" stellatrain_amd/libstg_codec_ut32.so; do
        echo "U=$U LIB=${L:-default}"
        STG_CODEC_LIB=${L:+$PWD/$L} STG_TK1_UNIT=$U timeout -k 10 120 python tools/bench_configs.py --only c2 --cpu-seconds 0 | grep '"config": "topk' | cut -c1-120 || exit 1
    done
done
