# C2 (Top-k) A/B: the production library against an alternative in-tree build, alternating
ALT=$PWD/$1
for L in "" "$ALT" "" "$ALT"; do
    echo "LIB=${L:-default}"
    STG_CODEC_LIB=$L timeout -k 10 120 python tools/bench_configs.py --only c2 --cpu-seconds 0 | grep '"config": "topk' | cut -c1-120 || exit 1
done
