# Top-k emission unit size A/B (STG_TK1_UNIT: superset entries per unit): C2 per setting
for U in ${UNITS:-2048 1024 512 256}; do
    echo "U=$U"
    STG_TK1_UNIT=$U timeout -k 10 120 python tools/bench_configs.py --only c2 --cpu-seconds 0 | grep '"config": "topk' | cut -c1-120 || exit 1
done
