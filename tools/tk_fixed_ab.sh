# Top-k superset slots A/B: fixed per-tile slots (default) against region offsets by atomics
for F in 1 0 1 0; do
    echo "FIXED=$F"
    STG_TK2_FIXED=$F timeout -k 10 120 python tools/bench_configs.py --only c2 --cpu-seconds 0 | grep '"config": "topk' | cut -c1-120 || exit 1
done
