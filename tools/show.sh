#!/bin/bash
# Summaries of the last GPU call's logs (run here, after gpurun).
cd "$(dirname "$0")/.."
for f in gpurun_out/*.log; do
    case $f in *tests*|*stamps*|*summary*) continue ;; esac
    l=$(tail -1 "$f")
    echo "$f: $(echo "$l" | python3 -c "import json,sys
try:
    d=json.loads(sys.stdin.read()); r=d.get('roofline',{})
    print(d['value'], r.get('avg_us'), d.get('per_bucket_us'), r.get('frac'))
except Exception as e: print('n/a')")"
done
[ -f gpurun_out/stamps.log ] && grep -E "W_Rn|phase" gpurun_out/stamps.log | tail -6
[ -f gpurun_out/summary.txt ] && cat gpurun_out/summary.txt
for f in gpurun_out/tests*.log; do [ -f "$f" ] && { echo "$f"; grep -E "passed|failed|FAILED|Error" "$f" | tail -5; }; done
python3 -c "import json;d=json.load(open('gpurun_out/.last_call.json'));print(d['status'],d.get('rc'),d.get('msg',''))" 2>/dev/null
