# price of a follow-on launch with nothing to do, after each lone call
# (tools/lone_bench single row; STG_DEBUG_NOOP = its workgroups, _LDS = dynamic LDS bytes each)
for cfg in "0 0" "1 0" "256 0" "1 156672" "256 156672" "0 0"; do
    set -- $cfg
    echo "noop grid=$1 lds=$2"
    STG_DEBUG_NOOP=$1 STG_DEBUG_NOOP_LDS=$2 timeout -k 10 120 ./tools/lone_bench 0 96 || exit $?
done
