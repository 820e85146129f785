#!/bin/bash
# Round-6 GPU call (developer script), from the repo root on the box:
#   TAG=r06b TESTS="tests/test_x.py" CHAIN=1 BENCH=1 AB="SFHE_ICOL=0" CHAINPROF=mult bash tools/gpu_r06.sh
# TESTS: pytest selection run with -m gpu (TESTS=all: the whole suite);
# CHAIN: tools/build/chainbench (and again under each AB setting);
# BENCH: the short metric bench (BENCHARGS replaces its arguments), again
# under each AB setting, alternating, REPS times.  Every step has its own
# time limit and the first failure ends the call.
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
T=${TAG:-r06x}
O=gpurun_out/$T
mkdir -p $O
if [ -n "$TESTS" ]; then
    [ "$TESTS" = all ] && TESTS=tests
    timeout -k 10 ${TESTS_LIMIT:-900} python -u -m pytest -x -v --timeout 600 --timeout-method thread --durations=15 \
        $TESTS -m gpu > $O/gpu_tests.log 2>&1 || exit $?
fi
if [ -n "$CHAIN" ]; then
    timeout -k 10 240 tools/build/chainbench ${CHAIN_REPS:-20} > $O/chain.log 2>&1 || exit $?
    for ab in $AB; do
        env ${ab//+/ } timeout -k 10 240 tools/build/chainbench ${CHAIN_REPS:-20} > $O/chain_$ab.log 2>&1 || exit $?
    done
fi
if [ -n "$BENCH" ]; then
    B=${BENCHARGS:-"--steps 10 --warmup 3 --no-kway --no-cpu-baseline --no-hybrid1 --no-c5 --trials 3"}
    for r in $(seq 1 ${REPS:-1}); do
        timeout -k 10 400 python -u bench.py $B > $O/bench$r.json 2> $O/bench$r.err || exit $?
        for ab in $AB; do  # (one setting per word; '+' joins several)
            env ${ab//+/ } timeout -k 10 400 python -u bench.py $B > $O/bench${r}_$ab.json 2> $O/bench${r}_$ab.err || exit $?
        done
    done
fi
if [ -n "$CHAINPROF" ]; then  # kernel trace of one chain (CHAINPROF = chainbench's chain list)
    export TMPDIR=/tmp
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cprof -o run -- \
        tools/build/chainbench 3 $CHAINPROF > $O/chainprof.log 2>&1 || exit $?
fi
exit 0
