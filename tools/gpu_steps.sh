#!/bin/bash
# Developer GPU script (round 4): run the pytest selection in $TESTS (default:
# the whole -m gpu suite), then the bench with $BENCH_ARGS, writing
# gpurun_out/${TAG}_*.log.  A step that ends in anything but success or an
# ordinary test failure (rc 1) -- a timeout, an abort, a segfault -- ends the
# script: nothing else touches the GPU after it.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
O=gpurun_out/${TAG:-r04}
mkdir -p gpurun_out
ok() {  # rc of the last step: 0 / 1 go on, anything else stops
    local rc=$1 what=$2
    echo "$what rc=$rc" >> ${O}_steps.log
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
        echo "stopping after $what (rc=$rc)" >> ${O}_steps.log
        exit "$rc"
    fi
}
if [ "${TESTS:-}" != "none" ]; then
    timeout -k 10 ${TEST_TIMEOUT:-1000} python -u -m pytest ${PYTEST_X:--x} -v -s --timeout ${PER_TEST:-400} \
        --timeout-method thread --durations=20 -m gpu ${TESTS:-tests} > ${O}_tests.log 2>&1
    ok $? tests
fi
if [ "${BENCH_ARGS:-none}" != "none" ]; then
    timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py ${BENCH_ARGS} > ${O}_bench.log 2>&1
    ok $? bench
fi
exit 0
