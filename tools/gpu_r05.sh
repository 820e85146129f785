#!/bin/bash
# Round-5 GPU call (developer script), from the repo root on the box:
#   TAG=r05a TESTS="tests/test_x.py" BENCH=1 PROFILE=1 bash tools/gpu_r05.sh
# TESTS: pytest selection run with -m gpu (TESTS=all: the whole suite, as the
# driver runs it); BENCH: the default bench line (BENCHARGS appended);
# PROFILE: tools/profile_round.sh.  Every step has its own time limit and the
# first failure ends the call.
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
T=${TAG:-r05x}
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
    [ "$TESTS" = all ] && TESTS=tests
    timeout -k 10 ${TESTS_LIMIT:-1000} python -u -m pytest -x -v --timeout 900 --timeout-method thread --durations=15 \
        $TESTS -m gpu > gpurun_out/${T}_gpu_tests.log 2>&1 || exit $?
fi
if [ -n "$BENCH" ]; then
    timeout -k 10 600 python -u bench.py $BENCHARGS > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
fi
if [ -n "$PROFILE" ]; then
    bash tools/profile_round.sh "$T" || exit $?
fi
exit 0
