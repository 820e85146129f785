#!/bin/bash
# Developer GPU script: the debug-sort graph test and the default bench line
# (trials: pure / as-test / cold).
set -o pipefail
cd "$(dirname "$0")/.."
T=${TAG:-astest}
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_graph.py tests/test_gpu_sort.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
exit 0
