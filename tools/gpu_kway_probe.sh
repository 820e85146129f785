#!/bin/bash
# The k-way graph-replay tests, then the k-way leg alone (BASELINE config 4)
# with graph / crash diagnostics.
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
T=${TAG:-r05k}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kway.py -m gpu \
    > gpurun_out/${T}_tests.log 2>&1 || exit $?
SFHE_GRAPH_DEBUG=1 SFHE_CRASH_TRACE=1 timeout -k 10 400 python -u -c "
import sys, json, time; sys.path.insert(0, '.'); sys.path.insert(0, 'sorting-fhe_amd/python')
import bench
print(json.dumps(bench.kway_leg(0)), flush=True)
" > gpurun_out/${T}_kway.json 2> gpurun_out/${T}_kway.err
echo "rc=$?" >> gpurun_out/${T}_kway.err
exit 0
