#!/bin/bash
# Developer GPU script: parity / fusion / graph tests, the microbench, then the default bench.
set -o pipefail
cd "$(dirname "$0")/.."
T=${TAG:-r04j}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_parity_metric.py tests/test_fusion.py tests/test_gpu_ntt_variants.py tests/test_gpu_graph.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
timeout -k 10 120 tools/build/microbench 16 > gpurun_out/${T}_microbench.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
[ -n "$PROFILE" ] && { bash tools/profile_round.sh "$T" || exit $?; }
exit 0
