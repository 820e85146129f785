#!/bin/bash
# Stacked launches: bit-exactness tests, then the metric sort A/B (stacked
# batches on / off), each bench leg-free and alternated twice on one box.
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
T=${TAG:-r05s}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_stack.py tests/test_gpu_parity_sort.py::test_metric_sort_bitexact tests/test_gpu_graph.py \
    tests/test_hybrid_variants.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit $?
B="--no-kway --no-hybrid1 --no-c5 --no-cpu-baseline --trials 5 --steps 20 --warmup 3"
for k in 1 2; do
    for v in 1 0; do
        SFHE_STACK_BATCHES=$v timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_stack${v}_$k.json 2> gpurun_out/${T}_stack${v}_$k.err || exit $?
    done
done
exit 0
