#!/bin/bash
# Batched PS / power waves: bit-exactness tests, then the metric sort A/B
# (A: the default; B: $BENV, default SFHE_PS_WAVES=0), alternated twice on one box.
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
T=${TAG:-r05w}
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_parity_metric.py tests/test_gpu_parity_sort.py tests/test_gpu_graph.py \
    tests/test_gpu_stack.py tests/test_hybrid_variants.py tests/test_kway.py tests/test_gpu_sort.py -m gpu \
    > gpurun_out/${T}_tests.log 2>&1 || exit $?
fi
B="--no-kway --no-hybrid1 --no-c5 --no-cpu-baseline --trials 3 --steps 20 --warmup 3"
for k in 1 2; do
    timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_on_$k.json 2> gpurun_out/${T}_on_$k.err || exit $?
    env ${BENV:-SFHE_PS_WAVES=0} timeout -k 10 300 python -u bench.py $B > gpurun_out/${T}_off_$k.json 2> gpurun_out/${T}_off_$k.err || exit $?
done
exit 0
