#!/bin/bash
# Quick GPU check (developer script): bit-exact parity + graph tests, the
# precision attribution and FHERMA-flow numbers, then the bench with lazy
# rescaling on and off.  Output under gpurun_out/${PROBE_TAG}_*.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
O=gpurun_out/${PROBE_TAG:-quick}
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_fusion.py tests/test_gpu_graph.py tests/test_shard.py \
    "tests/test_gpu_sort.py::test_precision_attribution" "tests/test_serialization.py::test_fherma_flow_config_json" \
    > ${O}_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-kway --no-c5 --no-cpu-baseline --trials 3 > ${O}_bench.log 2>&1 || exit 1
SFHE_LAZY=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-kway --no-c5 --no-cpu-baseline --no-hybrid1 --trials 3 > ${O}_bench_nolazy.log 2>&1
[ -n "$C5PROF" ] || exit 0
# the config-5 sort (2^17) under the kernel trace, eagerly launched: replaying
# its captured graph under rocprofv3 segfaults inside the profiler
export TMPDIR=/tmp SFHE_GRAPH=0
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof_eager -o run -- \
    python3 tools/c5_graph.py --replays 2 > ${O}_c5prof.log 2>&1
