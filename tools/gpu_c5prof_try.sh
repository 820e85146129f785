#!/bin/bash
# Bench (lazy on / off) and a retry of the config-5 graph under rocprofv3's
# kernel trace with HIP's graph packet batching off (developer script).
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${PROBE_TAG:-c5try}
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-kway --no-c5 --no-cpu-baseline --trials 3 > ${O}_bench.log 2>&1 || exit 1
SFHE_LAZY=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-kway --no-c5 --no-cpu-baseline --no-hybrid1 --trials 3 > ${O}_bench_nolazy.log 2>&1 || exit 1
export SFHE_CRASH_TRACE=1 DEBUG_HIP_GRAPH_PACKET_CAPTURE=0
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof2 -o run -- \
    python3 tools/c5_graph.py --replays 2 > ${O}_c5prof.log 2>&1
echo "c5 rocprof rc=$?" >> ${O}_c5prof.log
