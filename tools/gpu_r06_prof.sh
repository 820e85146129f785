#!/bin/bash
# Round-6 profiling call (developer script), from the repo root on the box:
#   TAG=r06p bash tools/gpu_r06_prof.sh
#  1. tools/profile_round.sh: rocprofv3 kernel trace of the bench's graph-
#     replayed sorts + the FETCH_SIZE / WRITE_SIZE / SQ passes over the
#     microbench (tools/pmc_traffic.py: per family and, for the NTT, per pass);
#  2. config 4: one eager k-way sort (SFHE_GRAPH=0: the 2^17 graphs' replay
#     crashes inside the profiler) under the kernel tracer,
#     summarised per kernel (the raw trace is deleted: it is large).
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r06p}
mkdir -p gpurun_out
timeout -k 10 900 bash tools/profile_round.sh "$T" || exit $?
if [ -z "$NO_KWAY" ]; then
    SFHE_GRAPH=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kwprof -o run -- \
        python3 tools/kway_run.py --sorts 1 > gpurun_out/${T}_kway_prof.log 2>&1 || exit $?
    python3 tools/trace_segments.py gpurun_out/kwprof/run_kernel_trace.csv --gap-us 200000 --top 40 \
        > gpurun_out/${T}_kway_segments.txt 2>&1
    rm -f gpurun_out/kwprof/run_kernel_trace.csv
fi
exit 0
