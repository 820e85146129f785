#!/bin/bash
# k-way sort (BASELINE config 4) attribution on the GPU box (developer
# script): per-bootstrap synchronised times, then the kernel trace of the
# same run summarised per sort (the raw trace is deleted: it is large).
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${PROBE_TAG:-kw}
SFHE_BOOT_TRACE=1 timeout -k 10 400 python tools/kway_run.py --sorts 2 > ${O}_kway.log 2> ${O}_kway_boot.log || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kwprof -o run -- \
    python3 tools/kway_run.py --sorts 2 > ${O}_kway_prof.log 2>&1 || exit 1
python3 tools/trace_segments.py gpurun_out/kwprof/run_kernel_trace.csv --gap-us 20000 > ${O}_kway_segments.txt 2>&1
rm -f gpurun_out/kwprof/run_kernel_trace.csv
