#!/bin/bash
# Attribution runs on the GPU box (developer script): hybrid II's series stage
# (tools/prec_probe.cpp h2s) at N = 64, 128, 256 on ring 2^17, then the
# config-5 graph (tools/c5_graph.py) under rocprofv3's kernel trace.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
P=tools/build/prec_probe_hip
O=gpurun_out/${PROBE_TAG:-attr}
for n in 64 128 256; do
    timeout -k 10 240 $P h2s $n 17 1 > ${O}_h2s_$n.log 2>&1 || exit 1
done
PROBE_EXACT_RANK=1 timeout -k 10 240 $P h2s 256 17 1 > ${O}_h2s_256_exact.log 2>&1 || exit 1
export SFHE_CRASH_TRACE=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof -o run -- \
    python3 tools/c5_graph.py --replays 2 > ${O}_c5prof.log 2>&1
echo "c5 rocprof rc=$?" >> ${O}_c5prof.log
