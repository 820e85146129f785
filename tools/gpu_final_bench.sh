#!/bin/bash
# Round-end measurements (developer script): the default bench line (all
# legs), the metric and config-5 sorts eagerly, and the precision tables.
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
O=gpurun_out/${PROBE_TAG:-fin}
timeout -k 10 600 python bench.py > ${O}_bench.log 2>&1 || exit 1
SFHE_GRAPH=0 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-kway --no-hybrid1 --no-cpu-baseline --trials 3 > ${O}_bench_eager.log 2>&1 || exit 1
timeout -k 10 300 python tools/precision_table.py > ${O}_prec_default.txt 2>&1 || exit 1
SFHE_LAZY=0 SFHE_SELF_OFFSET=0 SFHE_SINC_REBASE=0 timeout -k 10 300 python tools/precision_table.py > ${O}_prec_refordered.txt 2>&1
