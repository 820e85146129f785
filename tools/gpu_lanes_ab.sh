#!/bin/bash
# Developer A/B of runtime knobs on one box: HIP lanes per context (SFHE_LANES).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${PROBE_TAG:-lanes}
B="python bench.py --steps 10 --warmup 3 --no-kway --no-cpu-baseline --no-hybrid1 --no-c5 --trials 5"
for r in 1 2; do
    for L in 4 2 3; do
        SFHE_LANES=$L timeout -k 10 200 $B > ${O}_L$L.$r.log 2>&1 || exit $?
    done
done
exit 0
