#!/bin/bash
# Round-6 PMC A/B (developer script), from the repo root on the box:
#   TAG=r06r AB="SFHE_ROWTAB=0" bash tools/gpu_r06_pmc.sh
# The FETCH_SIZE / WRITE_SIZE passes of tools/profile_round.sh over the
# microbench, at the default settings and again under each AB setting:
# gpurun_out/<tag>_pmc_traffic[_<ab>].json (tools/pmc_traffic.py).
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r06x}
mkdir -p gpurun_out
for ab in default $AB; do
    sfx=$([ "$ab" = default ] && echo "" || echo "_$ab")
    envs=$([ "$ab" = default ] && echo "" || echo "$ab")
    for c in FETCH_SIZE WRITE_SIZE; do
        env $envs MB_REPS=3 timeout -s KILL 170 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${T}_${c}${sfx} -o run \
            -- tools/build/microbench 16 > gpurun_out/pmc_${T}_${c}${sfx}.log 2>&1 || exit $?
    done
    python3 tools/pmc_traffic.py gpurun_out/pmc_${T}_FETCH_SIZE${sfx}/run_counter_collection.csv \
        gpurun_out/pmc_${T}_WRITE_SIZE${sfx}/run_counter_collection.csv --n 65536 \
        --mb-log gpurun_out/pmc_${T}_FETCH_SIZE${sfx}.log --out gpurun_out/${T}_pmc_traffic${sfx}.json \
        > /dev/null 2>&1 || exit $?
done
exit 0
