#!/bin/bash
# Developer GPU script (round 4): the round's profile (tools/profile_round.sh:
# rocprofv3 trace + stats of the bench, PMC passes on the microbench), the
# bootstrapping precision probe at the k-way configuration (ring 2^17,
# S = 1024, {5, 5}) and a plain microbench run.  Outputs under gpurun_out/.
cd "$(dirname "$0")/.."
TAG=${TAG:-r04}
set -o pipefail
timeout -k 10 180 python3 -u tools/cold_probe.py > gpurun_out/${TAG}_cold_probe.txt 2>&1 || exit $?
timeout -k 10 240 python3 -u tools/split_probe.py > gpurun_out/${TAG}_split_probe.txt 2>&1 || exit $?
bash tools/profile_round.sh "$TAG" || exit $?
timeout -k 10 240 tools/build/boot_probe_hip 17 1024 5 5 > gpurun_out/${TAG}_boot_probe.txt 2>&1 || exit $?
timeout -k 10 120 tools/build/microbench 16 > gpurun_out/${TAG}_microbench.txt 2>&1 || exit $?
exit 0
