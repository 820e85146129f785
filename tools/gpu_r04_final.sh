#!/bin/bash
# Round-4 closing GPU call (developer script): the whole -m gpu suite as the
# driver runs it, the default bench line, an A/B of the lane-parallel baby
# rotations (SFHE_BABY_LANES=1 vs the default), then the round's profile.
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
T=${TAG:-r04z}
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread --durations=15 tests -m gpu > gpurun_out/${T}_gpu_suite.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
B="python bench.py --steps 10 --warmup 3 --no-kway --no-cpu-baseline --no-hybrid1 --no-c5 --trials 0"
SFHE_BABY_LANES=1 timeout -k 10 300 $B > gpurun_out/${T}_baby1.json 2>/dev/null || exit $?
timeout -k 10 300 $B > gpurun_out/${T}_baby4.json 2>/dev/null || exit $?
[ -n "$PROFILE" ] && { bash tools/profile_round.sh "$T" || exit $?; }
exit 0
