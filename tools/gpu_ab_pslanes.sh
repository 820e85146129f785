#!/bin/bash
# Developer A/B (round 4): the Chebyshev PS on lanes (SFHE_PS_LANES) for
# one-batch sorts -- config 3 (DirectSort<128> @ 2^16) and config 5's sort
# (the bench's c5 leg, DirectSort<256> @ 2^17) -- off, on, off, on.
cd "$(dirname "$0")/.."
TAG=${TAG:-r04}
for k in off on off2 on2; do
  if [ "${k#on}" != "$k" ]; then export SFHE_PS_LANES=4; else unset SFHE_PS_LANES; fi
  timeout -k 10 200 python3 -u bench.py --workload directsort_n128_2e16 --steps 10 --warmup 3 --trials 0 \
      --no-cpu-baseline --no-kway --no-hybrid1 > gpurun_out/${TAG}_ab_${k}.log 2>&1 || exit $?
done
exit 0
