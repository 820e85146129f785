# One GPU call's worth of round profiling (run from the repo root on the box):
#  1. rocprofv3 kernel trace + stats of the bench (graph-replayed timed sorts)
#     -> gpurun_out/<tag>_rocprof_summary.txt (tools/trace_segments.py) and
#        <tag>_kernel_stats.csv;
#  2. two PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs: gfx950 cannot
#     collect both in one) over tools/build/microbench -- the NTT at 1..96
#     limbs plus the key-switch prims at the top level, eagerly launched.  A
#     whole sort under PMC serialises ~5.5 k dispatches with counter reads and
#     outlives the box's 180 s silence limit, so the traffic ratio comes from
#     the same kernels on the microbench -> gpurun_out/pmc_traffic.json.
#   bash tools/profile_round.sh <tag>
set -e
tag=${1:-rXX}
mkdir -p gpurun_out
export TMPDIR=/tmp
# the bench's roofline replay re-instantiates graph nodes; the profiler's
# rewritten nodes are not replayed (the trace itself gives the durations)
export SFHE_NO_GRAPH_REPLAY=1
# --c5-eager: the 2^17 sort's graph replay segfaults inside librocprofiler-sdk
# under the kernel tracer; its kernels are traced eagerly
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --trials 0 --no-cpu-baseline --no-hybrid1 --no-kway --c5-eager > gpurun_out/prof_bench.log 2>&1
python3 tools/trace_segments.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/${tag}_rocprof_summary.txt 2>&1
cp gpurun_out/prof/run_kernel_stats.csv gpurun_out/${tag}_kernel_stats.csv
MB_REPS=3 timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcF -o run -- tools/build/microbench 16 > gpurun_out/pmcF.log 2>&1
MB_REPS=3 timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcW -o run -- tools/build/microbench 16 > gpurun_out/pmcW.log 2>&1
python3 tools/pmc_traffic.py gpurun_out/pmcF/run_counter_collection.csv gpurun_out/pmcW/run_counter_collection.csv --n 65536 --mb-log gpurun_out/pmcF.log --out gpurun_out/pmc_traffic.json > gpurun_out/pmc.log 2>&1
# where the conversion / NTT waves spend their cycles (one SQ pass, 8 counters)
MB_REPS=3 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmcSQ -o run -- tools/build/microbench 16 > gpurun_out/pmcSQ.log 2>&1 || true
