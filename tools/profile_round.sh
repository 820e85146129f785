# One GPU call's worth of round profiling (run from the repo root on the box):
# rocprofv3 kernel trace + stats, two PMC passes (FETCH_SIZE / WRITE_SIZE),
# HBM traffic per launch -> profiles/pmc_traffic.json (copied back through
# gpurun_out/), host enqueue probe, then the full bench line.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --trials 0 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcF -o run -- python3 bench.py --steps 1 --warmup 1 --trials 0 --no-cpu-baseline > gpurun_out/pmcF.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcW -o run -- python3 bench.py --steps 1 --warmup 1 --trials 0 --no-cpu-baseline > gpurun_out/pmcW.log 2>&1
python3 tools/pmc_traffic.py gpurun_out/pmcF/run_counter_collection.csv gpurun_out/pmcW/run_counter_collection.csv --n 65536 --out gpurun_out/pmc_traffic.json > gpurun_out/pmc.log 2>&1
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 200 python3 tools/hostbound.py > gpurun_out/hostbound.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_full.log 2>&1
