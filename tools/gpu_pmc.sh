#!/bin/bash
# PMC passes only (developer script): HBM traffic (FETCH_SIZE / WRITE_SIZE,
# separate runs) and the SQ cycle breakdown over tools/build/microbench.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp MB_REPS=3
( time timeout -k 5 60 tools/build/microbench 16 ) > gpurun_out/mb_plain.log 2>&1 || exit 1
timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcF -o run -- tools/build/microbench 16 > gpurun_out/pmcF.log 2>&1 || exit 1
timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcW -o run -- tools/build/microbench 16 > gpurun_out/pmcW.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/pmcF/run_counter_collection.csv gpurun_out/pmcW/run_counter_collection.csv --n 65536 --out gpurun_out/pmc_traffic.json > gpurun_out/pmc.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmcSQ -o run -- tools/build/microbench 16 > gpurun_out/pmcSQ.log 2>&1
