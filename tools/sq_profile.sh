#!/bin/bash
# Instruction-mix / stall counters per kernel (one rocprofv3 --pmc pass per group, kernel
# trace only), streams serialised so each kernel is measured alone.
set -e
OUT=${1:-gpurun_out/sq}
ARGS=${2:-"--mib 256 --steps 1 --warmup 1 --no-cpu-baseline"}
mkdir -p $OUT
export TMPDIR=/tmp KOLM_SERIAL=1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD -d $OUT/p1 -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR -d $OUT/p2 -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/p2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT -d $OUT/p3 -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/p3.log 2>&1
echo sq done
