#!/bin/bash
# SQ counters of one kernel (default k_lz_local) on the hot-path bench step, two PMC passes of
# at most 8 SQ counters each (rocprofv3 collects one pass per run; kernel-trace domain only),
# then tools/sq_summary.py turns them into per-wave figures.  Run on the GPU box:
#   bash tools/sq_lz.sh OUT [KERNEL_REGEX] [extra bench args]
OUT=${1:-gpurun_out/sq}
RE=${2:-k_lz_local}
ARGS="--mib 256 --steps 1 --warmup 0 --kt-steps 1 --no-serial-pass --no-cpu-baseline --full-steps 0 --decode-steps 0 \
--cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 --c4-steps 0 $3"
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"
P2="SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$RE" -d "$OUT/p$i" -o pmc --output-format csv \
    -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1 || { tail -20 "$OUT/p$i.log"; exit 1; }
done
python3 tools/sq_summary.py "$OUT" > "$OUT/sq_summary.txt" && cat "$OUT/sq_summary.txt"
