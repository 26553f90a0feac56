#!/bin/bash
# A/B of library builds in one GPU session: alternating bench runs (hot path only).
#   bash tools/ab.sh OUT ab/A.so ab/B.so [rounds]
OUT=$1; A=$2; B=$3; R=${4:-3}
mkdir -p $OUT
for i in $(seq 1 $R); do
  for L in $A $B; do
    KOLM_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    python3 -c "
import json,sys;d=json.load(open('$OUT/b.json'));print('$L', d['value'], d['ms_per_step'], flush=True)" | tee -a $OUT/ab.txt
  done
done
