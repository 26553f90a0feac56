#!/bin/bash
# A/B of library builds in one GPU session, alternating: the hot-path step, config 4's shard and
# configs 2 / 5 per run.   bash tools/ab2.sh OUT A.so B.so [rounds]
OUT=$1; A=$2; B=$3; R=${4:-2}
mkdir -p $OUT
for i in $(seq 1 $R); do
  for L in $A $B; do
    tag=$(basename $L .so)_$i
    KOLM_LIB=$L timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --full-steps 0 --decode-steps 0 \
      --cdc-steps 0 --v2-steps 0 --host-steps 0 --no-serial-pass > $OUT/$tag.json 2> $OUT/$tag.err || { tail -20 $OUT/$tag.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$OUT/$tag.json'));t=d['detail']
c=t.get('configs',{});s=t.get('config4_shard',{})
print('$tag', d['value'], d['ms_per_step'], t['parity_blocks'], 'shard', s.get('ms_per_step'), s.get('parity_blocks'),
      ' '.join(f\"{n}:{v['ids0_8']['ms_per_call']}\" for n,v in c.items()), flush=True)" | tee -a $OUT/ab.txt
  done
done
