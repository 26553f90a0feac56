#!/bin/bash
# Kernel traces of the hot-path step under several environment settings (one rocprofv3 run each):
#   bash tools/kt_ab.sh OUT TAG:VAR=v+VAR2=w [TAG:...]
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--mib 256 --steps 1 --warmup 1 --kt-steps 0 --no-serial-pass --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 --c4-steps 0"
for spec in "$@"; do
  tag=${spec%%:*}; envs=$(echo "${spec#*:}" | tr '+' ' ')
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$tag -o kt --output-format csv -- python3 bench.py $ARGS > $OUT/$tag.log 2>&1 || { tail -20 $OUT/$tag.log; exit 1; }
  echo "$tag done"
done
