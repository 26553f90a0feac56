# Duval span / merge phase profile (KOLM_DUVAL_PROF=1) on the bench stream
set -o pipefail
O=gpurun_out/dprof
mkdir -p $O
KOLM_DUVAL_PROF=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --kt-steps 0 --no-serial-pass --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
grep "duval" $O/b.err | tail -2
