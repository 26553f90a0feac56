# co-residence diagnosis: traces of the full-candidate step for k_repair builds at the default grid
set -o pipefail
O=gpurun_out/fc4
mkdir -p $O
export TMPDIR=/tmp
for v in n512 rk2; do
  KOLM_LIB=$PWD/ab/$v/libkolm_hip.so timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_$v -o fc -- python3 bench.py --steps 1 --warmup 1 --kt-steps 0 --no-serial-pass --no-cpu-baseline --full-steps 1 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
done
echo ok
