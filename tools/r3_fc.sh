# full-candidate (ids 0..9) step: kernel trace to see what runs beside / after k_repair
set -o pipefail
O=gpurun_out/fc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o fc -- python3 bench.py --steps 1 --warmup 1 --kt-steps 0 --no-serial-pass --no-cpu-baseline --full-steps 1 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
find $O/tr -name "*kernel_trace.csv" -exec cp {} $O/fc_trace.csv \;
ls -la $O
