# full-candidate step with the Re-Pair grid below the CU count (diagnosis of co-residence)
set -o pipefail
O=gpurun_out/fc2
mkdir -p $O
export TMPDIR=/tmp
KOLM_RP_WS_GB=62.95 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o fc -- python3 bench.py --steps 1 --warmup 1 --kt-steps 0 --no-serial-pass --no-cpu-baseline --full-steps 1 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo ok
