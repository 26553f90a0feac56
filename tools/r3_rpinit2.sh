set -o pipefail
O=gpurun_out/rpi2
mkdir -p $O
export KOLM_LIB=$PWD/ab/initprof/libkolm_hip.so
KOLM_RP_PROF=1 timeout -k 10 200 python tools/rp_trace.py run $O 256 enwik > $O/x256.log 2>&1 || { tail -20 $O/x256.log; exit 1; }
grep -h "ms_repair\|Re-Pair sections" $O/x256.log
