set -o pipefail
O=gpurun_out/rpi
mkdir -p $O
KOLM_RP_PROF=1 timeout -k 10 200 python tools/rp_trace.py run $O 1 enwik > $O/x1.log 2>&1 || { tail -20 $O/x1.log; exit 1; }
KOLM_RP_PROF=1 timeout -k 10 200 python tools/rp_trace.py run $O 256 enwik > $O/x256.log 2>&1 || { tail -20 $O/x256.log; exit 1; }
grep -h "ms_repair\|Re-Pair sections" $O/x1.log $O/x256.log
