set -o pipefail
O=gpurun_out/lzp
mkdir -p $O
KOLM_LZ_PROF=1 timeout -k 10 200 python tools/lz_probe.py mixed > $O/mixed.log 2>&1 || { tail -20 $O/mixed.log; exit 1; }
cat $O/mixed.log | cut -c1-3000
