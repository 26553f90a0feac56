# round 3: LSD histogram by ballot match (KOLM_LSD_HIST=1) vs LDS atomics per key
set -o pipefail
O=gpurun_out/r3h
mkdir -p $O
export TMPDIR=/tmp
KOLM_LSD_HIST=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_stream.py -x -q --timeout 200 --timeout-method thread -k "hot_path" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
KERNELS="k_lsd_hist" bash tools/kab.sh "KOLM_LSD_HIST=0" "KOLM_LSD_HIST=1" > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
