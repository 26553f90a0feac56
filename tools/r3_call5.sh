# round 3: correctness of the slab MTF / emit / lane-wise hist; A/B of hist loads and LZ77 start
set -o pipefail
O=gpurun_out/r3f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_bench_stream.py tests/test_gpu_parity.py tests/test_cdc.py tests/test_decode.py -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
KERNELS="k_lsd_hist k_mtf emit k_duval" bash tools/kab.sh "KOLM_X=0" "KOLM_LSD_HL=0" "KOLM_OVERLAP=1" "KOLM_OVERLAP=2" > $O/ab.txt 2>&1 || exit 1
echo done
