# round 3: MTF replay with 64-byte per-thread accesses: parity + timing
set -o pipefail
O=gpurun_out/r3g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_bench_stream.py tests/test_gpu_parity.py tests/test_decode.py -x -q --timeout 300 --timeout-method thread -k "not adversarial_repair and not repair_full" > $O/gpu_tests.log 2>&1 || exit 1
KERNELS="k_mtf emit" bash tools/kab.sh "KOLM_X=0" > $O/ab.txt 2>&1 || exit 1
echo done
