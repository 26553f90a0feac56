# round 3: windowed round-0 RK write: parity tests, A/B, PMC write bytes
set -o pipefail
O=gpurun_out/r3d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_bench_stream.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
KERNELS="k_r0_ k_lsd_scan" bash tools/kab.sh "KOLM_X=0" "KOLM_R0F_WIN=0" > $O/ab.txt 2>&1 || exit 1
ARGS="--mib 256 --steps 1 --warmup 1 --kt-steps 1 --no-serial-pass --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/w0 -o pmc --output-format csv -- python3 bench.py $ARGS > $O/w0.log 2>&1 || exit 1
echo done
