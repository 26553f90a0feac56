# round 3: fused first LSD histogram + flat Duval merges: parity, Duval profile, kernel list
set -o pipefail
O=gpurun_out/r3e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_bench_stream.py tests/test_gpu_parity.py tests/test_cdc.py -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
KOLM_DUVAL_PROF=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --kt-steps 1 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --no-serial-pass --host-steps 0 > $O/dprof.json 2> $O/dprof.err || exit 1
KOLM_BENCH_ALLK=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 > $O/bench.json 2> $O/bench.err || exit 1
echo done
