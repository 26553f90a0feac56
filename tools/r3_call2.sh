# round 3: flat Duval chunk pass + binned round-0 RK write: GPU tests, Duval profile, A/B
set -o pipefail
O=gpurun_out/r3c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
KOLM_DUVAL_PROF=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --kt-steps 1 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --no-serial-pass --host-steps 0 > $O/dprof.json 2> $O/dprof.err || exit 1
KERNELS="k_r0_ k_duval" bash tools/kab.sh "KOLM_X=0" "KOLM_R0F_BIN=0" > $O/ab.txt 2>&1 || exit 1
ARGS="--mib 256 --steps 1 --warmup 1 --kt-steps 1 --no-serial-pass --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/w0 -o pmc --output-format csv -- python3 bench.py $ARGS > $O/w0.log 2>&1 || exit 1
echo done
