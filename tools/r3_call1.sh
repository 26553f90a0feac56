# round 3, GPU call 2: compress_fixed correctness, host-buffer leg, Duval phase profile,
# k_r0_final / round-0 width A/B, PMC write bytes of k_r0_final with and without NT loads
set -o pipefail
O=gpurun_out/r3b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_decode.py -x -q --timeout 200 --timeout-method thread -k "container or edge or golden_containers" > $O/tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --no-serial-pass --host-steps 3 > $O/host.json 2> $O/host.err || exit 1
KOLM_DUVAL_PROF=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --kt-steps 1 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --no-serial-pass --host-steps 0 > $O/dprof.json 2> $O/dprof.err || exit 1
KERNELS="k_r0_final k_r0_tile k_lsd_scatter<3" bash tools/kab.sh "KOLM_X=0" "KOLM_R0F_NT=1" "KOLM_R0F_NT=1 KOLM_R0F_PARTS=4" "KOLM_R0_CMAX=9" "KOLM_R0_CMAX=8" > $O/ab.txt 2>&1 || exit 1
ARGS="--mib 256 --steps 1 --warmup 1 --kt-steps 1 --no-serial-pass --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/w0 -o pmc --output-format csv -- python3 bench.py $ARGS > $O/w0.log 2>&1 || exit 1
KOLM_R0F_NT=1 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/w1 -o pmc --output-format csv -- python3 bench.py $ARGS > $O/w1.log 2>&1 || exit 1
echo done
