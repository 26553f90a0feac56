# round 3: factor-start lists instead of the per-position factor record: parity + timing
set -o pipefail
O=gpurun_out/r3g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not adversarial_repair and not repair_full" > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
KERNELS="k_duval k_tile k_fed k_prevc k_keypos k_r0 k_keygen" bash tools/kab.sh "KOLM_X=0" > $O/ab.txt 2>&1 || exit 1
cat $O/ab.txt
