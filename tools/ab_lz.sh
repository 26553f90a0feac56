# A/B of two library builds: LZ-related GPU tests on B, overlapped A/B bench lines, serial LZ kernel times
set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lz77 or adversarial or multiblock or edge or smoke or cdc_vs or variable" > gpurun_out/t_lz.log 2>&1 || { tail -30 gpurun_out/t_lz.log; exit 1; }
tail -1 gpurun_out/t_lz.log
bash tools/ab.sh gpurun_out/ab ab/A.so ab/B.so 3 || exit 1
bash tools/serial_ab.sh || exit 1
