# LZ77-related GPU tests, then an A/B of two library builds (serial + overlapped, LZ profile)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lz77 or adversarial or multiblock or edge or smoke or cdc_vs or variable or golden" > gpurun_out/t_lz.log 2>&1 || { tail -30 gpurun_out/t_lz.log; exit 1; }
tail -1 gpurun_out/t_lz.log
bash tools/env_ab.sh "KOLM_SERIAL=1 KOLM_LZ_PROF=1 KOLM_LIB=$1" "KOLM_SERIAL=1 KOLM_LZ_PROF=1 KOLM_LIB=$2" "KOLM_LIB=$1" "KOLM_LIB=$2" || exit 1
grep -h "k_lz_local us" gpurun_out/ab_1.err gpurun_out/ab_2.err | tail -2
