# parity tests of the BBWT path, then an A/B of environment settings (tools/env_ab.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_r0.log 2>&1 || { tail -30 gpurun_out/t_r0.log; exit 1; }
tail -1 gpurun_out/t_r0.log
bash tools/env_ab.sh "$@"
