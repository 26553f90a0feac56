# round 3 evidence: profiles (stats + PMC), then the default bench
set -o pipefail
bash tools/gpu_profile.sh gpurun_out/r3prof || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3prof/bench_default.json 2> gpurun_out/r3prof/bench_default.err || exit 1
echo evidence done
