# round-3 evidence, part B: rocprofv3 kernel stats (overlapped, serialised), PMC passes, and
# the kernel stats of a full-candidate (ids 0..9) step
set -o pipefail
O=gpurun_out/r3p
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_profile.sh $O || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fc -o fc --output-format csv -- python3 bench.py --steps 1 --warmup 1 --kt-steps 0 --no-serial-pass --no-cpu-baseline --full-steps 1 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 > $O/fc.log 2>&1 || { tail -20 $O/fc.log; exit 1; }
echo done
