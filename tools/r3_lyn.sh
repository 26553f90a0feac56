# Lyndon change: parity (GPU parity suite + the 256-block bench stream, hot path) and phase profile
set -o pipefail
O=gpurun_out/lyn
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_stream.py -x -q --timeout 300 --timeout-method thread -m gpu -k "not full_candidates" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
bash tools/r3_dprof.sh
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --kt-steps 1 --no-serial-pass --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/b.json'));k=d['detail']['sort_stream_kernels_ms_per_step']
print('hot', d['value'], d['ms_per_step'], 'duval_span', k.get('k_duval_span'), 'merge', k.get('k_duval_merge'), 'parity', d['detail']['parity_blocks'])"
