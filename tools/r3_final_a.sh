# round-3 evidence, part A: the GPU test suite, then the default bench (20 steps)
set -o pipefail
O=gpurun_out/r3e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/bench_default.json'));f=d['detail']['full_candidates']
print('hot', d['value'], d['ms_per_step'], '| full', f['value'], 'MB/s step', f['ms_per_step'], 'repair', f['ms_repair'], 'parity', d['detail']['parity_blocks'], f['parity_blocks'])"
