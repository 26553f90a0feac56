# Re-Pair restructure: parity (repair GPU tests + the 256-block full-candidate stream) and timing
set -o pipefail
O=gpurun_out/rpn
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_stream.py tests/test_decode.py -x -q --timeout 300 --timeout-method thread -m gpu -k "repair or full" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 200 python tools/rp_trace.py run $O 1 enwik > $O/x1.log 2>&1 || { tail -20 $O/x1.log; exit 1; }
head -3 $O/x1.log
timeout -k 10 200 python tools/rp_trace.py run $O 256 enwik > $O/x256.log 2>&1 || { tail -20 $O/x256.log; exit 1; }
head -3 $O/x256.log
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --kt-steps 0 --no-serial-pass --no-cpu-baseline --full-steps 2 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/bench.json'));f=d['detail']['full_candidates']
print('hot', d['value'], '| full', f['value'], 'MB/s step', f['ms_per_step'], 'repair', f['ms_repair'], 'parity', f['parity_blocks'])"
