set -o pipefail
O=gpurun_out/lzp
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_stream.py -x -q --timeout 300 --timeout-method thread -m gpu -k "lz or mixed or config or stream" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 200 python tools/lz_probe.py mixed > $O/mixed.log 2>&1 || { tail -20 $O/mixed.log; exit 1; }
grep "mixed stats" $O/mixed.log | cut -c1-400
true <<'PY'
import ast,re
s=open('gpurun_out/lzp/mixed.log').read().splitlines()[-1]
d=ast.literal_eval(s)
for k,v in sorted(d.items(), key=lambda kv:-kv[1]['ms'])[:12]: print(f"{k:32s} {v['ms']:8.3f} {v['launches']}")
PY
