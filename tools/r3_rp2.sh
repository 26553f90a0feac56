# Re-Pair A/B of k_repair builds (ab/<name>/libkolm_hip.so): alone (256 blocks) and in the
# full-candidate bench step beside the hot path
set -o pipefail
O=gpurun_out/rp2
mkdir -p $O
for v in base v96 v80 n512; do
  if [ $v = base ]; then unset KOLM_LIB; else export KOLM_LIB=$PWD/ab/$v/libkolm_hip.so; fi
  timeout -k 10 200 python tools/rp_trace.py run $O 256 enwik > $O/alone_$v.log 2>&1 || { tail -20 $O/alone_$v.log; exit 1; }
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --kt-steps 0 --no-serial-pass --no-cpu-baseline --full-steps 2 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/bench_$v.json'));f=d['detail']['full_candidates']
print('$v', open('$O/alone_$v.log').readline().strip(), '| full', f['value'], 'MB/s step', f['ms_per_step'], 'repair', f['ms_repair'], 'parity', f['parity_blocks'])"
done
