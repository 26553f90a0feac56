# co-residence diagnosis: k_repair without scratch (RK=1) at a 240- and a 256-block grid
set -o pipefail
O=gpurun_out/fc3
mkdir -p $O
export TMPDIR=/tmp
for cfg in "rk1 62.95" "rk1 70" "rk2 62.95"; do
  set -- $cfg
  KOLM_LIB=$PWD/ab/$1/libkolm_hip.so KOLM_RP_WS_GB=$2 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_$1_$2 -o fc -- python3 bench.py --steps 1 --warmup 1 --kt-steps 0 --no-serial-pass --no-cpu-baseline --full-steps 1 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 > $O/bench_$1_$2.json 2> $O/bench_$1_$2.err || { tail -20 $O/bench_$1_$2.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/bench_$1_$2.json'));f=d['detail']['full_candidates']
print('$1 $2', '| full', f['value'], 'MB/s step', f['ms_per_step'], 'repair', f['ms_repair'], 'parity', f['parity_blocks'])"
done
