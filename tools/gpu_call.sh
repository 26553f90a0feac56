#!/bin/bash
# One parameterised GPU call (run through gpurun from the repo root):
#   bash tools/gpu_call.sh OUT STEP [STEP ...]
# STEPs, run in order, each under its own time limit, stopping at the first failure:
#   tests            pytest -m gpu (whole suite)
#   tests:EXPR       pytest -m gpu -k EXPR
#   bench            bench.py --steps 20 --warmup 5 (the driver's headline run)
#   quick            bench.py hot path only, 5 steps
#   smoke            __graft_entry__.smoke()
#   profile          tools/gpu_profile.sh OUT/prof (rocprofv3 stats overlapped + serialised + PMC)
#   profile_full     the same on the ids 0..9 step (Re-Pair included)
# Results land under OUT (default gpurun_out/call); the summary lines go to stdout.
set -o pipefail
OUT=${1:-gpurun_out/call}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
QUICK="--steps 5 --warmup 2 --no-cpu-baseline --full-steps 0 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 --c4-steps 0 --no-serial-pass"
summ() {
  python3 -c "
import json,sys;d=json.load(open('$1'));t=d['detail']
print('value', d['value'], 'ms', d['ms_per_step'], 'parity', t['parity_blocks'], 'frac', d['roofline']['frac'])
for k in ('full_candidates','config4_shard','host_e2e'):
    v=t.get(k)
    if v: print(' ', k, v.get('value'), v.get('ms_per_step', v.get('ms_per_call')), v.get('parity_blocks'))
fam=t.get('families_ms_per_step');print('  families', fam)"
}
for step in "$@"; do
  case "$step" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 \
        || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
      tail -2 "$OUT/gpu_tests.log" ;;
    tests:*)
      # tests:EXPR with '+' for ' or ' (e.g. tests:rccl+gpu_dist)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        -k "$(echo "${step#tests:}" | sed 's/+/ or /g')" > "$OUT/gpu_tests_k.log" 2>&1 || { tail -40 "$OUT/gpu_tests_k.log"; exit 1; }
      tail -3 "$OUT/gpu_tests_k.log" ;;
    bench)
      timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" \
        || { tail -30 "$OUT/bench.err"; exit 1; }
      summ "$OUT/bench.json" ;;
    quick)
      timeout -k 10 300 python bench.py $QUICK > "$OUT/quick.json" 2> "$OUT/quick.err" || { tail -30 "$OUT/quick.err"; exit 1; }
      summ "$OUT/quick.json" ;;
    ab:*)
      # ab:VAR=v+VAR2=w  the hot-path quick bench under those environment settings
      envs=$(echo "${step#ab:}" | tr '+' ' ')
      tag=$(echo "${step#ab:}" | tr -c 'A-Za-z0-9=_\n' '_')
      env $envs KOLM_BENCH_ALLK=1 timeout -k 10 300 python bench.py $QUICK > "$OUT/ab_$tag.json" 2> "$OUT/ab_$tag.err" \
        || { tail -30 "$OUT/ab_$tag.err"; exit 1; }
      echo "[$envs]"; summ "$OUT/ab_$tag.json" ;;
    run:*)
      # run:TAG:VAR=v+VAR2=w:bench args (spaces as commas) — bench.py with those settings
      IFS=: read -r _ tag envs args <<< "$step"
      env $(echo "$envs" | tr '+' ' ') KOLM_BENCH_ALLK=1 timeout -k 10 300 python bench.py $(echo "$args" | tr ',' ' ') \
        > "$OUT/run_$tag.json" 2> "$OUT/run_$tag.err" || { tail -30 "$OUT/run_$tag.err"; exit 1; }
      python3 -c "
import json;d=json.load(open('$OUT/run_$tag.json'));t=d['detail']
print('[$tag]', d['value'], d['ms_per_step'], t['parity_blocks'], 'dev', t.get('device_ms'))
k=t.get('kernels_all_ms_per_step') or {}
print('  top', dict(sorted(k.items(), key=lambda kv: -kv[1])[:18]))
for kk in ('config4_shard', 'config4', 'host_e2e'):
    v=t.get(kk)
    if v: print('  ', kk, v.get('value'), v.get('ms_per_step', v.get('ms_per_call')), v.get('parity_blocks'), v.get('device_ms_of_call'))
c=t.get('configs')
if c:
    for n,v in c.items(): print('  ', n, {kk: (vv.get('value'), vv.get('ms_per_call'), vv.get('ms_sa'), vv.get('ms_lz'), vv.get('parity_blocks')) for kk,vv in v.items() if isinstance(vv, dict)})"
      ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || { tail -30 "$OUT/smoke.log"; exit 1; }
      tail -4 "$OUT/smoke.log" ;;
    profile)
      bash tools/gpu_profile.sh "$OUT/prof" || exit 1 ;;
    profile_full)
      bash tools/gpu_profile.sh "$OUT/prof_full" "--mib 256 --steps 1 --warmup 1 --kt-steps 1 --no-serial-pass --no-cpu-baseline --full-steps 1 --decode-steps 0 --cdc-steps 0 --v2-steps 0 --config-steps 0 --host-steps 0 --c4-steps 0" stats || exit 1 ;;
    probe:*)
      # probe:KIND — rocprofv3 kernel trace of tools/lz_probe.py KIND (4 batches, the last kernel-timed)
      kind=${step#probe:}
      PROBE_ITERS=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/probe_$kind" -o kt --output-format csv \
        -- python3 tools/lz_probe.py "$kind" > "$OUT/probe_$kind.log" 2>&1 || { tail -30 "$OUT/probe_$kind.log"; exit 1; }
      KOLM_DEBUG_ROUNDS=1 KOLM_HOST_PROF=1 PROBE_ITERS=3 timeout -k 10 300 python3 tools/lz_probe.py "$kind" \
        > "$OUT/probe_${kind}_rounds.log" 2>&1 || { tail -30 "$OUT/probe_${kind}_rounds.log"; exit 1; }
      head -3 "$OUT/probe_$kind.log" | cut -c1-400 ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
