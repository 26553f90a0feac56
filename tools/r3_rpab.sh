# Re-Pair A/B of k_repair builds (ab/<name>/libkolm_hip.so): 256 blocks alone, block spread
set -o pipefail
O=gpurun_out/rpab
mkdir -p $O
for v in base mc15 mc1 mc3 rk2 base; do
  if [ $v = base ]; then unset KOLM_LIB; else export KOLM_LIB=$PWD/ab/$v/libkolm_hip.so; fi
  KOLM_RP_PROF=1 timeout -k 10 200 python tools/rp_trace.py run $O 256 enwik > $O/x256_$v.log 2>&1 || { tail -20 $O/x256_$v.log; exit 1; }
  echo "$v: $(grep -h 'ms_repair' $O/x256_$v.log) $(grep -ho 'block total.*' $O/x256_$v.log)"
done
