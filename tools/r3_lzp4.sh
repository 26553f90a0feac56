set -o pipefail
O=gpurun_out/lzp
mkdir -p $O
for a in "checker" "mixed 0x1ff 1"; do
  KOLM_LZ_PROF=1 KOLM_DUVAL_PROF=1 timeout -k 10 200 python tools/lz_probe.py $a > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
  grep -h "stitch_l\|duval_span us\|k_lz_stitch \|k_duval_merge\|k_mtf" $O/p.log | tail -6 | cut -c1-400
done
