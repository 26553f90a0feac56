# Re-Pair: per-block time vs number of concurrently resident blocks (workspace budget)
set -o pipefail
O=gpurun_out/rp1
mkdir -p $O
for gb in 70 34 17 8.5; do
  KOLM_RP_WS_GB=$gb timeout -k 10 200 python tools/rp_trace.py run $O 256 enwik > $O/ws_$gb.log 2>&1 || { tail -20 $O/ws_$gb.log; exit 1; }
  echo "ws $gb GB: $(head -1 $O/ws_$gb.log)"
done
