# Re-Pair: per-block time vs concurrently resident blocks (workspace budget -> group size)
set -o pipefail
O=gpurun_out/rps
mkdir -p $O
timeout -k 10 200 python tools/rp_trace.py run $O 1 enwik > $O/x1.log 2>&1 || { tail -20 $O/x1.log; exit 1; }
head -3 $O/x1.log
for gb in 70 34 17 8.5 4.3; do
  KOLM_RP_WS_GB=$gb timeout -k 10 200 python tools/rp_trace.py run $O 256 enwik > $O/ws_$gb.log 2>&1 || { tail -20 $O/ws_$gb.log; exit 1; }
  echo "ws $gb GB: $(head -1 $O/ws_$gb.log)"; sed -n 3p $O/ws_$gb.log
done
