set -o pipefail
O=gpurun_out/lzp
mkdir -p $O
for a in "mixed 0x1ff 0" "mixed 0x1ff 1" "mixed 0x1ff 2" "wav" "checker"; do
  timeout -k 10 200 python tools/lz_probe.py $a > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
  grep -v amdgpu.ids $O/p.log | cut -c1-600
done
