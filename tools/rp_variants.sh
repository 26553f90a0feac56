#!/bin/bash
# Build A/B variants of libkolm_hip.so that differ only in k_repair.hip's compile flags:
#   bash tools/rp_variants.sh name "-DKOLM_RP_VGPR=96" [name2 "flags2" ...]  -> ab/<name>/libkolm_hip.so
set -e
cd "$(dirname "$0")/../kolmogorovlike-datacompressor_amd"
make -j8 >/dev/null
while [ $# -ge 2 ]; do
  d=../ab/$1; mkdir -p $d
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics \
    -ffp-contract=fast $2 -x hip -c csrc/k_repair.hip -o $d/k_repair.hip.o
  objs=$(ls build/*.o | grep -v k_repair.hip.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/libkolm_hip.so $objs $d/k_repair.hip.o
  echo "built $d"
  shift 2
done
