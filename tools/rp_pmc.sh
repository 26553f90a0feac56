#!/bin/bash
OUT=${1:-gpurun_out/rpk}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o pmc --output-format csv -- python3 tools/rp_trace.py run $OUT 256 enwik > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o pmc --output-format csv -- python3 tools/rp_trace.py run $OUT 256 enwik > $OUT/write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/hit -o pmc --output-format csv -- python3 tools/rp_trace.py run $OUT 256 enwik > $OUT/hit.log 2>&1 || exit 1
echo done
