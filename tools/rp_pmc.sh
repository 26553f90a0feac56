#!/bin/bash
OUT=gpurun_out/r02k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o pmc --output-format csv -- python3 tools/rp_trace.py run $OUT 256 enwik > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o pmc --output-format csv -- python3 tools/rp_trace.py run $OUT 256 enwik > $OUT/write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/hit -o pmc --output-format csv -- python3 tools/rp_trace.py run $OUT 256 enwik > $OUT/hit.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch1 -o pmc --output-format csv -- python3 tools/rp_trace.py run $OUT 1 enwik > $OUT/fetch1.log 2>&1 || exit 1
echo done
