#!/bin/bash
# overlapped and serialised (KOLM_SERIAL=1) kernel traces of the bench step
OUT=${1:-gpurun_out/ktb}
bash tools/kt_profile.sh $OUT/ovl || exit 1
KOLM_SERIAL=1 bash tools/kt_profile.sh $OUT/ser || exit 1
