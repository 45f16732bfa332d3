#!/bin/bash
# Download-loop cost at network-realistic arrival rates (tools/native/paced_probe):
# 256 KiB pieces at 1, 4, 16 and 40 GB/s, plus 2 MiB / 16 KiB at 4 GB/s.
set -o pipefail
OUT=gpurun_out/${1:-paced}
mkdir -p $OUT
for spec in "262144 1" "262144 4" "262144 16" "262144 40" "2097152 4" "16384 4" "262144 60"; do
  set -- $spec
  timeout -k 10 60 ./tools/native/paced_probe $1 $2 1.5 1000 8192 >> $OUT/paced.jsonl 2>> $OUT/paced.err || { echo "FAIL $spec"; tail -5 $OUT/paced.err; exit 1; }
  tail -1 $OUT/paced.jsonl
done
