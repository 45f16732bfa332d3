#!/bin/bash
# Warm re-verify read bound: page-cache pread rate of the
# linux-mint-sized file by read size and order, with and without a competing
# H2D stream: chunk-major 256 KiB reads (today's resumable rounds) against
# whole 2 MiB pieces and 4 MiB coalesced runs (a piece-major stage).
set -o pipefail
OUT=gpurun_out/${1:-pread_sizes}
mkdir -p $OUT
D=${TMPDIR:-/tmp}
F=$D/vx_pread_sizes_$$.bin
dd if=/dev/zero of=$F bs=1M count=2773 status=none || exit 1
cat $F > /dev/null
for rep in 1 2; do
  timeout -k 10 120 ./tools/native/pread_probe $F 8 16 c=262144 p=2097152 >> $OUT/pread.jsonl 2>> $OUT/pread.err || { rm -f $F; exit 1; }
  timeout -k 10 120 ./tools/native/pread_probe $F 8 16 c=2097152 c=4194304 >> $OUT/pread.jsonl 2>> $OUT/pread.err || { rm -f $F; exit 1; }
  timeout -k 10 120 ./tools/native/pread_probe $F 16 c=262144 p=2097152 dma >> $OUT/pread.jsonl 2>> $OUT/pread.err || { rm -f $F; exit 1; }
  timeout -k 10 120 ./tools/native/pread_probe $F 16 c=2097152 c=4194304 dma >> $OUT/pread.jsonl 2>> $OUT/pread.err || { rm -f $F; exit 1; }
done
rm -f $F
cat $OUT/pread.jsonl
