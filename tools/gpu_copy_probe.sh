#!/bin/bash
# The warm re-verify's page-cache copy three ways under the H2D chain
# (tools/native/copy_probe.hip): pread / mmap+memcpy / mmap+streaming stores,
# alternating, with and without the DMA.
set -o pipefail
OUT=gpurun_out/${1:-copy_probe}
mkdir -p $OUT
D=${TMPDIR:-/var/tmp}
[ -w /var/tmp ] && D=/var/tmp
F=$D/vx_copy_probe_$$.bin
trap 'rm -f $F' EXIT
timeout -k 10 120 python3 -c "
import os, numpy as np
rng = np.random.default_rng(5)
with open('$F', 'wb') as f:
    left = 2907832320
    while left:
        k = min(left, 64 << 20)
        f.write(rng.integers(0, 256, k, dtype=np.uint8).tobytes())
        left -= k
    f.flush(); os.fsync(f.fileno())
" || { echo WRITE_FAIL; exit 1; }
cat $F > /dev/null
for rep in 1 2 3; do
  for dma in 1 0; do
    for mode in 0 1 2; do
      timeout -k 10 120 tools/native/copy_probe $F 2097152 $mode 16 262144 $dma 3 >> $OUT/copy.jsonl 2>> $OUT/copy.err \
        || { echo PROBE_FAIL mode=$mode dma=$dma; tail -5 $OUT/copy.err; exit 1; }
    done
  done
  tail -6 $OUT/copy.jsonl
done
for mode in 1 2; do
  timeout -k 10 120 tools/native/copy_probe $F 2097152 $mode 16 262144 1 3 1 >> $OUT/copy.jsonl 2>> $OUT/copy.err \
    || { echo PROBE_FAIL populate mode=$mode; exit 1; }
done
tail -2 $OUT/copy.jsonl
