#!/bin/bash
# Cold re-verify with unprobed O_DIRECT for uncached files: the read side alone
# (evicted before every rep, with a copy chain) and the engine, direct_io 1 vs 0.
set -o pipefail
OUT=gpurun_out/${1:-cold_ab}
mkdir -p $OUT
D=/var/tmp
F=$D/vx_cold_$$.bin
dd if=/dev/urandom of=$F bs=1M count=2773 status=none || exit 1
sync $F
P=./tools/native/readers_probe
for rep in 1 2; do
  for args in "16 262144 2 4 1 1 2 1" "16 262144 2 4 0 1 2 1" "8 262144 2 4 1 1 2 1" "16 1048576 2 4 1 1 2 1"; do
    timeout -k 10 120 $P $F 2097152 $args >> $OUT/readers.jsonl 2>> $OUT/readers.err || { rm -f $F; echo FAIL $args; exit 1; }
    tail -1 $OUT/readers.jsonl
  done
done
rm -f $F
timeout -k 10 500 python -u tools/reverify_ab.py --reps 4 --cold-reps 5 \
  --configs "dio1=;dio0=direct_io=0;dio1c1m=verify_cold_chunk=1048576" > $OUT/ab.jsonl 2> $OUT/ab.err || { echo AB_FAIL; tail -5 $OUT/ab.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print(d['config'], d.get('warm'), d.get('cold'), [round(t['read_GiBps_per_thread'] or 0,2) for t in d.get('cold_tr',[])])"
