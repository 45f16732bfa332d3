#!/bin/bash
# Warm re-verify: the per-read residency probe (vx_config.direct_io = 1) against
# plain buffered reads (0), engine and read side alone.
set -o pipefail
OUT=gpurun_out/${1:-dio_ab}
mkdir -p $OUT
D=${TMPDIR:-/tmp}
F=$D/vx_dio_$$.bin
dd if=/dev/urandom of=$F bs=1M count=2773 status=none || exit 1
sync $F; cat $F > /dev/null
P=./tools/native/readers_probe
for rep in 1 2; do
  for args in "16 262144 2 4 1 1" "16 262144 2 4 0 1" "16 262144 2 4 1 0" "16 262144 2 4 0 0"; do
    timeout -k 10 120 $P $F 2097152 $args >> $OUT/readers.jsonl 2>> $OUT/readers.err || { rm -f $F; echo FAIL $args; exit 1; }
    tail -1 $OUT/readers.jsonl
  done
done
rm -f $F
timeout -k 10 400 python -u tools/reverify_ab.py --reps 8 --cold-reps 2 \
  --configs "dio1=;dio0=direct_io=0" > $OUT/ab.jsonl 2> $OUT/ab.err || { echo AB_FAIL; tail -5 $OUT/ab.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print(d['config'], d.get('warm'), d.get('cold'), [round(t['read_GiBps_per_thread'] or 0,2) for t in d.get('warm_tr',[])])"
