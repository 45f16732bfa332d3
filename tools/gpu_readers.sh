#!/bin/bash
# Where the warm re-verify's reads bind: the read side alone
# (tools/native/readers_probe: vx_files::Readers in the resumable rounds, pinned
# stages, with and without the residency probe and a concurrent copy chain), then
# the engine itself at several reader counts (tools/reverify_ab.py).
set -o pipefail
OUT=gpurun_out/${1:-readers}
mkdir -p $OUT
D=${TMPDIR:-/tmp}
F=$D/vx_readers_$$.bin
dd if=/dev/urandom of=$F bs=1M count=2773 status=none || exit 1
sync $F; cat $F > /dev/null
P=./tools/native/readers_probe
for args in "16 262144 2 4 1 0" "16 262144 2 4 0 0" "16 262144 2 4 1 1" "12 262144 2 4 1 1" "8 262144 2 4 1 1" \
            "24 262144 2 4 1 1" "16 2097152 2 4 1 1" "16 262144 3 5 1 1"; do
  timeout -k 10 120 $P $F 2097152 $args >> $OUT/readers.jsonl 2>> $OUT/readers.err || { rm -f $F; echo FAIL $args; exit 1; }
  tail -1 $OUT/readers.jsonl
done
rm -f $F
timeout -k 10 400 python -u tools/reverify_ab.py --reps 4 --cold-reps 1 \
  --configs "t16=;t12=IO_THREADS=12;t8=IO_THREADS=8;t24=IO_THREADS=24;s6=SLOTS=6;s3=SLOTS=3" > $OUT/ab.jsonl 2> $OUT/ab.err || { echo AB_FAIL; tail -5 $OUT/ab.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print(d['config'], d.get('warm'), d.get('cold'), [round(t['read_GiBps_per_thread'] or 0,2) for t in d.get('warm_tr',[])])"
