#!/bin/bash
# Warm re-verify with 12 / 16 / 24 / 32 reader threads, alternating (the box's
# CPU share is 16): does the read side scale past the share?
set -o pipefail
OUT=gpurun_out/${1:-reader_count}
mkdir -p $OUT
timeout -k 10 400 python -u tools/reverify_ab.py --reps 8 --cold-reps 0 --no-cpu \
  --configs "t16=IO_THREADS=16;t12=IO_THREADS=12;t24=IO_THREADS=24;t32=IO_THREADS=32" > $OUT/ab.jsonl 2> $OUT/ab.err \
  || { echo AB_FAIL; tail -5 $OUT/ab.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); w=d.get('warm') or []
    tr=d.get('warm_tr') or []
    busy=[round(t['read_busy_ms']/(t['readers']*t['read_span_ms']),2) for t in tr if t.get('readers') and t.get('read_span_ms')]
    print(d['config'], sorted(w)[len(w)//2] if w else None, w, 'busy', busy, 'copy_busy', [round(t['copy_busy_frac'],2) for t in tr])"
