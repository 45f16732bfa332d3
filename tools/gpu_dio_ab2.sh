#!/bin/bash
# After sampling residency once per call: default (direct_io = 1) against plain
# buffered reads (0), warm and cold, alternating.
set -o pipefail
OUT=gpurun_out/${1:-dio_ab2}
mkdir -p $OUT
timeout -k 10 500 python -u tools/reverify_ab.py --reps 10 --cold-reps 3 \
  --configs "${CONFIGS:-dio1=;dio0=direct_io=0}" > $OUT/ab.jsonl 2> $OUT/ab.err || { echo AB_FAIL; tail -5 $OUT/ab.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print(d['config'], d.get('warm'), d.get('cold'), [round(t['read_GiBps_per_thread'] or 0,2) for t in d.get('warm_tr',[])], [t.get('direct_bytes') for t in d.get('cold_tr',[])])"
