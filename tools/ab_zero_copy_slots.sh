# Slot count against the async path's rate, gather (VX_ZERO_COPY=0) and
# zero-copy (=1) slots alternating: 256 KiB pieces, 8,192 registered mmaps,
# an 8 GiB stream (tools/native/async_probe's 7th argument = slots).
#   /usr/local/graft/bin/gpurun --timeout 600 -- bash tools/ab_zero_copy_slots.sh [tag] ["slots ..."] [piece_len] [GiB]
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03/zc
OUT=gpurun_out/r03/zc/ab_slots_${1:-run}.jsonl; : > $OUT
PL=${3:-262144}; GIB=${4:-8}
for rep in 1 2 3; do for slots in ${2:-4 6 8}; do for zc in 0 1; do
  line=$(VX_ZERO_COPY=$zc timeout -k 10 120 ./tools/native/async_probe $PL 8192 $GIB 64 2 0 $slots) || exit 1
  echo "{\"zc\": $zc, \"slots\": $slots, \"rep\": $rep, \"res\": $line}" >> $OUT
done; done; done
python3 -c "
import json,collections
a=collections.defaultdict(list)
for l in open('$OUT'):
    r=json.loads(l); a[(r['slots'],r['zc'])].append(r['res']['GiBps'])
for k,v in sorted(a.items()): print('slots', k[0], 'zero_copy', k[1], sorted(v))
"
