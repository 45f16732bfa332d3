set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03/zc
OUT=gpurun_out/r03/zc/ab_slots.jsonl; : > $OUT
for rep in 1 2 3; do for slots in 4 6 8; do for zc in 0 1; do
  line=$(VX_ZERO_COPY=$zc timeout -k 10 120 ./tools/native/async_probe 262144 8192 8 64 2 0 $slots) || exit 1
  echo "{\"zc\": $zc, \"slots\": $slots, \"rep\": $rep, \"res\": $line}" >> $OUT
done; done; done
python3 -c "
import json,collections
a=collections.defaultdict(list)
for l in open('$OUT'):
    r=json.loads(l); a[(r['slots'],r['zc'])].append(r['res']['GiBps'])
for k,v in sorted(a.items()): print(k, sorted(v))
"
