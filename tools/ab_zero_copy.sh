# A/B of the zero-copy slot kernel on the async download path:
# tools/native/async_probe with VX_ZERO_COPY=0 (gather kernel + hash) and =1
# (the hash kernel reads the registered pieces itself), alternating per rep,
# one registered mmap per pool buffer (vortex's BufferPool), flush every 64.
# ZC_VALUES="0 2" compares the gather against the default policy instead;
# REG=1 puts every buffer in one registered mmap (async_probe registered=1).
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash tools/ab_zero_copy.sh [tag] [reps] ["piece_len:nbuf:GiB ..."]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/r03/zc
OUT=gpurun_out/r03/zc/ab_${1:-run}.jsonl
: > $OUT
REPS=${2:-3}
# piece_len nbuf total_GiB
CASES=${3:-"262144:8192:2 262144:8192:8 16384:8192:1 1048576:2048:4 2097152:1024:4 4194304:512:4"}
for rep in $(seq 1 $REPS); do
  for c in $CASES; do
    IFS=: read pl nbuf gib <<< "$c"
    for zc in ${ZC_VALUES:-0 1}; do
      line=$(VX_ZERO_COPY=$zc timeout -k 10 120 ./tools/native/async_probe $pl $nbuf $gib 64 ${REG:-2}) || { echo "FAIL pl=$pl zc=$zc"; exit 1; }
      echo "{\"zc\": $zc, \"rep\": $rep, \"piece_len\": $pl, \"GiB\": $gib, \"res\": $line}" >> $OUT
    done
  done
done
python3 - "$OUT" <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
agg = collections.defaultdict(list)
for r in rows:
    assert r["res"].get("mismatched", 0) == 0, r
    agg[(r["piece_len"], r["GiB"], r["zc"])].append(r["res"]["GiBps"])
for (pl, gib, zc), v in sorted(agg.items()):
    v = sorted(v)
    print(f"piece {pl // 1024:>5} KiB  {gib:>3} GiB  zero_copy={zc}: median {v[len(v) // 2]:6.2f}  runs {v}")
PY
