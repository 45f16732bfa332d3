# Gather grid A/B across the paths that use the gather kernel:
# async 16 KiB / 256 KiB / 2 MiB pieces in per-buffer registered mmaps, and
# per-buffer sync batches (chunked gather) of 256 KiB / 2 MiB, alternating
# grids twice.  Writes gpurun_out/gather_grid/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gather_grid
mkdir -p $O && cd $R
for rep in 1 2; do
  for g in 64 128; do
    export VX_GATHER_GRID=$g
    for a in "16384 1024 2 512 2" "262144 1024 8 512 2" "2097152 1024 16 512 2"; do
      echo -n "{\"grid\": $g, \"rep\": $rep, \"async\": " >> $O/async.jsonl
      timeout -k 10 120 ./tools/native/async_probe $a >> $O/async.jsonl || exit 1
      sed -i '$ s/$/}/' $O/async.jsonl
    done
    for pl in 262144 2097152; do
      n=$((2147483648 / pl))
      echo -n "{\"grid\": $g, \"rep\": $rep, \"perbuf\": " >> $O/perbuf.jsonl
      timeout -k 10 120 python3 tools/e2e_perbuf.py --pieces $n --piece-len $pl --chunks 65536 --reps 3 >> $O/perbuf.jsonl 2>/dev/null || exit 1
      sed -i '$ s/$/}/' $O/perbuf.jsonl
    done
  done
done
cat $O/async.jsonl $O/perbuf.jsonl
