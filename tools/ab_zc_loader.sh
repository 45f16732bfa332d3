# Zero-copy pair (VX_ZC_LOADER=0) against the three-wave form with a loader
# wave (=1) on the async path, alternating: one JSON line per run.
#   bash tools/ab_zc_loader.sh REPS "piece_len:nbuf:GiB ..."
set -o pipefail
reps=${1:-3}
for rep in $(seq 1 $reps); do
  for spec in $2; do
    IFS=: read pl nbuf gib <<< "$spec"
    for L in 0 1; do
      line=$(VX_ZC_LOADER=$L VX_ZERO_COPY=1 timeout -k 10 120 ./tools/native/async_probe $pl $nbuf $gib 64 2) || { echo "FAIL pl=$pl L=$L"; exit 1; }
      echo "{\"loader\": $L, \"rep\": $rep, \"res\": $line}"
    done
  done
done
