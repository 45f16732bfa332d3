# Async download-path throughput sweep (tools/native/async_probe.cpp).
#   /usr/local/graft/bin/gpurun --timeout 600 -- bash tools/gpu_async_probe.sh [tag]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/async
OUT=gpurun_out/async/sweep_${1:-run}.jsonl
: > $OUT
for pl in 16384 262144 2097152 4194304; do
  for fe in 64 512; do
    for reg in 2 1 0; do
      gib=4; [ $pl -eq 16384 ] && gib=1
      timeout -k 10 120 ./tools/native/async_probe $pl 1024 $gib $fe $reg >> $OUT || { echo "FAIL pl=$pl fe=$fe reg=$reg"; exit 1; }
    done
  done
done
cat $OUT
