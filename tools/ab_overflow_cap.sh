set -o pipefail
mkdir -p gpurun_out/r06_cap
for rep in 1 2 3; do
 for spec in "262144 8192 2.0" "2097152 1024 2.0" "16384 65536 1.0"; do
  set -- $spec
  for cap in model measured; do
   timeout -k 10 120 tools/native/async_probe $1 $2 $3 64 2 0 4 15 $cap >> gpurun_out/r06_cap/ab.jsonl 2>> gpurun_out/r06_cap/ab.err || exit 1
  done
 done
done
