# Async gather grid policy A/B (long-piece slots at grid 128): prewide = before,
# ggrid = after; async 16 KiB / 256 KiB / 1 / 2 / 4 MiB, one mmap per buffer.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/ggrid
for rep in 1 2; do
  for v in prewide ggrid; do
    cp tools/ab/libvortex_amd_$v.so vortex_amd/libvortex_amd.so
    for a in "16384 1024 2 512 2" "262144 1024 8 512 2" "1048576 1024 16 512 2" "2097152 1024 16 512 2" "4194304 1024 16 512 2"; do
      echo -n "{\"v\": \"$v\", \"rep\": $rep, \"r\": " >> gpurun_out/ggrid/out.jsonl
      timeout -k 10 120 ./tools/native/async_probe $a | tr -d '\n' >> gpurun_out/ggrid/out.jsonl || exit 1
      echo "}" >> gpurun_out/ggrid/out.jsonl
    done
  done
done
cp tools/ab/libvortex_amd_ggrid.so vortex_amd/libvortex_amd.so
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ggrid/out.jsonl"):
    j = json.loads(l)
    d[(j["r"]["piece_len"], j["v"])].append(j["r"]["GiBps"])
for k in sorted(d):
    print(k, d[k])
PY
