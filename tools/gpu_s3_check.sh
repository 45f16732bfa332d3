# Default split ring 3 vs 2 (tools/ab/libvortex_amd_s2.so), same box: tests, A/B, e2e paths.
set -o pipefail
O=gpurun_out/s3; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 python tools/ab_builds.py --a tools/ab/libvortex_amd_s2.so --b vortex_amd/libvortex_amd.so --rounds 2 --only 16384x256K_split,8192x2MiB_split,ragged_config3_config5 > $O/ab.json 2> $O/ab.err || exit 1
cat $O/ab.json
for lib in tools/ab/libvortex_amd_s2.so vortex_amd/libvortex_amd.so; do
  echo "== $lib"
  VX_LIB_OVERRIDE=$PWD/$lib timeout -k 10 200 python tools/e2e_perbuf.py --chunks 65536 --reps 2 || exit 1
  VX_LIB_OVERRIDE=$PWD/$lib timeout -k 10 300 python tools/reverify_bench.py --reps 2 --slots 3 --slot-mib 1024 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('reverify', d['best'])" || exit 1
done
