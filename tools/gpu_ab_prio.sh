set -o pipefail
mkdir -p gpurun_out/prio
for lib in tools/ab/libvortex_amd_noprio.so vortex_amd/libvortex_amd.so tools/ab/libvortex_amd_noprio.so vortex_amd/libvortex_amd.so; do
  echo "== $lib"
  VX_LIB_OVERRIDE=$PWD/$lib timeout -k 10 200 python tools/e2e_perbuf.py --chunks 65536 --reps 2 || exit 1
done
timeout -k 10 900 python tools/ab_builds.py --a tools/ab/libvortex_amd_noprio.so --b vortex_amd/libvortex_amd.so --rounds 2 --only 16384x256K_split,8192x2MiB_split,ragged_config3_config5 > gpurun_out/prio/ab.json 2> gpurun_out/prio/ab.err && cat gpurun_out/prio/ab.json
