# A/B: the lane kernel's schedule xor as VOP3 v_bitop3 (default build) vs VOP2
# v_xor_b32_e32 (-DVX_XOR2_VOP2), at 1, 2 and 4 waves per SIMD; alternating
# processes on one box.  Libraries are built beforehand under tools/ab/.
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for lib in base xorvop2; do
    for shape in "65536 262144" "131072 131072" "262144 65536"; do
      set -- $shape
      VX_LIB_OVERRIDE=tools/ab/libvortex_amd_$lib.so timeout -k 10 120 python tools/ab_uniform.py --variants 0 --pieces $1 --piece-len $2 --rounds 3 > gpurun_out/abx.json 2>/dev/null || exit 1
      python -c "import json; d=json.load(open('gpurun_out/abx.json')); print('$r', '$lib', $1, $2, d['results']['0']['median_ms'])"
    done
  done
done
