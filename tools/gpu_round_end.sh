#!/bin/bash
# Round-end check on HEAD: the full GPU suite, smoke(), the default bench line,
# then the 8-rank config-4 rehearsal with the full-size multi-GPU re-verify.
set -o pipefail
bash tools/gpu_check_all.sh ${1:-round_end} || exit 1
bash tools/gpu_config4_rehearsal.sh ${1:-round_end}_config4
