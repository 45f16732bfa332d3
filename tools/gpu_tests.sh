#!/bin/bash
# The GPU test suite on the box, one pytest process, output under gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-gputest}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${@:2} \
    > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -5 $OUT/pytest_gpu.log
echo "pytest rc=$rc"
exit $rc
