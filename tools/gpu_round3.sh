set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -k "verify_files or async or host_batches or seeding" > gpurun_out/pytest_files.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_files.log; exit 1; }
tail -2 gpurun_out/pytest_files.log
for cfg in "4 256" "4 512" "3 1024" "2 1536"; do set -- $cfg
timeout -k 10 300 python tools/reverify_bench.py --reps 2 --slots $1 --slot-mib $2 > gpurun_out/reverify_$1_$2.json 2> gpurun_out/reverify.err || { echo REVERIFY_FAIL; tail -20 gpurun_out/reverify.err; exit 1; }
echo "slots=$1 mib=$2"; cat gpurun_out/reverify_$1_$2.json
done
