# Soaks of the current build against the oracle / hashlib, one after another,
# each under its own time limit.  Writes gpurun_out/${OUT:-soak}/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-soak}
cd $R && mkdir -p $O
S=${SECS:-60}
timeout -k 10 $((S + 90)) python -u tools/soak_async.py --seconds $S --seed 41 > $O/async_seed41.json 2> $O/async.err || { echo ASYNC_FAIL; tail -20 $O/async.err; exit 1; }
tail -c 600 $O/async_seed41.json; echo
timeout -k 10 $((S + 90)) python -u tools/soak_async.py --seconds $S --seed 42 --faults > $O/async_faults_seed42.json 2> $O/async_faults.err || { echo FAULTS_FAIL; tail -20 $O/async_faults.err; exit 1; }
tail -c 600 $O/async_faults_seed42.json; echo
timeout -k 10 $((S + 90)) python -u tools/soak_batches.py --seconds $S --seed 43 > $O/batches_seed43.json 2> $O/batches.err || { echo BATCH_FAIL; tail -20 $O/batches.err; exit 1; }
tail -c 600 $O/batches_seed43.json; echo
mkdir -p /var/tmp/vx_soak_$$
timeout -k 10 $((S + 90)) python -u tools/soak_files.py --seconds $S --seed 44 --dir /var/tmp/vx_soak_$$ > $O/files_seed44.json 2> $O/files.err || { echo FILES_FAIL; tail -20 $O/files.err; rm -rf /var/tmp/vx_soak_$$; exit 1; }
rm -rf /var/tmp/vx_soak_$$
tail -c 600 $O/files_seed44.json; echo
