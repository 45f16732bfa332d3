# Soaks of the current build against the oracle / hashlib, one after another,
# each under its own time limit.  Writes gpurun_out/${OUT:-soak}/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-soak}
cd $R && mkdir -p $O
S=${SECS:-60}
B=${SEED0:-41}
timeout -k 10 $((S + 90)) python -u tools/soak_async.py --seconds $S --seed $B > $O/async_seed$B.json 2> $O/async.err || { echo ASYNC_FAIL; tail -20 $O/async.err; exit 1; }
tail -c 600 $O/async_seed$B.json; echo
timeout -k 10 $((S + 90)) python -u tools/soak_async.py --seconds $S --seed $((B + 1)) --faults > $O/async_faults_seed$((B + 1)).json 2> $O/async_faults.err || { echo FAULTS_FAIL; tail -20 $O/async_faults.err; exit 1; }
tail -c 600 $O/async_faults_seed$((B + 1)).json; echo
timeout -k 10 $((S + 90)) python -u tools/soak_batches.py --seconds $S --seed $((B + 2)) > $O/batches_seed$((B + 2)).json 2> $O/batches.err || { echo BATCH_FAIL; tail -20 $O/batches.err; exit 1; }
tail -c 600 $O/batches_seed$((B + 2)).json; echo
mkdir -p /var/tmp/vx_soak_$$
timeout -k 10 $((S + 90)) python -u tools/soak_files.py --seconds $S --seed $((B + 3)) --dir /var/tmp/vx_soak_$$ > $O/files_seed$((B + 3)).json 2> $O/files.err || { echo FILES_FAIL; tail -20 $O/files.err; rm -rf /var/tmp/vx_soak_$$; exit 1; }
rm -rf /var/tmp/vx_soak_$$
tail -c 600 $O/files_seed$((B + 3)).json; echo
mkdir -p /var/tmp/vx_soakc_$$
timeout -k 10 $((S + 90)) python -u tools/soak_files.py --seconds $S --seed $((B + 4)) --cold --dir /var/tmp/vx_soakc_$$ > $O/files_cold_seed$((B + 4)).json 2> $O/files_cold.err || { echo COLD_FAIL; tail -20 $O/files_cold.err; rm -rf /var/tmp/vx_soakc_$$; exit 1; }
rm -rf /var/tmp/vx_soakc_$$
tail -c 600 $O/files_cold_seed$((B + 4)).json; echo
