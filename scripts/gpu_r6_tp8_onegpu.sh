# the 8-rank TP engine on one GPU, token-exact against TP=1, on the final tree (few-pair attention split)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/tp_ranks_one_gpu.py --world 8 > gpurun_out/tp8one.log 2>&1 || { echo "FAILED"; tail -20 gpurun_out/tp8one.log; exit 1; }
grep '^{' gpurun_out/tp8one.log | cut -c1-600
timeout -k 10 300 python -u scripts/tp_ranks_one_gpu.py --world 4 > gpurun_out/tp4one.log 2>&1 || { echo "FAILED"; tail -20 gpurun_out/tp4one.log; exit 2; }
grep '^{' gpurun_out/tp4one.log | cut -c1-600
