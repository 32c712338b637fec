# prefill GEMM table: tune the one-GPU o / down projections as they now run (resid += x @ w^T, beta = 1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u bench/micro_prefill_tunableop.py --residual --models 8b --out gpurun_out/tunableop_resid.csv > gpurun_out/tune_resid.log 2>&1 || { tail -10 gpurun_out/tune_resid.log; exit 1; }
grep '"bench"' gpurun_out/tune_resid.log
grep -v Validator gpurun_out/tunableop_resid.csv
