# persistent decode diagnostics: timeline + stage cycles (diagnostics build), then PMC passes (release build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
DIE_C_DIAG=1 timeout -k 10 240 python -u bench/prof_decode_persistent.py 4 0,1,2,4,6 > gpurun_out/dp_diag.log 2>&1 || { tail -20 gpurun_out/dp_diag.log; exit 1; }
grep '^{' gpurun_out/dp_diag.log | grep -v '"layer"' 
timeout -k 10 600 bash scripts/pmc_persistent.sh > gpurun_out/dp_pmc.log 2>&1 || { tail -20 gpurun_out/dp_pmc.log; exit 2; }
cat gpurun_out/pmc/summary.txt
