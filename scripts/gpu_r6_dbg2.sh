set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== 8 ranks, window 8, default spin"; timeout -k 5 60 python -u scripts/dbg_tp8.py 8 8 > gpurun_out/dbg_a.log 2>&1; echo "exit $?"; grep -E "^plan|^generate|^sampled|^got 6" gpurun_out/dbg_a.log
echo "== 8 ranks, window 8, parent holds a context"; timeout -k 5 60 python -u scripts/dbg_tp8.py 8 8 parentcuda > gpurun_out/dbg_b.log 2>&1; echo "exit $?"; grep -E "^plan|^generate|^sampled|^got 6" gpurun_out/dbg_b.log
echo "== 8 ranks, window 1, parent holds a context"; timeout -k 5 60 python -u scripts/dbg_tp8.py 8 1 parentcuda > gpurun_out/dbg_c.log 2>&1; echo "exit $?"; grep -E "^plan|^generate|^sampled|^got 6" gpurun_out/dbg_c.log
