# per-rank compute of TP configurations on one GPU (bench/tp_probe.py): 70B TP=8 (config 4), 8B TP=2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u bench/tp_probe.py --preset llama3-70b --tp 8 --steps 2 --warmup 1 > gpurun_out/tp_probe_70b.log 2>&1 || exit 1
timeout -k 10 300 python -u bench/tp_probe.py --preset llama3-8b --tp 2 --steps 2 --warmup 1 > gpurun_out/tp_probe_8b.log 2>&1 || exit 2
