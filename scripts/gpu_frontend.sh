# BASELINE config 1 (mock echo model, 2 workers, CPU only) on the GPU box's CPU share: the coordinator
# in its own process, single and multi-process (SO_REUSEPORT) coordinators; the client-side-LB direct rows
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench/serve_bench.py --mode mock --workers 2 --concurrency 1,64,256 --requests 4000 --coord-procs 1 > gpurun_out/fe.jsonl 2>&1 || exit 1
timeout -k 10 300 python bench/serve_bench.py --mode mock --workers 2 --concurrency 64,256 --requests 8000 --coord-procs 4 --client-procs 4 >> gpurun_out/fe.jsonl 2>&1 || exit 2
timeout -k 10 300 python bench/serve_bench.py --mode mock --workers 2 --concurrency 1,64,256 --requests 4000 >> gpurun_out/fe.jsonl 2>&1 || exit 3
timeout -k 10 300 python bench/serve_bench.py --mode mock --workers 2 --concurrency 1,64 --requests 4000 --direct >> gpurun_out/fe.jsonl 2>&1 || exit 4
grep '^{' gpurun_out/fe.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['topology'], 'coord', d.get('coordinator_procs'), 'clients', d.get('client_procs'), 'conc', d['concurrency'], d['req_per_s'], 'p50', d['p50_ms'])"
