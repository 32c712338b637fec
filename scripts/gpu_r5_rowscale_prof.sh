# round 5: kernel stats — bench prefill with / without the row-scale norms, 70B TP=8 probe with / without single-chunk parts
# (the DIE_AB_* switches were temporary: removed once the A/B was recorded in profiles/r5_*)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
prof() {  # name, env, cmd...
  local name=$1 envv=$2; shift 2
  env $envv timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$name -o run -- "$@" \
    > gpurun_out/prof_$name.log 2>&1 || { tail -5 gpurun_out/prof_$name.log; return 1; }
  f=$(find gpurun_out/prof_$name -name '*kernel_stats.csv' | head -1)
  python scripts/prof_summary.py $f "$name" 16
}
prof pf_new X=1 python3 bench.py --steps 2 --warmup 1 && prof pf_old DIE_AB_PF_OLD=1 python3 bench.py --steps 2 --warmup 1 && \
prof tp_new X=1 python3 bench/tp_probe.py && prof tp_old DIE_AB_ATTN_OLD=1 python3 bench/tp_probe.py
