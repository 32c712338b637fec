set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum --output-format csv -d $R/gpurun_out/pmc1 -o a -- python3 $R/bench/micro_attn_decode.py 32 512 640 > $R/gpurun_out/pmc1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc2 -o a -- python3 $R/bench/micro_attn_decode.py 32 512 640 > $R/gpurun_out/pmc2.log 2>&1 || exit 2
