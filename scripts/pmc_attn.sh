# counter collection (--pmc, kernel trace only) on the attention microbenchmarks, one pass per run:
# WHICH=decode (default): decode attention, translation and L2-request counters (two passes);
# WHICH=prefill: prefill attention at ATTN_N x ATTN_L (default 4 x 4096), wave-state / VALU / MFMA / LDS counters
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
if [ "${WHICH:-decode}" = prefill ]; then
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $R/gpurun_out/pmc_attn -o attn -- python3 $R/bench/micro_attn_prefill.py ${ATTN_N:-4} ${ATTN_L:-4096} > $R/gpurun_out/pmc_attn.log 2>&1
  exit $?
fi
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum --output-format csv -d $R/gpurun_out/pmc1 -o a -- python3 $R/bench/micro_attn_decode.py 32 512 640 > $R/gpurun_out/pmc1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc2 -o a -- python3 $R/bench/micro_attn_decode.py 32 512 640 > $R/gpurun_out/pmc2.log 2>&1 || exit 2
