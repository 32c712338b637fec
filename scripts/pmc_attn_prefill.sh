# PMC counters of the prefill attention kernel (bench/micro_attn_prefill.py 4 4096): one pass, <= 8 SQ counters
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc_attn -o attn -- python3 bench/micro_attn_prefill.py ${ATTN_N:-4} ${ATTN_L:-4096} > gpurun_out/pmc_attn.log 2>&1
echo "EXIT $?" >> gpurun_out/pmc_attn.log
