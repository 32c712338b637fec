set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE TCC_EA0_RDREQ_sum --output-format csv -d $R/gpurun_out/pmcg1 -o a -- python3 $R/bench/pmc_gate_up.py > $R/gpurun_out/pmcg1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum --output-format csv -d $R/gpurun_out/pmcg2 -o a -- python3 $R/bench/pmc_gate_up.py > $R/gpurun_out/pmcg2.log 2>&1 || exit 2
