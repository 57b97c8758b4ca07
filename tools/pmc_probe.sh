#!/bin/bash
# List counters, then collect SQ/TCC counter passes (one rocprofv3 run per pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-pmc}
timeout -k 10 120 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1
run() { # name counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/${TAG}_$name -o p \
    -- python3 bench.py --steps 6 --warmup 2 --no-cpu --no-e2e --copies 4 ${BENCH_ARGS} > gpurun_out/${TAG}_$name.log 2>&1
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
 && run sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
 && run sq3 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH \
 && run fetch FETCH_SIZE \
 && run write WRITE_SIZE \
 && echo PMC_OK
