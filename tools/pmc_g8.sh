#!/bin/bash
# timing-only engine modes need the experiments build: CLSKD_EXPERIMENTS=1 python -m clskd.build (run on the CPU first)
export CLSKD_LIB=exp
# PMC passes over the conv_gemm8 microbenchmark (one layer, CLSKD_G8 modes in $MODES); each
# pass its own rocprofv3 run (gfx950 per-block slot limits), kernel-trace only.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc8
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_DATA_FIFO_FULL SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE"
P3="TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES"
for m in ${MODES:-1 13}; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    CLSKD_G8=$m timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/m${m}_p$i -o run -- python3 $R/tools/conv_micro.py --only ${ONLY:-enc3} --iters 10 > $O/m${m}_p$i.log 2>&1
  done
done
echo ok
