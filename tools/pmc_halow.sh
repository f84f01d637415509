#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, kernel-trace only) over the single-layer
# microbenchmark of enc3: conv_halow (CLSKD_HALOW=1) vs conv_gemm8 (0).  Summary:
# tools/pmc_summary_kernels.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-pmchw}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
for hw in 1 0; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    rc=0; CLSKD_HALOW=$hw timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/hw${hw}_p$i -o run -- python3 $R/tools/conv_micro.py --only enc3 --iters 10 > $O/hw${hw}_p$i.log 2>&1 || rc=$?
    if [ $rc -ne 0 ]; then echo "stop: rc=$rc"; exit $rc; fi
  done
done
python3 $R/tools/pmc_summary_kernels.py $O > $O/summary.txt 2>&1; cat $O/summary.txt
