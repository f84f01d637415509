#!/bin/bash
# conv_gemm8 on the teacher's conv shapes vs plain GEMMs of the same engine (1x1, contiguous rows),
# product library, then the experiments library's timing modes (11 no DMA, 12 no MFMA).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${ITER:-g8plain}
mkdir -p $O
ok() { local rc=$1; if [ $rc -ne 0 ]; then echo "stop: rc=$rc"; exit $rc; fi; }
L=enc3,enc4,pw_enc4,pw64k
rc=0; timeout -k 10 150 python -u $R/tools/conv_micro.py --iters 30 --only $L > $O/prod.txt 2>&1 || rc=$?; ok $rc
for m in 11 12 13; do
  rc=0; CLSKD_LIB=exp CLSKD_G8=$m timeout -k 10 150 python -u $R/tools/conv_micro.py --iters 30 --only $L > $O/exp$m.txt 2>&1 || rc=$?; ok $rc
done
rc=0; timeout -k 10 100 $R/tools/probe/stage_rate > $O/stage_rate.txt 2>&1 || rc=$?; ok $rc
for f in $O/*.txt; do echo "== $f"; grep -v amdgpu.ids $f; done
