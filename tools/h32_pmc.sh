#!/bin/bash
# SQ counters of the halo-tiled fp32 conv on the enc3 shape (diagnostic), one pass per group.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/h32pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
p=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU"; do
  p=$((p+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$p -o run -- python3 $R/tools/h32_modes.py --one > $O/p$p.log 2>&1 || { echo "pass $p failed"; tail -5 $O/p$p.log; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for f in sorted(glob.glob(O + "/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "conv_halo_f32" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(f"{k:28s} mean per dispatch {sum(v) / len(v):16.1f} over {len(v)}")
PY
