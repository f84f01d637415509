#!/bin/bash
# C5 fused hop: SQ / SQC counters of the hop kernel (diagnostic), one pass per counter group.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c5pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o -E "^[[:space:]]*(SQ|SQC)_[A-Z0-9_]+" $O/avail.txt | sort -u > $O/sq_names.txt || true
p=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" \
           "SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"; do
  p=$((p+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$p -o run -- python $R/tools/stream_bench.py --engine fused --streams 1 --seconds 2 > $O/p$p.log 2>&1 || echo "pass $p failed"
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for f in sorted(glob.glob(O + "/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "stream_hop_kernel" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(f"{k:28s} mean per dispatch {sum(v) / len(v):14.1f} over {len(v)}")
PY
