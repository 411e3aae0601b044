#!/bin/bash
# SQ (shader sequencer) counter passes for the validate kernel: where do the
# waves' cycles go (issue vs wait), and the per-wave instruction mix.  One
# rocprofv3 pass per counter group (no --pmc together with any trace domain).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/sq
mkdir -p $OUT
ARGS=${SQ_ARGS:---steps 5 --warmup 1 --cpu-seconds 0 --ttfs-runs 0}
timeout -k 10 120 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1 || echo "list-avail rc=$?"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM" \
           "SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o sq -- \
      python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i ($grp) rc=$?"; tail -3 $OUT/p$i.log; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob("gpurun_out/sq/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "k_validate" in r["Kernel_Name"]:
            acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"  {c:28s} {sum(v)/len(v):16.1f}")
PY
