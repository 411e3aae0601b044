#!/bin/bash
# SQ (shader sequencer) counter passes for the validate kernel: where do the
# waves' cycles go (issue vs wait), the per-wave instruction mix, and the mean
# VMEM / LDS latency (SQ_INST_LEVEL_x / SQ_INSTS_x, cycles in flight per
# instruction).  One rocprofv3 pass per counter group (<= 8 SQ counters each,
# no --pmc together with any trace domain); each pass has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${SQ_OUT:-gpurun_out/sq}
mkdir -p $OUT
ARGS=${SQ_ARGS:---steps 5 --warmup 1 --cpu-seconds 0 --ttfs-runs 0 --lookup-micro 0 --config2 0 --fresh-batches 0 --streams 1}
timeout -k 10 60 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1 || echo "list-avail rc=$?"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM" \
           "SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64" \
           "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVE_CYCLES"; do
  i=$((i+1))
  echo "sq pass $i: $grp"
  timeout -k 10 150 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o sq -- \
      ${SQ_CMD:-python3 bench.py $ARGS} > $OUT/p$i.log 2>&1 || { echo "pass $i ($grp) rc=$?"; tail -3 $OUT/p$i.log; }
done
python3 - "$OUT" "${SQ_KERNEL:-k_validate}" <<'PY'
import csv, glob, collections, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if sys.argv[2] in r["Kernel_Name"]:
            acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    for c, v in sorted(m.items()):
        print(f"  {c:28s} {v:16.1f}")
    for lvl, n in (("SQ_INST_LEVEL_VMEM", "SQ_INSTS_VMEM"), ("SQ_INST_LEVEL_LDS", "SQ_INSTS_LDS")):
        if m.get(n):
            print(f"  {lvl + '/' + n:28s} {m.get(lvl, 0) / m[n]:16.1f}  (mean cycles in flight)")
    if m.get("SQ_WAVE_CYCLES"):
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if c in m:
                print(f"  {c + ' / WAVE_CYCLES':28s} {m[c] / m['SQ_WAVE_CYCLES']:16.3f}")
PY
