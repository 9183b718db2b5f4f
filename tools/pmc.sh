#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only: no
# sys/runtime traces with --pmc) over tools/prof_run.py.  Usage: pmc.sh <what> <tag>
set -o pipefail
cd "$(dirname "$0")/.."
WHAT=${1:-pfb2}; TAG=${2:-pmc}; SQONLY=${3:-}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG; rm -rf $OUT; mkdir -p $OUT
python -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1 || exit 1
i=0
while read -r CTRS; do
  [ -z "$CTRS" ] && continue
  i=$((i+1))
  # third argument "sq": the three SQ passes only
  [ -n "$SQONLY" ] && [ $i -gt 3 ] && continue
  timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/p$i -o run -- python3 tools/prof_run.py --what $WHAT --iters 2 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done <<LIST
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM
SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_CVT_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32
FETCH_SIZE
WRITE_SIZE
GRBM_GUI_ACTIVE GRBM_COUNT
TCC_EA0_WRREQ_STALL TCC_TAG_STALL TCC_HIT TCC_MISS
LIST
for f in $(find $OUT -name "*counter_collection.csv"); do
  python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for r in rows:
    k = r.get("Kernel_Name", "?")[:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[k].add(r.get("Dispatch_Id", ""))
for k, d in agg.items():
    if "pfb2" in k or "firfilt" in k or "resamp" in k or "fftfilt" in k:
        print(k, len(cnt[k]), {c: "%.4g" % (v / max(1, len(cnt[k]))) for c, v in d.items()})
PY
done
