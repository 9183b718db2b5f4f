#!/bin/bash
# Two SQ counter passes (kernel-trace only) over tools/prof_run.py for each
# --what given (dev tool; the library must already be built in-tree).
# Usage: pmc_sq.sh <tag> what1 [what2 ...]
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG; rm -rf $OUT; mkdir -p $OUT
for W in "$@"; do
  i=0
  while read -r CTRS; do
    [ -z "$CTRS" ] && continue
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/$W$i -o run -- python3 tools/prof_run.py --what $W --iters 2 > $OUT/$W$i.log 2>&1 || { echo "pass $W $i failed"; tail -5 $OUT/$W$i.log; exit 1; }
  done <<LIST
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM
LIST
done
for f in $(find $OUT -name "*counter_collection.csv" | sort); do
  python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for r in rows:
    k = r.get("Kernel_Name", "?")[:50]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[k].add(r.get("Dispatch_Id", ""))
for k, d in agg.items():
    if "resamp" in k or "pfb" in k or "fir" in k or "fft" in k:
        print(sys.argv[1].split("/")[2], k, len(cnt[k]), {c: "%.4g" % (v / max(1, len(cnt[k]))) for c, v in d.items()})
PY
done
