#!/bin/bash
# Kernel-trace summary of the bench command + PMC traffic passes; writes
# gpurun_out/<tag>/ (copy the summaries into profiles/).
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-prof}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG; rm -rf $OUT; mkdir -p $OUT
python -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1 || exit 1
# the driver's command (--steps 20 --warmup 5; bench.py adds its warm-up floor)
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-percall > $OUT/bench_under_rocprof.log 2>&1 || { tail -20 $OUT/bench_under_rocprof.log; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $OUT/$C -o run -- python3 tools/prof_run.py --what all --iters 2 > $OUT/$C.log 2>&1 || { tail -5 $OUT/$C.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, json, os, sys, collections
out = sys.argv[1]
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(os.path.join(out, c, "**", "*counter_collection.csv"), recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        key = "firpfbch2" if "pfb2" in k else ("firfilt" if "firfilt" in k else ("resamp" if "k_resamp" in k else
                                                                              ("fftfilt" if "k_fftfilt" in k else None)))
        if key:
            res.setdefault(key, {})[c] = sum(v) / len(v)
traffic = {}
for key, d in res.items():
    # gfx950: FETCH_SIZE (KB) reports half the bytes of a wide coalesced stream -> x2;
    # WRITE_SIZE (KB) is exact for streaming stores (MI355X_MICROARCH.md, HBM)
    rd = 2.0 * d.get("FETCH_SIZE", 0) * 1024
    wr = d.get("WRITE_SIZE", 0) * 1024
    traffic[key] = {"read_bytes": rd, "write_bytes": wr, "total_bytes": rd + wr,
                    "raw_FETCH_SIZE_KB": d.get("FETCH_SIZE"), "raw_WRITE_SIZE_KB": d.get("WRITE_SIZE")}
json.dump({"firpfbch2_bytes_per_launch": traffic.get("firpfbch2", {}).get("total_bytes"),
           "firfilt_bytes_per_launch": traffic.get("firfilt", {}).get("total_bytes"),
           "resamp_bytes_per_launch": traffic.get("resamp", {}).get("total_bytes"),
           "fftfilt_bytes_per_launch": traffic.get("fftfilt", {}).get("total_bytes"),
           "detail": traffic,
           "launch_shapes": {"firpfbch2": "M=1024 m=4, 2^27 input samples", "firfilt": "h=64, 2^28 samples",
                             "resamp": "r=1.037 m=7 npfb=64, 2^25 input samples (k_resamp4: 8-byte loads, "
                                       "16-byte stores; the x2 FETCH correction is calibrated for 16-byte streams)",
                             "fftfilt": "h=512, 4096-point overlap-save, 2^26 samples"},
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over tools/prof_run.py; "
                     "FETCH_SIZE doubled per the gfx950 correction",
           "measured": "%s, profile tag %s" % (__import__("time").strftime("%Y-%m-%d"), os.path.basename(out))},
          open(os.path.join(out, "traffic.json"), "w"), indent=1)
print(json.dumps(traffic))
PY
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
# the bench's timed window: the last 20 dispatches of each hot kernel (the
# warm-up dispatches before them are in kernel_stats.csv's average)
python3 - $OUT <<'PY'
import csv, glob, json, os, sys, collections
out = sys.argv[1]
f = glob.glob(os.path.join(out, "trace", "**", "*kernel_trace.csv"), recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    d[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
res = {}
for k, v in d.items():
    key = "firpfbch2" if "pfb2" in k else ("firfilt" if ("k_firfilt<" in k or "k_firfilt_mx" in k) else
                                           ("resamp" if "k_resamp" in k else ("fftfilt" if "k_fftfilt" in k else None)))
    if not key or len(v) < 20:
        continue
    v.sort()
    last = [e - s for s, e in v[-20:]]
    res[key] = {"kernel": k[:120], "dispatches": len(v), "timed_window_avg_us": sum(last) / len(last) / 1e3,
                "timed_window_min_us": min(last) / 1e3, "timed_window_max_us": max(last) / 1e3,
                "all_avg_us": sum(e - s for s, e in v) / len(v) / 1e3}
json.dump(res, open(os.path.join(out, "timed_window.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
PY
head -5 $OUT/kernel_stats.csv | cut -c1-200
