set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r06final3_pytest.log 2>&1; rc=$?
tail -6 gpurun_out/r06final3_pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06final3_smoke.log 2>&1 || { cat gpurun_out/r06final3_smoke.log; exit 1; }
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06final3_bench.log 2>&1 || { tail -30 gpurun_out/r06final3_bench.log; exit 1; }
tail -c 1500 gpurun_out/r06final3_bench.log
bash tools/profile_round.sh r06final3_prof > gpurun_out/r06final3_prof.log 2>&1 || { tail -30 gpurun_out/r06final3_prof.log; exit 1; }
tail -30 gpurun_out/r06final3_prof.log
timeout -k 10 600 python tools/bench_widened.py > gpurun_out/r06final3_widened.json 2> gpurun_out/r06final3_widened.err || { tail -5 gpurun_out/r06final3_widened.err; exit 1; }
wc -l gpurun_out/r06final3_widened.json
