set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06c_ab.txt
ab() { timeout -k 10 120 env "$@" >> gpurun_out/r06c_ab.txt || exit 1; }
for i in 1 2; do
  for e in 0 1 2 3 4 5; do
    ab LQ_LIB_PATH=/root/repo/ab/e$e/libliquid_mi355x.so AB_TAG=pfb2_e$e python dev/ab_r06.py pfb2 1024
  done
done
ab AB_TAG=fir256 python dev/ab_r06.py firfilt 256
ab AB_TAG=fir128 python dev/ab_r06.py firfilt 128
ab AB_TAG=ff512 python dev/ab_r06.py fftfilt 512
ab AB_TAG=pfb4096 python dev/ab_r06.py pfb2 4096
cat gpurun_out/r06c_ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r06c_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r06c_pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06c_smoke.log 2>&1 || { cat gpurun_out/r06c_smoke.log; exit 1; }
cat gpurun_out/r06c_smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06c_bench.log 2>&1 || { tail -30 gpurun_out/r06c_bench.log; exit 1; }
tail -c 3000 gpurun_out/r06c_bench.log
