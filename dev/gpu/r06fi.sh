set -o pipefail
cd /root/repo
mkdir -p gpurun_out
rm -f gpurun_out/r06fi_ab.txt
for rep in 1 2; do for v in fi0 fi1; do for M in 8 2 4; do
  LQ_LIB_PATH=$PWD/ab/$v/libliquid_mi355x.so timeout -k 10 120 python -u dev/ab_r06.py firinterp $M > gpurun_out/r06fi_one.txt 2>&1 || { cat gpurun_out/r06fi_one.txt; exit 1; }
  echo "$v $(grep -v amdgpu.ids gpurun_out/r06fi_one.txt | tail -1)" >> gpurun_out/r06fi_ab.txt
done; done; done
cat gpurun_out/r06fi_ab.txt
LQ_LIB_PATH=$PWD/ab/fi1/libliquid_mi355x.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "interp" --timeout 120 --timeout-method thread > gpurun_out/r06fi_pytest.log 2>&1 || { tail -30 gpurun_out/r06fi_pytest.log; exit 1; }
tail -1 gpurun_out/r06fi_pytest.log
