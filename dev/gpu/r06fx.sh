set -o pipefail
cd /root/repo
mkdir -p gpurun_out
for rep in 1 2 3; do for v in fx0 fx1; do
  LQ_LIB_PATH=$PWD/ab/$v/libliquid_mi355x.so timeout -k 10 120 python -u dev/ab_r06.py firfilt 64 > gpurun_out/r06fx_one.txt 2>&1 || { cat gpurun_out/r06fx_one.txt; exit 1; }
  echo "$v $(grep -v amdgpu.ids gpurun_out/r06fx_one.txt | tail -1)" >> gpurun_out/r06fx_ab.txt
  LQ_LIB_PATH=$PWD/ab/$v/libliquid_mi355x.so timeout -k 10 120 python -u dev/ab_r06.py firfilt_cccf 64 > gpurun_out/r06fx_one.txt 2>&1 || { cat gpurun_out/r06fx_one.txt; exit 1; }
  echo "$v $(grep -v amdgpu.ids gpurun_out/r06fx_one.txt | tail -1)" >> gpurun_out/r06fx_ab.txt
done; done
cat gpurun_out/r06fx_ab.txt
LQ_LIB_PATH=$PWD/ab/fx1/libliquid_mi355x.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "firfilt" --timeout 120 --timeout-method thread > gpurun_out/r06fx_pytest.log 2>&1 || { tail -30 gpurun_out/r06fx_pytest.log; exit 1; }
tail -2 gpurun_out/r06fx_pytest.log
