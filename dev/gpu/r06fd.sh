set -o pipefail
cd /root/repo
mkdir -p gpurun_out
rm -f gpurun_out/r06fd6_ab.txt
for v in fdC fdH; do for M in 2 3 4 5 6 8 12 16 20; do
  LQ_LIB_PATH=$PWD/ab/$v/libliquid_mi355x.so timeout -k 10 120 python -u dev/ab_r06.py firdecim $M > gpurun_out/r06fd_one.txt 2>&1 || { cat gpurun_out/r06fd_one.txt; exit 1; }
  echo "$v $(grep -v amdgpu.ids gpurun_out/r06fd_one.txt | tail -1)" >> gpurun_out/r06fd6_ab.txt
done; done
cat gpurun_out/r06fd6_ab.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_configs.py tests/test_gpu_small_calls.py -q -x -k "decim or firdecim" --timeout 120 --timeout-method thread > gpurun_out/r06fd_pytest.log 2>&1 || { tail -30 gpurun_out/r06fd_pytest.log; exit 1; }
tail -1 gpurun_out/r06fd_pytest.log
