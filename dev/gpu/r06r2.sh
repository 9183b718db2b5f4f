set -o pipefail
cd /root/repo
mkdir -p gpurun_out
rm -f gpurun_out/r06r2_ab.txt
for rep in 1 2; do for v in r20 r21; do for w in "resamp2 0" "resamp2 1" "msresamp 0.3" "msresamp 3.3"; do
  LQ_LIB_PATH=$PWD/ab/$v/libliquid_mi355x.so timeout -k 10 120 python -u dev/ab_r06.py $w > gpurun_out/r06r2_one.txt 2>&1 || { cat gpurun_out/r06r2_one.txt; exit 1; }
  echo "$v $(grep -v amdgpu.ids gpurun_out/r06r2_one.txt | tail -1)" >> gpurun_out/r06r2_ab.txt
done; done; done
cat gpurun_out/r06r2_ab.txt
LQ_LIB_PATH=$PWD/ab/r21/libliquid_mi355x.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "resamp2 or msresamp" --timeout 120 --timeout-method thread > gpurun_out/r06r2_pytest.log 2>&1 || { tail -30 gpurun_out/r06r2_pytest.log; exit 1; }
tail -1 gpurun_out/r06r2_pytest.log
