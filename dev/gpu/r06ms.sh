set -o pipefail
cd /root/repo
mkdir -p gpurun_out
for c in off 24 23 22 21 off 23 22; do
  if [ $c = off ]; then unset LQ_MS_CHUNK; else export LQ_MS_CHUNK=$c; fi
  timeout -k 10 120 python -u dev/ab_ms.py >> gpurun_out/r06ms_ab.txt 2>&1 || { tail -20 gpurun_out/r06ms_ab.txt; exit 1; }
done
cat gpurun_out/r06ms_ab.txt
LQ_MS_CHUNK=12 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "msresamp" --timeout 120 --timeout-method thread > gpurun_out/r06ms_pytest.log 2>&1 || { tail -30 gpurun_out/r06ms_pytest.log; exit 1; }
tail -2 gpurun_out/r06ms_pytest.log
