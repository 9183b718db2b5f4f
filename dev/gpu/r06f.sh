set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06f_ab.txt
ab() { timeout -k 10 120 env "$@" >> gpurun_out/r06f_ab.txt || exit 1; }
for i in 1 2; do
  for r in 0 4 8 16 32; do
    ab LQ_DEV_PFB2R=$r AB_TAG=runs$r python dev/ab_r06.py pfb2 1024
  done
done
cat gpurun_out/r06f_ab.txt
LQ_DEV_PFB2R=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_shard.py -m gpu -q --timeout 120 --timeout-method thread -k "firpfbch2 or pfb2 or shard" > gpurun_out/r06f_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/r06f_pytest.log
[ $rc -le 1 ] || exit $rc
