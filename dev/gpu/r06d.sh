set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06d_ab.txt
ab() { timeout -k 10 120 env "$@" >> gpurun_out/r06d_ab.txt || exit 1; }
B=/root/repo/ab/base/libliquid_mi355x.so
S=/root/repo/ab/ldsync/libliquid_mi355x.so
for i in 1 2; do
  for w in "fftfilt 512" "fft 4096" "fft 1024" "pfb2 256" "pfb2 512" "pfbsyn 256" "pfb2 2048"; do
    ab LQ_LIB_PATH=$B AB_TAG=base python dev/ab_r06.py $w
    ab LQ_LIB_PATH=$S AB_TAG=ldsync python dev/ab_r06.py $w
  done
  ab LQ_LIB_PATH=/root/repo/ab/e0/libliquid_mi355x.so AB_TAG=pfb_e0 python dev/ab_r06.py pfb2 1024
  ab LQ_LIB_PATH=/root/repo/ab/e6/libliquid_mi355x.so AB_TAG=pfb_e6 python dev/ab_r06.py pfb2 1024
  ab LQ_LIB_PATH=$S AB_TAG=nt python dev/ab_r06.py resamp 1.037
  ab LQ_LIB_PATH=/root/repo/ab/plain/libliquid_mi355x.so AB_TAG=plain python dev/ab_r06.py resamp 1.037
  ab LQ_LIB_PATH=$S LQ_DEV_RS4ST=2 AB_TAG=nt_st2 python dev/ab_r06.py resamp 1.037
  ab LQ_LIB_PATH=/root/repo/ab/plain/libliquid_mi355x.so LQ_DEV_RS4ST=2 AB_TAG=plain_st2 python dev/ab_r06.py resamp 1.037
  ab LQ_LIB_PATH=/root/repo/ab/plain/libliquid_mi355x.so AB_TAG=plain python dev/ab_r06.py fftfilt 512
  ab LQ_LIB_PATH=$S AB_TAG=fw4 python dev/ab_r06.py firfilt 64
  ab LQ_LIB_PATH=/root/repo/ab/fw5/libliquid_mi355x.so AB_TAG=fw5 python dev/ab_r06.py firfilt 64
  ab LQ_LIB_PATH=/root/repo/ab/fw6/libliquid_mi355x.so AB_TAG=fw6 python dev/ab_r06.py firfilt 64
  ab LQ_LIB_PATH=$S LQ_DEV_FF8ALL=1 LQ_DEV_FF8H=1 AB_TAG=ff8h python dev/ab_r06.py fftfilt 512
  ab LQ_LIB_PATH=$S LQ_DEV_FF8ALL=1 LQ_DEV_FF8H=1 AB_TAG=ff8h python dev/ab_r06.py fftfilt 64
  ab LQ_LIB_PATH=$S LQ_DEV_FF8ALL=1 LQ_DEV_FF8H=1 AB_TAG=ff8h python dev/ab_r06.py firfilt 256
done
cat gpurun_out/r06d_ab.txt
LQ_DEV_FF8ALL=1 LQ_DEV_FF8H=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu -q --timeout 120 --timeout-method thread -k "fftfilt or firfilt" > gpurun_out/r06d_pytest_ff8h.log 2>&1; rc=$?
tail -5 gpurun_out/r06d_pytest_ff8h.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r06d_pytest.log 2>&1; rc=$?
tail -8 gpurun_out/r06d_pytest.log
[ $rc -le 1 ] || exit $rc
