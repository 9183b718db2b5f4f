set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r06b_ab.txt
ab() { timeout -k 10 120 env "$@" >> gpurun_out/r06b_ab.txt || exit 1; }
for i in 1 2; do
  ab LQ_DEV_FF4K=1 AB_TAG=ff4k python dev/ab_r06.py fftfilt 512
  ab LQ_DEV_FF8=2 AB_TAG=ff8_wpc2 python dev/ab_r06.py fftfilt 512
  ab LQ_DEV_FF8=3 AB_TAG=ff8_wpc3 python dev/ab_r06.py fftfilt 512
  ab LQ_DEV_RS4ST=1 AB_TAG=rs4st1 python dev/ab_r06.py resamp 1.037
  ab LQ_DEV_RS4ST=2 AB_TAG=rs4st2 python dev/ab_r06.py resamp 1.037
  ab LQ_DEV_FIRILV=0 AB_TAG=firilv0 python dev/ab_r06.py firfilt 64
  ab LQ_DEV_FIRILV=1 AB_TAG=firilv1 python dev/ab_r06.py firfilt 64
  ab LQ_DEV_FIRILV=2 AB_TAG=firilv2 python dev/ab_r06.py firfilt 64
  ab LQ_DEV_A4OLD=1 AB_TAG=a4old python dev/ab_r06.py pfb2 4096
  ab AB_TAG=a4dma python dev/ab_r06.py pfb2 4096
done
ab LQ_DEV_FF4K=1 AB_TAG=ff4k python dev/ab_r06.py fftfilt 64
ab LQ_DEV_FF8=2 AB_TAG=ff8_wpc2 python dev/ab_r06.py fftfilt 64
ab AB_TAG=fir256_fft python dev/ab_r06.py firfilt 256
cat gpurun_out/r06b_ab.txt
timeout -k 10 200 tools/mb/bin/mb_pat12b > gpurun_out/r06b_pat12b.txt || exit 1
cat gpurun_out/r06b_pat12b.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r06b_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r06b_pytest.log
[ $rc -le 1 ] || exit $rc
