# dev: firfilt_crcf h=64 timing, matrix-core kernel vs the VALU kernel (bench.py firfilt leg)
set -o pipefail
run() { timeout -k 10 300 python bench.py --no-cpu-baseline --no-resamp --no-extra --steps 30 --warmup 10 > gpurun_out/bv.log 2>&1 || return 1
  python -c "import json; d=json.loads(open('gpurun_out/bv.log').read().strip().splitlines()[-1]); print('$1', round(d['firfilt_crcf_h64']['ms_per_step'],4), 'pfb2', round(d['ms_per_step'],4))"; }
run mfma_warm && run mfma && LQ_FIRFILT_NO_MFMA=1 run valu
