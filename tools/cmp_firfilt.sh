# dev: firfilt_crcf h=64 timing across kernel variants (bench.py firfilt leg)
set -o pipefail
run() { timeout -k 10 300 python bench.py --no-cpu-baseline --no-resamp --no-extra --steps 30 --warmup 10 > gpurun_out/bv.log 2>&1 || return 1
  python -c "import json; d=json.loads(open('gpurun_out/bv.log').read().strip().splitlines()[-1]); print('$1', round(d['firfilt_crcf_h64']['ms_per_step'],4), 'pfb2', round(d['ms_per_step'],4))"; }
LQ_FIRFILT_NO_MFMA=1 run valu_warm && LQ_FIRFILT_NO_MFMA=1 run valu && LQ_MX_VARIANT=3 run mx_ntl_nts && LQ_MX_VARIANT=1 run mx_ntl && LQ_MX_VARIANT=2 run mx_nts && LQ_MX_VARIANT=0 run mx_plain
