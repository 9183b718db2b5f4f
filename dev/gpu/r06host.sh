set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_small_calls.py tests/test_host_dot.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r06host5_pytest.log 2>&1 || { tail -30 gpurun_out/r06host5_pytest.log; exit 1; }
tail -2 gpurun_out/r06host5_pytest.log
N="firfilt_crcf_64 dotprod_crcf_64 dotprod_cccf_64 resamp_crcf_m8 firdecim_crcf_m8_h32 firinterp_crcf_m8_h32 fftfilt_crcf_64"
for i in 1 2 3; do for v in host_sse host_new host_al; do echo "== $v" >> gpurun_out/r06host5_percall.txt; LD_LIBRARY_PATH=$PWD/ab/$v timeout -k 10 120 build/ref_bench/percall --runtime 0.25 $N >> gpurun_out/r06host5_percall.txt 2>&1 || exit 1; done; done
python3 - <<'P'
import json,collections
r=collections.defaultdict(list); v=None
for l in open('gpurun_out/r06host5_percall.txt'):
    if l.startswith('=='): v=l.split()[1]; continue
    try: d=json.loads(l)
    except Exception: continue
    r[(d['name'],v)].append(round(d['trials_per_s']/1e6,1))
for k in sorted(r): print(k, r[k])
P
