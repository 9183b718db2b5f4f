#!/bin/bash
# Round-6: channelizer parity on the main build after the M = 1024 prefetch
# changes (firpfbch2 / firpfbch analyzers and synthesizers, full-size config 4,
# shards).
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_shard.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread -k "pfb or shard or config4" > gpurun_out/r06m_pytest.log 2>&1; rc=$?
tail -4 gpurun_out/r06m_pytest.log
exit $rc
