#!/bin/bash
# round 3: one-pass host MT19937 rows -- the NumPy-stream GPU tests, then the drop-in breakdown twice
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -m gpu -v --timeout 200 --timeout-method thread tests/test_gpu_mt.py \
  tests/test_gpu_dropin_soak.py tests/test_gpu_parity.py -k "mt or dropin or soak or fast_path or numpy_stream" \
  > gpurun_out/r03_mtflat_tests.log 2>&1 &&
timeout -k 10 200 python tools/dropin_breakdown.py ppo_defaults 400 > gpurun_out/r03_mtflat_breakdown.json 2>/dev/null &&
timeout -k 10 200 python tools/dropin_breakdown.py ppo_defaults 400 >> gpurun_out/r03_mtflat_breakdown.json 2>/dev/null
