#!/bin/bash
# round 3: the whole GPU suite with its printed error envelopes (-s), one process
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -v -s --timeout 300 --timeout-method thread tests "$@" \
  > gpurun_out/r03_full.log 2>&1
