#!/bin/bash
# round 4: a team-kernel change against build/variants/libbcmpc_oldteam.so (the previous commit) -- the GPU suite, then small-K A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests \
  \
  > gpurun_out/r04_team_sched2_tests.log 2>&1 || { tail -30 gpurun_out/r04_team_sched2_tests.log; exit 1; }
tail -1 gpurun_out/r04_team_sched2_tests.log
rm -f gpurun_out/r04_team_sched2_ab.jsonl
for r in 0 1; do
  for v in new ${VARIANTS:-oldteam}; do
    if [ $v = new ]; then L=""; else L=$PWD/build/variants/libbcmpc_$v.so; fi
    BCMPC_LIB=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --dropin-calls 0 --no-f16 \
      --no-cfg2 2>/dev/null | python -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print(json.dumps({'lib': '$v', 'round': $r, **{k: [round(v['p50_ms']*1e3,1), round(v['kernel_ms']*1e3,1), round(v['dropin_parity_p50_ms']*1e3,1) if v.get('dropin_parity_p50_ms') else None] for k, v in d['small_k'].items()}}))
" >> gpurun_out/r04_team_sched2_ab.jsonl || exit 1
  done
done
cat gpurun_out/r04_team_sched2_ab.jsonl
