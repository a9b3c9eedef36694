# split kernels at hidden 256: candidate-group width (NC) sweep at cfg3's K
set -e
mkdir -p gpurun_out
for k in split2 split4; do
  for wl in cfg3_h256 cfg3_ppo_net; do
    BCMPC_KERNEL=$k timeout -k 10 120 python -u bench.py --workload $wl --precision split --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/aknc.log 2>&1
  done
done
