# relu / LayerNorm nets: split vs fp32 bench lines (profiles/r01_relu_ln_split_vs_fp32_bench.log)
set -e
mkdir -p gpurun_out
for wl in ppo_defaults cfg3_ppo_net cfg3_relu cfg3_h256; do
  for p in split fp32; do
    timeout -k 10 120 python -u bench.py --workload $wl --precision $p --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/ak.log 2>&1
  done
done
timeout -k 10 120 python -u bench.py --workload ppo_defaults --steps 20 --warmup 5 --cpu-baseline-seconds 5 >> gpurun_out/ak.log 2>&1
