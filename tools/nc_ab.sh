cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for wl in cfg3_policy cfg3_polrew; do
  for k in split4 split2 split4 split2; do
    BCMPC_KERNEL=$k timeout -k 10 120 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/nc_$wl_$k.log 2>&1 || exit $?
    python -c "
import json,sys; d=json.loads(open('gpurun_out/nc_$wl_$k.log').read().strip().split('\n')[-1]); print('$wl $k', round(d['value']/1e8,3), d['kernel_ms_avg'], d['config'].get('workload','')[:60])"
  done
done
