"""p50 of the synchronous get_action for a bench workload, without reading the kernel events
(so BCMPC_EVENTS=0 can be A/B'd).  usage: python tools/p50_probe.py workload [calls]"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402

wl_name = sys.argv[1]
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 500
wl = bench.WORKLOADS[wl_name]
prob = bench.synthetic_problem(wl)
eng = bench.make_engine(wl, prob, 0, "split")
state = prob["state"]
for i in range(50):
    eng.get_action(state, None, seed=i)
ts = []
for i in range(calls):
    t0 = time.perf_counter()
    eng.get_action(state, None, seed=1000 + i)
    ts.append(time.perf_counter() - t0)
print(f"{wl_name} events={os.environ.get('BCMPC_EVENTS', '1')} kernel={eng.info()['kernel']} "
      f"p50={np.median(ts) * 1e3:.4f} ms p10={np.percentile(ts, 10) * 1e3:.4f} ms", flush=True)
eng.close()
