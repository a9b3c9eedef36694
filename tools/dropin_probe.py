"""Drop-in (NumPy-stream) MPCcontroller.get_action p50 for a bench workload (plain delta nets),
for A/B of the draw path (BCMPC_MT_PATH=host|device).  usage: python tools/dropin_probe.py wl [calls]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402

name = sys.argv[1]
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 300
wl = bench.WORKLOADS[name]
p = bench.synthetic_problem(wl)
r = bench.dropin_parity_p50(wl["K"], wl["H"], wl["hidden"], wl["L"], wl["act"], p["ln"], p["kernels"], p["biases"],
                            p["ln_g"], p["ln_b"], p["norm"], p["state"], 0, calls, 1)
print(f"{name} mt_path={os.environ.get('BCMPC_MT_PATH', 'device')} dropin p50={r['p50_ms']:.4f} ms "
      f"p90={r['p90_ms']:.4f} ms", flush=True)
