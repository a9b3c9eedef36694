"""Time NNDynamicsModel.fit on the GPU (csrc/fit.hip) vs the NumPy oracle on the host.

train_mpc_ppo.py defaults: dyn_iters 200 (:49), batch_size 512 (:50), 2x256 relu + LayerNorm
(:52, :74-75, :539), lr 1e-3 (:47).  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--act", default="relu")
    ap.add_argument("--ln", type=int, default=1)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--rows", type=int, default=20000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-iters", type=int, default=20)
    ap.add_argument("--reward", type=int, default=0,
                    help="1: NNDynamicsRewardModel.fit (dynamics.py:195-219; run.sh's model: 500 trunk + two "
                         "500 heads, tanh, LayerNorm with --ln 1)")
    args = ap.parse_args()
    if args.reward:
        return reward_main(args)
    import torch  # noqa: F401  (single HIP runtime)
    from bc_mpc_amd.engine import MLPSpec
    from bc_mpc_amd.fit import GPUFitter
    from oracle import mpc_oracle as orc
    S, A = 20, 6
    w = orc.synthetic_weights(S, A, args.hidden, args.layers, args.act, bool(args.ln), seed_base=11)
    rs = np.random.RandomState(5)
    norm = orc.synthetic_normalization(S, A)
    states = norm[0] + norm[1] * rs.standard_normal((args.rows, S))
    actions = rs.uniform(-1, 1, (args.rows, A))
    deltas = norm[8] + norm[9] * rs.standard_normal((args.rows, S))
    batches = [rs.choice(args.rows, args.batch, replace=False) for _ in range(args.iters)]
    f = GPUFitter(S, A, args.hidden, args.layers, args.act, bool(args.ln), args.batch, 1e-3, device=0)
    f.set_params(MLPSpec(w.kernels, w.biases, args.act, w.ln_gamma, w.ln_beta), norm)
    f.set_data(states, actions, deltas)
    f.run(batches[:10])                                   # warm-up
    times = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        f.run(batches)
        times.append(time.perf_counter() - t0)
    gpu_s = float(np.median(times))
    ps = orc.fit_params(w)
    st = orc.AdamState.zeros_like(ps)
    t0 = time.perf_counter()
    orc.fit(ps, st, args.layers, args.act, bool(args.ln), norm, states, actions, deltas,
            batches[:args.cpu_iters], 1e-3)
    cpu_per_iter = (time.perf_counter() - t0) / args.cpu_iters
    dims = [S + A] + [args.hidden] * args.layers + [S]
    mac = sum(dims[i] * dims[i + 1] for i in range(len(dims) - 1))
    flop_iter = 3 * 2 * mac * args.batch                 # forward + two backward GEMMs per layer
    print(json.dumps({
        "metric": "NNDynamicsModel.fit wall time (dynamics.py:81-104)",
        "config": f"{args.layers}x{args.hidden} {args.act}{' + LN' if args.ln else ''}, batch {args.batch}, "
                  f"{args.iters} Adam iterations",
        "gpu_ms_per_fit": gpu_s * 1e3, "gpu_us_per_iteration": gpu_s / args.iters * 1e6,
        "gpu_tflops": flop_iter * args.iters / gpu_s / 1e12,
        "cpu_oracle_ms_per_iteration": cpu_per_iter * 1e3,
        "cpu_oracle_ms_per_fit_extrapolated": cpu_per_iter * args.iters * 1e3,
        "cpu_threads": os.environ.get("OMP_NUM_THREADS", "default"),
    }))
    f.close()


def reward_main(args):
    import torch  # noqa: F401  (single HIP runtime)
    from bc_mpc_amd.engine import MLPSpec
    from bc_mpc_amd.fit import GPUFitter
    from oracle import mpc_oracle as orc
    S, A, h, ln = 20, 6, args.hidden, bool(args.ln)
    w = orc.synthetic_reward_weights(S, A, h, ln, seed_base=31)
    rs = np.random.RandomState(5)
    norm = orc.synthetic_normalization(S, A, reward=True)
    states = norm[0] + norm[1] * rs.standard_normal((args.rows, S))
    actions = rs.uniform(-1, 1, (args.rows, A))
    deltas = norm[8] + norm[9] * rs.standard_normal((args.rows, S))
    rewards = rs.standard_normal(args.rows)
    batches = [rs.choice(args.rows, args.batch, replace=False) for _ in range(args.iters)]
    f = GPUFitter(S, A, h, 2, "tanh", ln, args.batch, 1e-3, device=0, model="reward")
    f.set_params(MLPSpec(w.kernels, w.biases, "tanh", w.ln_gamma, w.ln_beta, model="reward"), norm)
    f.set_data(states, actions, deltas)
    f.set_rewards(rewards)
    f.run(batches[:10])                                   # warm-up
    times = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        f.run(batches)
        times.append(time.perf_counter() - t0)
    gpu_s = float(np.median(times))
    ps = orc.fit_reward_params(w)
    st = orc.AdamState.zeros_like(ps)
    t0 = time.perf_counter()
    orc.fit_reward(ps, st, ln, norm, states, actions, rewards, deltas, batches[:args.cpu_iters], 1e-3)
    cpu_per_iter = (time.perf_counter() - t0) / args.cpu_iters
    mac = (S + A) * h + 2 * h * h + h * S + h
    flop_iter = 3 * 2 * mac * args.batch
    print(json.dumps({
        "metric": "NNDynamicsRewardModel.fit wall time (dynamics.py:195-219)",
        "config": f"reward net {h} trunk + 2x{h} heads tanh{' + LN' if ln else ''}, batch {args.batch}, "
                  f"{args.iters} Adam iterations",
        "gpu_ms_per_fit": gpu_s * 1e3, "gpu_us_per_iteration": gpu_s / args.iters * 1e6,
        "gpu_tflops": flop_iter * args.iters / gpu_s / 1e12,
        "cpu_oracle_ms_per_iteration": cpu_per_iter * 1e3,
        "cpu_oracle_ms_per_fit_extrapolated": cpu_per_iter * args.iters * 1e3,
        "cpu_threads": os.environ.get("OMP_NUM_THREADS", "default"),
    }))
    f.close()


if __name__ == "__main__":
    main()
