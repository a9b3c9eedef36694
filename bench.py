#!/usr/bin/env python3
"""Benchmark: random-shooting MPC get_action on MI355X (libbcmpc).

One "step" = one complete control step of MPCcontroller.get_action
(controllers.py:57-88) through the library's synchronous entry point
(bcmpc_get_action): the host state goes in, K candidate action sequences of
horizon H are drawn on the device (Philox, ``--actions device``, default),
rolled through the dynamics MLP, scored with the cheetah cost, argmin'd, and
the result (index, cost, first action) comes back to the host.  ``p50_ms`` is
the latency of that call; ``value`` = K*H*N / wall time.  ``--actions hbm``
times the older resident-input rollout (a [H, K, A] f64 array uploaded once
before timing) for A/B only.

``dropin_parity_p50_ms``: ``bc_mpc_amd.MPCcontroller.get_action`` with the
reference's RNG contract (rng="numpy": exactly the np.random.uniform(size=
[H, K_global, A]) draw of controllers.py:53 from the global legacy stream,
the first action taken from that array) at the same K and H -- the
drop-in's latency including the draw.

Multi-GPU: ``--gpus N`` runs N ranks, one per GPU -- started by the driver's
torch.distributed.run (WORLD_SIZE must equal N), or, without WORLD_SIZE, by
this script itself (a child torch.distributed.run, before any GPU call).
Strong scaling on the north_star point by default: the workload's K is the
GLOBAL K (cfg3: K = 65,536, H = 20, split contiguously, 65,536 / N per GPU);
per step every rank runs its shard and the ranks agree on the global argmin
through ONE all-gather of the 144-byte result records, reduced on the device
(distributed.RecordExchange).  ``scale`` adds BASELINE's other global configs
at the same N (cfg4: K = 262,144; cfg5: K = 65,536 with CEM x4) and cfg3
weak-scaled.  Rank 0 prints ONE JSON line; its ``summary`` key (last) holds
every line's value / p50 / roofline fraction.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# BASELINE.json configs (S=20, A=6, 2x500 tanh unless stated)
WORKLOADS = {
    "cfg1": dict(K=1000, H=15, hidden=500, L=2, act="tanh"),
    "cfg2": dict(K=4096, H=20, hidden=500, L=2, act="tanh"),
    "cfg3": dict(K=65536, H=20, hidden=500, L=2, act="tanh"),
    "cfg4_shard": dict(K=32768, H=20, hidden=500, L=2, act="tanh"),   # 262144 / 8 per GPU
    "ns_shard": dict(K=8192, H=20, hidden=500, L=2, act="tanh"),      # the north_star's per-GPU shard: 65536 / 8
    "cfg3_relu": dict(K=65536, H=20, hidden=500, L=2, act="relu"),    # diagnostic: no tanh
    # diagnostics: cfg2's net at other K (the multi-column team kernel's auto bound)
    "k2048": dict(K=2048, H=20, hidden=500, L=2, act="tanh"),
    "k8192": dict(K=8192, H=20, hidden=500, L=2, act="tanh"),
    "k16384": dict(K=16384, H=20, hidden=500, L=2, act="tanh"),
    "cfg3_h256": dict(K=65536, H=20, hidden=256, L=2, act="tanh"),    # diagnostic: a 256-wide tanh net
    "cfg5_pass": dict(K=65536, H=50, hidden=1024, L=3, act="tanh"),   # one random-shooting pass of cfg5
    # MPCcontrollerPolicyNet (controllers.py:160-237) at cfg3 dims: 20->128->128->6 tanh policy fused per step,
    # self_exp=False, explore=0.5 (train_mpc_ppo.py:36-37,178 defaults)
    "cfg3_policy": dict(K=65536, H=20, hidden=500, L=2, act="tanh", policy=(128, 2), explore=0.5),
    # train_mpc_ppo.py's own net (:52,74-75,539): 2x256 relu + LayerNorm, 400 paths, horizon 7
    "ppo_defaults": dict(K=400, H=7, hidden=256, L=2, act="relu", ln=True),
    "cfg3_ppo_net": dict(K=65536, H=20, hidden=256, L=2, act="relu", ln=True),   # that net at cfg3's K, H
    # MPCcontrollerReward (controllers.py:90-158) on NNDynamicsRewardModel (dynamics.py:121-238): tanh trunk 500,
    # two 500 heads, argmax of sum_h reward * gamma**h
    "cfg3_reward": dict(K=65536, H=20, hidden=500, L=2, act="tanh", reward=True, gamma=0.99),
    # MPCcontrollerPolicyNetReward (controllers.py:289-363) at cfg3 dims, self_exp=False explore=0.5
    "cfg3_polrew": dict(K=65536, H=20, hidden=500, L=2, act="tanh", reward=True, policy=(128, 2), explore=0.5),
    # run.sh's active recipe: --LEARN_REWARD=True --SELFEXP=True --mpc_horizon=30, simulated_paths 400
    # (train_mpc_ppo.py:71): MPCcontrollerPolicyNetReward with the stochastic policy
    # BASELINE cfg5: K=65536, H=50, 3x1024 tanh with the CEM outer loop (4 iterations; elites 10%, smoothing 0.1;
    # DESIGN.md "CEM" -- the reference has no CEM).  One step = one CEMcontroller.get_action = 4 rollout passes.
    "cfg5": dict(K=65536, H=50, hidden=1024, L=3, act="tanh", cem=dict(iterations=4, elite_frac=0.1, alpha=0.1)),
    # (LAYER_NORM is not passed by run.sh, so its default True holds, train_mpc_ppo.py:52: the trunk and both heads
    # are LayerNorm'd, dynamics.py:165-177)
    "runsh_recipe": dict(K=400, H=30, hidden=500, L=2, act="tanh", ln=True, reward=True, policy=(128, 2),
                         explore=0.5, policy_mode="stochastic"),
    # the default MPC-aug path of train_mpc_ppo.py (:198-216, flags :36-37, :52, :71, :74-77, :178, :539):
    # MPCcontrollerPolicyNet over the 2x256 relu + LayerNorm NNDynamicsModel with the 2x128 tanh MlpPolicy,
    # self_exp=False, explore=0.5, 400 paths, horizon 7
    "ppo_mpc_default": dict(K=400, H=7, hidden=256, L=2, act="relu", ln=True, policy=(128, 2), explore=0.5),
    # diagnostic: the run.sh recipe's net without its LayerNorms (round 2's "runsh_recipe" line)
    "runsh_noln": dict(K=400, H=30, hidden=500, L=2, act="tanh", reward=True, policy=(128, 2), explore=0.5,
                       policy_mode="stochastic"),
}
S_DIM, A_DIM = 20, 6
FP32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: FP32 matrix, v_mfma_f32_16x16x4_f32
F16_MFMA_PEAK_TFLOPS = 2516.6     # dense f16/bf16 MFMA: 512 MAC/clk/SIMD x 1024 SIMDs x 2.4 GHz
# split precision: every f32 product = 3 f16 MFMA passes (hi*hi + hi*lo + lo*hi), so the
# f32-equivalent (algorithmic) ceiling is a third of the f16 peak
SPLIT_PEAK_TFLOPS = F16_MFMA_PEAK_TFLOPS / 3
HBM_PEAK_GBS = 8000.0
TRAFFIC_FILE = "r06_traffic_per_launch.json"


def flop_per_cand_step(hidden, L, S=S_DIM, A=A_DIM, policy=None, reward=False):
    """Algorithmic MLP FLOPs per candidate-step: 2*[(S+A)h + (L-1)h^2 + hS]
    (reward net, dynamics.py:167-174: 2*[(S+A)h + 2h^2 + hS + h])
    (+ the policy stack 2*[S*ph + (PL-1)ph^2 + ph*A] when fused)."""
    if reward:
        f = 2 * ((S + A) * hidden + 2 * hidden * hidden + hidden * S + hidden)
    else:
        f = 2 * ((S + A) * hidden + (L - 1) * hidden * hidden + hidden * S)
    if policy:
        ph, pl = policy
        f += 2 * (S * ph + (pl - 1) * ph * ph + ph * A)
    return f


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(spec_w, norm, state, H, budget_s, K_full, net, pol=None, explore=0.5, gamma=1.0, cem=None):
    """The oracle (NumPy restatement of the reference path, kind "port") timed on the host cores at the
    workload's FULL K (CEM workloads -- cfg5: minutes per full-size oracle call -- at K=1024) twice: with
    the BLAS pool's threads (calls until ``budget_s``) and with 1 thread (a K sample of about the same
    wall time when a full-K call would not fit).  ``value`` / ``cores`` are the faster of the two per
    candidate-step (at K=400 one thread beats the pool: NumPy's per-call overhead, not the GEMMs); the
    other stays in the record.  The pool size is the process's BLAS setting (OMP_NUM_THREADS, which the
    GPU box sets to its CPU share per GPU), not the machine's CPU count; the record names both and the
    process's CPU affinity."""
    from oracle import mpc_oracle as orc
    from threadpoolctl import threadpool_info, threadpool_limits
    reward = isinstance(spec_w, orc.RewardMLPWeights)
    threads = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    dyn = orc.NumpyRewardDynamics(spec_w, norm) if reward else orc.NumpyDynamics(spec_w, norm)
    low, high = -np.ones(A_DIM), np.ones(A_DIM)

    def one_call(Ks, calls, rs):
        if cem:                           # the oracle's CEM loop: iterations x Ks x H candidate-steps
            E = max(1, int(round(cem["elite_frac"] * Ks)))
            orc.cem_get_action(lambda s, a: orc.rollout(dyn, s, a)[0], state, H, Ks, low, high, cem["iterations"],
                               E, cem["alpha"], calls, np.zeros((H, A_DIM)), np.full((H, A_DIM), 0.5))
            return Ks * H * cem["iterations"]
        if reward and pol is None:        # MPCcontrollerReward body (env.sample stand-in: one uniform draw)
            orc.reward_rollout(dyn, state, rs.uniform(low, high, (H, Ks, A_DIM)), gamma)
        elif reward:
            orc.policy_reward_get_action(dyn, orc.NumpyPolicy(orc.PolicyWeights(*pol)), state, H, Ks, low, high,
                                         explore, rng=rs)
        elif pol is None:
            orc.get_action(dyn, state, H, Ks, low, high, rng=rs)
        else:
            orc.policy_get_action(dyn, orc.NumpyPolicy(orc.PolicyWeights(*pol)), state, H, Ks, low, high,
                                  explore, rng=rs)
        return Ks * H

    def timed(Ks, budget, max_calls=1 << 30):
        rs = np.random.RandomState(0)
        done, calls, t0 = 0, 0, time.perf_counter()
        while calls < max_calls:
            done += one_call(Ks, calls, rs)
            calls += 1
            if time.perf_counter() - t0 >= budget:
                break
        el = time.perf_counter() - t0
        return done / el, calls, el

    Ks = min(1024, K_full) if cem else K_full
    v, calls, el = timed(Ks, budget_s)
    per_call = el / calls
    # 1 thread: a K sample sized to take about the budget (assuming linear in the pool size, at most 1x
    # the pool's per-call time per thread), never below 64 candidates, never above the line's K
    K1 = int(min(Ks, max(64, Ks * budget_s / max(per_call * threads, 1e-9))))
    short = per_call * threads < 0.1 * budget_s          # (small K: many 1-thread calls, not one)
    with threadpool_limits(limits=1, user_api="blas"):
        v1, calls1, el1 = timed(K1, budget_s / 2 if short else 0.0, max_calls=(1 << 30) if short else 1)
    # the 1-thread figure replaces the pool's only when it was measured at the same K (an extrapolation from
    # a smaller K sample is kept in the record, never promoted to `value`)
    best_pool = v >= v1 or K1 < Ks
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return dict(value=v if best_pool else v1, unit="candidate-steps/s", cores=int(threads) if best_pool else 1,
                kind="port", K_sampled=Ks if best_pool else K1,
                value_pool=v, pool_threads=int(threads), K_sampled_pool=Ks,
                value_1thread=v1, K_sampled_1thread=K1, value_1thread_extrapolated=K1 < Ks, cpu_model=_cpu_model(), host_cpus=os.cpu_count(),
                affinity_cpus=aff, omp_num_threads=os.environ.get("OMP_NUM_THREADS"),
                threads_note=("value/cores = the faster of the BLAS pool and 1 thread per candidate-step, the 1-thread "
                              "figure only when sampled at the same K (value_1thread_extrapolated otherwise); the "
                              "pool size is OMP_NUM_THREADS (the GPU box's CPU share per GPU), not host_cpus"),
                sample=f"{calls} oracle get_action calls at K={Ks} (workload K={K_full}), H={H}, {net}, "
                       f"OpenBLAS {threads} threads, {el:.1f} s; 1 thread: {calls1} call(s) at K={K1}, {el1:.1f} s"
                       + (f"; CEM {cem['iterations']} iterations per call" if cem else ""))


class _Space:
    def __init__(self, n, lo=None, hi=None):
        self.shape = (n,)
        if lo is not None:
            self.low, self.high = lo, hi


class _Env:                        # HalfCheetah's spaces (cheetah_env.py:21-27; ctrlrange [-1, 1])
    observation_space = _Space(S_DIM)
    action_space = _Space(A_DIM, -np.ones(A_DIM, np.float32), np.ones(A_DIM, np.float32))


def dropin_parity_p50(K_global, H, hidden, L, act, ln, kernels, biases, ln_g, ln_b, norm, state, device, calls,
                      world):
    """p50 of the drop-in ``bc_mpc_amd.MPCcontroller.get_action`` in parity mode (rng="numpy": the
    reference's np.random.uniform draw of controllers.py:53 from the seeded global stream, the
    first action taken from that array), host state in, host action out; every rank calls it
    (K_global sharded over the ranks by the controller)."""
    import torch
    import torch.distributed as dist
    from bc_mpc_amd import MPCcontroller, cheetah_cost_fn
    from bc_mpc_amd.dynamics import NNDynamicsModel
    dyn = NNDynamicsModel(_Env(), L, hidden, act, None, norm, 512, 1, 1e-3, layer_norm=ln, device=device)
    dyn.load_weights(kernels, biases, ln_g, ln_b)
    ctrl = MPCcontroller(_Env(), dyn, horizon=H, cost_fn=cheetah_cost_fn, num_simulated_paths=K_global,
                         device=device)
    np.random.seed(0)                                  # train_mpc_ppo.py:499
    pre = prewarm(lambda i: ctrl.get_action(state), fixed_calls=20 if world > 1 else None)
    ts = []
    for _ in range(calls):
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        ctrl.get_action(state)
        ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize(device)
    p50 = float(np.median(ts))
    out = {"p50_ms": p50 * 1e3, "p90_ms": float(np.percentile(ts, 90)) * 1e3, "calls": calls,
           "cand_steps_per_s": K_global * H / p50, "K_global": K_global, "horizon": H,
           "rng": "numpy legacy MT19937 stream (np.random.seed(0)), drawn by the library",
           "mt_path": os.environ.get("BCMPC_MT_PATH", "default"), "prewarm": pre}
    ctrl._engine.close()
    return out


class _BenchPolicy:
    """A policy container for the drop-in policy controllers (bc_mpc_amd.policy.extract: policy_spec() and
    an integer version -- the weights are fixed during a control loop; the reference's TF MlpPolicy is read
    through its session instead)."""

    def __init__(self, arrays):
        from bc_mpc_amd.engine import PolicySpec
        self._spec = PolicySpec(*arrays)
        self.version = 1

    def policy_spec(self):
        return self._spec


def dropin_small_k(name, wl, prob, device, calls=200, gap_us=50.0):
    """The reference's controller for a small-K workload, driven exactly as utils.py:193-213 drives it
    (one get_action per env step; NumPy's global stream seeded, train_mpc_ppo.py:499): MPCcontroller
    (plain nets), MPCcontrollerPolicyNet (a fused policy, explore / self_exp from the workload) or
    MPCcontrollerPolicyNetReward (the reward net).  p50 back to back, and with ``gap_us`` of host work
    between calls (an env.step stand-in: the call's pre-draw of the next rows overlaps it)."""
    import torch
    from bc_mpc_amd import MPCcontroller, MPCcontrollerPolicyNet, MPCcontrollerPolicyNetReward, cheetah_cost_fn
    from bc_mpc_amd.dynamics import NNDynamicsModel, NNDynamicsRewardModel
    K, H = wl["K"], wl["H"]
    if prob["reward"]:
        dyn = NNDynamicsRewardModel(_Env(), prob["norm"], 512, 1, 1e-3, layer_norm=prob["ln"], size=wl["hidden"],
                                    device=device)
        dyn.load_weights(prob["kernels"], prob["biases"], prob["ln_g"], prob["ln_b"])
    else:
        dyn = NNDynamicsModel(_Env(), wl["L"], wl["hidden"], wl["act"], None, prob["norm"], 512, 1, 1e-3,
                              layer_norm=prob["ln"], device=device)
        dyn.load_weights(prob["kernels"], prob["biases"], prob["ln_g"], prob["ln_b"])
    stochastic = wl.get("policy_mode") == "stochastic"
    if prob["policy"] and prob["reward"]:
        ctrl = MPCcontrollerPolicyNetReward(_Env(), dyn, _BenchPolicy(prob["pol_arrays"]), explore=wl["explore"],
                                            self_exp=stochastic, horizon=H, num_simulated_paths=K, device=device)
        kind = "MPCcontrollerPolicyNetReward"
    elif prob["policy"]:
        ctrl = MPCcontrollerPolicyNet(_Env(), dyn, _BenchPolicy(prob["pol_arrays"]), explore=wl["explore"],
                                      self_exp=stochastic, horizon=H, cost_fn=cheetah_cost_fn, num_simulated_paths=K,
                                      device=device)
        kind = "MPCcontrollerPolicyNet"
    else:
        ctrl = MPCcontroller(_Env(), dyn, horizon=H, cost_fn=cheetah_cost_fn, num_simulated_paths=K, device=device)
        kind = "MPCcontroller"
    np.random.seed(0)                                  # train_mpc_ppo.py:499
    prewarm(lambda i: ctrl.get_action(prob["state"]))
    ts, tg = [], []
    for _ in range(calls):
        t0 = time.perf_counter()
        ctrl.get_action(prob["state"])
        ts.append(time.perf_counter() - t0)
    for _ in range(calls):
        t1 = time.perf_counter()
        while time.perf_counter() - t1 < gap_us * 1e-6:
            pass
        t0 = time.perf_counter()
        ctrl.get_action(prob["state"])
        tg.append(time.perf_counter() - t0)
    torch.cuda.synchronize(device)
    out = {"controller": kind, "kernel": ctrl._engine.info()["kernel"], "precision": ctrl._engine.precision,
           "p50_ms": float(np.median(ts) * 1e3), f"p50_gap{int(gap_us)}us_ms": float(np.median(tg) * 1e3)}
    ctrl._engine.close()
    return out


def synthetic_problem(wl):
    """Synthetic inputs of a workload: glorot kernels, 0.1 N biases, synthetic stats /
    state, the policy's normc kernels (random init: no checkpoints)."""
    K, H, hidden, L, act = wl["K"], wl["H"], wl["hidden"], wl["L"], wl["act"]
    reward = bool(wl.get("reward"))
    if reward:   # dense, dense_1 (delta hidden), dense_2 (delta out), dense_3 (reward hidden), dense_4 (reward out)
        shapes = [(S_DIM + A_DIM, hidden), (hidden, hidden), (hidden, S_DIM), (hidden, hidden), (hidden, 1)]
    else:
        dims = [S_DIM + A_DIM] + [hidden] * L + [S_DIM]
        shapes = list(zip(dims[:-1], dims[1:]))
    kernels, biases = [], []
    for i, (fi, fo) in enumerate(shapes):
        r = np.random.RandomState(1000 + i)
        lim = np.sqrt(6.0 / (fi + fo))
        kernels.append(r.uniform(-lim, lim, (fi, fo)).astype(np.float32))
        biases.append((0.1 * r.standard_normal(fo)).astype(np.float32))
    ln = bool(wl.get("ln"))
    ln_g, ln_b = None, None
    if ln:   # gamma ~ 1 + 0.1 N, beta ~ 0.1 N per hidden layer (reward net: trunk, delta head, reward head)
        rl = np.random.RandomState(99)
        nln = 3 if reward else L
        ln_g = [(1.0 + 0.1 * rl.standard_normal(hidden)).astype(np.float32) for _ in range(nln)]
        ln_b = [(0.1 * rl.standard_normal(hidden)).astype(np.float32) for _ in range(nln)]
    r7 = np.random.RandomState(7)
    mean_obs = 0.1 * r7.standard_normal(S_DIM)
    std_obs = np.abs(r7.standard_normal(S_DIM)) * 0.5 + 0.2
    mean_d = 0.005 * r7.standard_normal(S_DIM)
    std_d = 0.05 * (np.abs(r7.standard_normal(S_DIM)) + 0.2)
    norm = [mean_obs, std_obs, np.zeros(A_DIM), np.full(A_DIM, 1 / np.sqrt(3)), np.full(1, 0.3), np.full(1, 1.2),
            mean_obs, std_obs, mean_d, std_d]
    state = mean_obs + 0.5 * std_obs * np.random.RandomState(11).standard_normal(S_DIM)
    policy = wl.get("policy")
    pol_arrays = None
    if policy:
        ph, pl = policy
        rp = np.random.RandomState(2024)
        pdims = [S_DIM] + [ph] * pl + [A_DIM]
        pks, pbs = [], []
        for i in range(len(pdims) - 1):
            k = rp.standard_normal((pdims[i], pdims[i + 1]))
            k *= (1.0 if i < pl else 0.5) / np.sqrt(np.square(k).sum(axis=0, keepdims=True))   # normc init
            pks.append(k.astype(np.float32))
            pbs.append((0.05 * rp.standard_normal(pdims[i + 1])).astype(np.float32))
        pol_arrays = (pks, pbs, mean_obs.astype(np.float32), (std_obs + 0.05).astype(np.float32),
                      np.full(A_DIM, -0.5, np.float32))
    return dict(kernels=kernels, biases=biases, ln_g=ln_g, ln_b=ln_b, norm=norm, state=state, reward=reward, ln=ln,
                model="reward" if reward else "delta", cost="reward" if reward else "cheetah",
                gamma=float(wl.get("gamma", 1.0)), policy=policy, pol_arrays=pol_arrays)


def make_engine(wl, prob, device, precision, K=None):
    """The workload's engine; ``K``: this rank's shard size (default: the workload's K)."""
    from bc_mpc_amd.engine import MLPSpec, PolicySpec, RolloutEngine
    H, hidden, L, act = wl["H"], wl["hidden"], wl["L"], wl["act"]
    K = wl["K"] if K is None else int(K)
    if prob["policy"]:
        ph, pl = prob["policy"]
        eng = RolloutEngine(S_DIM, A_DIM, hidden, L, act, prob["ln"], H, K, device=device, policy_hidden=ph,
                            policy_layers=pl, policy_mode=wl.get("policy_mode", "explore"), cost=prob["cost"],
                            model=prob["model"], precision=precision)
        eng.set_policy(PolicySpec(*prob["pol_arrays"]), wl["explore"], 1)
    else:
        eng = RolloutEngine(S_DIM, A_DIM, hidden, L, act, prob["ln"], H, K, device=device, cost=prob["cost"],
                            model=prob["model"], precision=precision)
    eng.set_weights(MLPSpec(prob["kernels"], prob["biases"], act, prob["ln_g"], prob["ln_b"], model=prob["model"]),
                    prob["norm"], 1)
    if prob["reward"]:
        eng.set_discount(prob["gamma"])
    return eng


# the reference's own small configurations: MPCcontroller at train_mpc_ppo.py's defaults, its default MPC-aug
# controller (MPCcontrollerPolicyNet), run.sh's recipe (MPCcontrollerPolicyNetReward, LayerNorm reward net,
# stochastic policy), BASELINE cfg1
SMALL_K = ("ppo_defaults", "ppo_mpc_default", "runsh_recipe", "cfg1")


PREWARM_S = float(os.environ.get("BCMPC_BENCH_PREWARM_S", "0.25"))


def prewarm(step, ctx=None, budget_s=None, fixed_calls=None, seed_base=1 << 40):
    """Run the line's own control step for about ``budget_s`` before its warmup steps.  After idle -- process
    start, or the seconds of CPU baseline between two lines -- the GPU's clocks ramp over the first ~40 ms of
    work: at cfg3 the launches take 2.34 → 1.79 ms over the first 20 (`profiles/r06_cold_ramp.txt`), so a line
    whose few warmup steps fall inside that ramp would time its first steps at the idle clocks.  The prewarm
    calls do the same work as the timed steps (other seeds), are untimed, and are reported in the line's
    ``prewarm`` record.  With ``ctx`` (several ranks) the call count is agreed on (every step holds a
    collective); ``fixed_calls`` sets it outright."""
    import math
    import torch
    budget_s = PREWARM_S if budget_s is None else budget_s
    t0 = time.perf_counter()
    done = 0
    if fixed_calls is None:
        step(seed_base)                                # (the first call carries one-time costs: not the estimate)
        t1 = time.perf_counter()
        step(seed_base + 1)
        step(seed_base + 2)
        done = 3
        per = (time.perf_counter() - t1) / 2
        calls = max(0, int(math.ceil((budget_s - (time.perf_counter() - t0)) / max(per, 1e-6))))
        if ctx is not None:
            calls = int(ctx.allreduce(calls, "max"))
    else:
        calls = int(fixed_calls)
    for i in range(calls):
        step(seed_base + done + i)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return {"calls": done + calls, "seconds": time.perf_counter() - t0}


def pmc_traffic(key):
    """HBM bytes per launch measured by the PMC passes of this round (profiles/TRAFFIC_FILE), or None."""
    try:
        tr = json.load(open(os.path.join(REPO, "profiles", TRAFFIC_FILE))).get(key)
        return tr["hbm_bytes_per_launch"] if tr else None
    except Exception:
        return None


# what the PMC passes name as the limiter below the MFMA roofline, per line
LIMITER = {
    "cfg3": "the lock-step chain of one 64-candidate group per CU (MFMA pipe busy 0.60; profiles/r05_pmc_x3_issue.txt)",
    "cfg4_shard": "as cfg3 (same kernel, two workgroups per CU over the launch)",
    "cfg2": "the per-CU weight stream of 16-candidate groups (L1->L2 41.5 B/clk/CU at 242 cycles, MFMA busy 0.27; "
            "profiles/r05_pmc_cfg2_issue.txt)",
    "ns_shard": "the per-CU weight stream of 32-candidate groups (L1->L2 40.4 B/clk/CU at 210 cycles, MFMA busy 0.47; "
                "profiles/r06_pmc_ns_shard_issue.txt)",
    "cfg5": "the per-CU vector-memory path of the 3x1024 net's fragment stream (48 B/clk/CU, L2 hit 96.7%; "
            "profiles/r03_pmc_cfg5/summary.txt)",
    "f16": "vector issue (VALU 0.49 + MFMA 0.43 of SIMD-cycles, two transcendentals per tanh; "
           "profiles/r05_pmc_pp_issue.txt)",
}


def roofline_line(K, H, fpcs, kernel_ms, precision, iters=1, traffic_key=None, limiter=None):
    """The MFMA roofline of one launch: algorithmic FLOPs (K x H x flop_per_cand_step) / HIP-event kernel
    time, against the peak of the precision the engine computes in; ``limiter``: the LIMITER key naming what
    the counters show binding below it."""
    peak = {"fp32": FP32_MFMA_PEAK_TFLOPS, "f16": F16_MFMA_PEAK_TFLOPS}.get(precision, SPLIT_PEAK_TFLOPS)
    tf = K * H * iters * fpcs / (kernel_ms / 1e3) / 1e12
    out = {"bound": "mfma", "achieved": tf, "peak": peak, "unit": "TFLOP/s", "frac": tf / peak,
           "flop_per_launch": K * H * iters * fpcs}
    if limiter in LIMITER:
        out["limiter"] = LIMITER[limiter]
    if traffic_key:
        t = pmc_traffic(traffic_key)
        # (the PMC passes measure one rollout launch; a CEM call is `iters` of them)
        out["traffic"] = t * iters if t is not None else None
        out["traffic_source"] = f"profiles/{TRAFFIC_FILE} [{traffic_key}]" + (f" x {iters} passes" if iters > 1 else "")
    return out


def oracle_weights(prob, wl):
    from oracle import mpc_oracle as orc      # (the cpu_baseline leg only: the checker, timed on the host)
    if prob["reward"]:
        return orc.RewardMLPWeights(prob["kernels"], prob["biases"], prob["ln_g"], prob["ln_b"])
    return orc.MLPWeights(prob["kernels"], prob["biases"], wl["act"], prob["ln_g"], prob["ln_b"])


def net_label(wl, prob):
    net = (f"reward net {wl['hidden']}" if prob["reward"] else f"{wl['L']}x{wl['hidden']} {wl['act']}") + \
        (" + LN" if prob["ln"] else "") + (f" + policy {prob['policy']}" if prob["policy"] else "")
    if prob["policy"] and wl.get("policy_mode") == "stochastic":
        net += " (oracle policy in its deterministic explore branch: TF's sampler is not restatable)"
    return net


def cfg2_line(device, calls=100, warmup=10, cpu_seconds=4.0, dropin_calls=20, with_cpu=True):
    """BASELINE configs[1] (K=4096, H=20, 2x500 tanh, 1 GPU, fp32 tolerance): complete get_action p50, the
    rollout kernel's HIP-event time and roofline, the drop-in controller's p50 and the oracle on the host."""
    wl = WORKLOADS["cfg2"]
    prob = synthetic_problem(wl)
    eng = make_engine(wl, prob, device, "auto")
    pre = prewarm(lambda i: eng.get_action(prob["state"], None, seed=0xC2 + i))
    ts = []
    for i in range(warmup + calls):
        t0 = time.perf_counter()
        eng.get_action(prob["state"], None, seed=0xC2 + i)
        if i >= warmup:
            ts.append(time.perf_counter() - t0)
    eng.set_timing(True)
    ks = []
    for i in range(max(20, calls // 2)):
        eng.get_action(prob["state"], None, seed=0xC2 + i)
        ks.append(eng.last_kernel_ms()[0])
    fpcs = flop_per_cand_step(wl["hidden"], wl["L"])
    row = {"K": wl["K"], "H": wl["H"], "kernel": eng.info()["layout"], "precision": eng.precision,
           "value": wl["K"] * wl["H"] / float(np.median(ts)), "unit": "candidate-steps/s",
           "p50_ms": float(np.median(ts) * 1e3), "kernel_ms": float(np.mean(ks)),
           "roofline": roofline_line(wl["K"], wl["H"], fpcs, float(np.mean(ks)), eng.precision,
                                     traffic_key="cfg2:split:device" if eng.precision == "split" else None,
                                     limiter="cfg2"),
           "prewarm": pre}
    eng.close()
    if dropin_calls:
        d = dropin_parity_p50(wl["K"], wl["H"], wl["hidden"], wl["L"], wl["act"], False, prob["kernels"],
                              prob["biases"], None, None, prob["norm"], prob["state"], device, dropin_calls, 1)
        row["dropin_parity_p50_ms"] = d["p50_ms"]
    if with_cpu:
        row["cpu_baseline"] = cpu_baseline(oracle_weights(prob, wl), prob["norm"], prob["state"], wl["H"], cpu_seconds,
                                           wl["K"], net_label(wl, prob))
    return row


def workload_line(name, device, steps=20, warmup=3, cpu_seconds=4.0, with_cpu=True):
    """Another BASELINE config timed on this GPU as the headline is (a complete get_action per step, HIP
    events inside the timed region, precision "auto"): cfg4_shard (configs[3]'s per-GPU shard, K=32768,
    H=20: the N=1 rank of the 8-GPU weak-scaling run) and cfg5 (configs[4]: K=65536, H=50, 3x1024 tanh,
    CEM x4 on one GPU; one step = one CEMcontroller.get_action = 4 rollout passes + the device elite
    select / refit, HIP events around the whole device-side call).  The oracle on the host beside it
    (cfg5 sampled at K=1024: a full-size oracle CEM call takes minutes)."""
    wl = WORKLOADS[name]
    prob = synthetic_problem(wl)
    K, H, cem = wl["K"], wl["H"], wl.get("cem")
    iters = cem["iterations"] if cem else 1
    eng = make_engine(wl, prob, device, "auto")
    if cem:
        n_elite = max(1, int(round(cem["elite_frac"] * K)))
        mu0, sd0 = np.zeros((H, A_DIM)), np.full((H, A_DIM), 0.5)

        def call(i):
            return eng.cem_get_action(prob["state"], mu0, sd0, iters, n_elite, cem["alpha"], 0xC5 + i)[0]
    else:
        def call(i):
            return eng.get_action(prob["state"], None, seed=0xC4 + i)
    eng.set_timing(True)
    pre = prewarm(call)
    for i in range(warmup):
        call(i)
    ts, ks = [], []
    for i in range(steps):
        t0 = time.perf_counter()
        call(warmup + i)
        ts.append(time.perf_counter() - t0)
        ks.append(eng.last_kernel_ms()[0])
    fpcs = flop_per_cand_step(wl["hidden"], wl["L"])
    info = eng.info()
    prec = eng.precision
    key = f"{name}:{prec}:device"
    row = {"K": K, "H": H, "net": net_label(wl, prob), "kernel": info["layout"], "precision": prec,
           "value": K * H * iters / float(np.median(ts)), "unit": "candidate-steps/s", "steps": steps,
           "p50_ms": float(np.median(ts) * 1e3), "kernel_ms": float(np.mean(ks)),
           "roofline": roofline_line(K, H, fpcs, float(np.mean(ks)), prec, iters=iters, traffic_key=key,
                                     limiter=name),
           "prewarm": pre}
    if cem:
        row["cem"] = dict(cem, n_elite=n_elite)
        row["roofline"]["kernel_note"] = ("HIP events around the whole device-side CEM call: 4 rollout passes + "
                                          "elite select + refit + argmin")
    eng.close()
    if with_cpu:
        row["cpu_baseline"] = cpu_baseline(oracle_weights(prob, wl), prob["norm"], prob["state"], H, cpu_seconds, K,
                                           net_label(wl, prob), cem=cem)
    return row


def library_comm_line(eng, state, offset, K, H, steps, warmup, world, local, backend):
    """N > 1: the north_star's collective as the library owns it, timed beside the default line.  The same
    engine gets libbcmpc's communicator (bcmpc_comm_init over RCCL, its id bootstrapped through
    torch.distributed) attached, so every get_action ends with the device pack, ONE ncclAllGather of the
    144-byte records over xGMI and the device np.argmin select (csrc/comm.hip) -- then the same timed loop
    as the headline.  Guarded: a communicator that cannot be created (e.g. RCCL refusing two ranks on one
    GPU in a rehearsal) or an exchange that fails / times out (BCMPC_COMM_TIMEOUT_MS, 20 s here) is
    recorded, every rank agreeing on the outcome, and the bench goes on."""
    import torch
    import torch.distributed as dist
    from bc_mpc_amd import distributed as bdist
    os.environ.setdefault("BCMPC_COMM_TIMEOUT_MS", "20000")
    tdev = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")

    def agree(v, op):
        t = torch.tensor([float(v)], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=op)
        return float(t.item())

    comm, err = None, ""
    try:
        comm = bdist.LibraryComm(local)
    except Exception as ex:                            # (RCCL: "Duplicate GPU detected" on one card)
        err = str(ex)
    if agree(1.0 if comm is not None else 0.0, dist.ReduceOp.MIN) < 1.0:
        if comm is not None:
            comm.close()
        return {"status": "init-failed", "error": err or "another rank's bcmpc_comm_init failed"}
    status, ts, el = "ok", [], float("nan")
    eng.set_comm(comm)
    try:
        for i in range(warmup):
            eng.get_action(state, None, seed=0xC0 + i, cand_offset=offset)
        dist.barrier()
        torch.cuda.synchronize(local)
        t0 = time.perf_counter()
        for i in range(steps):
            t1 = time.perf_counter()
            eng.get_action(state, None, seed=0xC0 + warmup + i, cand_offset=offset)
            ts.append(time.perf_counter() - t1)
        torch.cuda.synchronize(local)
        el = time.perf_counter() - t0
    except Exception as ex:
        status, err = "exchange-failed", str(ex)
    finally:
        eng.set_comm(None)
        comm.close()
    if agree(1.0 if status == "ok" else 0.0, dist.ReduceOp.MIN) < 1.0:
        return {"status": "exchange-failed", "error": err or "another rank's exchange failed"}
    dist.barrier()
    el = agree(el, dist.ReduceOp.MAX)
    return {"status": "ok", "value": K * world * H * steps / el, "unit": "candidate-steps/s",
            "ms_per_step": el / steps * 1e3, "p50_ms": float(np.median(ts) * 1e3),
            "collective": "libbcmpc RCCL all-gather of the 144-byte result records + device np.argmin select, "
                          "in get_action (bcmpc_engine_set_comm)"}


def small_k_lines(device, calls=200, warmup=20, cpu_seconds=3.0, with_cpu=True):
    """get_action p50 (host state in, device-drawn actions, host result out) and the rollout kernel's
    HIP-event time for the small-K workloads the reference actually runs (train_mpc_ppo.py:71,77: K=400;
    run.sh:27-31; BASELINE cfg1), with the auto kernel (the team kernel, rollout_team.hip) and with the
    kernel it replaced (BCMPC_TEAM=0: the split slab kernel, or for the nets only the team kernel takes in
    split precision -- a policy over relu + LN, the LayerNorm reward net -- the fp32 group kernel), on
    this process's GPU."""
    out = {}
    for name in SMALL_K:
        wl = WORKLOADS[name]
        prob = synthetic_problem(wl)
        row = {"K": wl["K"], "H": wl["H"]}
        for tag, team in (("", None), ("slab_", "0")):
            old = os.environ.get("BCMPC_TEAM")
            if team is not None:
                os.environ["BCMPC_TEAM"] = team
            try:
                eng = make_engine(wl, prob, device, "auto")
            finally:
                if team is not None:
                    if old is None:
                        os.environ.pop("BCMPC_TEAM", None)
                    else:
                        os.environ["BCMPC_TEAM"] = old
            # p50 of the product path (no event markers: bcmpc_engine_set_timing off, its default), then
            # the kernel's HIP-event time over a second, timed pass
            prewarm(lambda i: eng.get_action(prob["state"], None, seed=0x5EED + i))
            ts, ks = [], []
            for i in range(warmup + calls):
                t0 = time.perf_counter()
                eng.get_action(prob["state"], None, seed=0x5EED + i)
                if i >= warmup:
                    ts.append(time.perf_counter() - t0)
            eng.set_timing(True)
            for i in range(max(20, calls // 4)):
                eng.get_action(prob["state"], None, seed=0x5EED + i)
                ks.append(eng.last_kernel_ms()[0])
            row[tag + "kernel"] = eng.info()["kernel"]
            row[tag + "precision"] = eng.precision
            row[tag + "p50_ms"] = float(np.percentile(ts, 50) * 1e3)
            row[tag + "kernel_ms"] = float(np.mean(ks))
            eng.close()
        row["speedup_p50"] = row["slab_p50_ms"] / row["p50_ms"]
        fpcs = flop_per_cand_step(wl["hidden"], wl["L"], policy=prob["policy"], reward=prob["reward"])
        row["roofline"] = roofline_line(wl["K"], wl["H"], fpcs, row["kernel_ms"], row["precision"])
        row["roofline"]["note"] = ("small K is latency-bound by design (a few dozen 16-candidate columns on "
                                   "256 CUs); the line's figure of merit is p50")
        # the drop-in controller in parity mode (NumPy's stream, controllers.py:53 / :191 / :310)
        d = dropin_small_k(name, wl, prob, device)
        row["dropin_controller"] = d["controller"]
        row["dropin_parity_p50_ms"] = d["p50_ms"]
        row["dropin_parity_p50_gap50us_ms"] = d["p50_gap50us_ms"]
        if with_cpu:
            # the reference's own configuration on the host: the oracle (NumPy restatement) at this full K
            row["cpu_baseline"] = cpu_baseline(oracle_weights(prob, wl), prob["norm"], prob["state"], wl["H"],
                                               cpu_seconds, wl["K"], net_label(wl, prob), prob["pol_arrays"],
                                               wl.get("explore", 0.5), prob["gamma"], None)
            row["cpu_baseline"]["p50_ms_per_get_action"] = wl["K"] * wl["H"] / row["cpu_baseline"]["value"] * 1e3
        out[name] = row
    return out


def f16_line(wl, prob, device, steps=50, warmup=5, name="cfg3"):
    """BASELINE configs[2] as it is worded ("bf16 MFMA GEMM + fp32 cost accumulate"): the same complete
    get_action with the single-pass f16 engine (precision "f16"; f16's 11-bit significand,
    f32 accumulate, f64 state and cost).  Not `value`: its costs meet the f16 bar of tests/test_gpu_f16.py,
    not the fp32 tolerance.  Roofline against the f16 dense MFMA peak (one pass per product)."""
    K, H = wl["K"], wl["H"]
    eng = make_engine(wl, prob, device, "f16")
    eng.set_timing(True)
    pre = prewarm(lambda i: eng.get_action(prob["state"], None, seed=0xF16 + i))
    for i in range(warmup):
        eng.get_action(prob["state"], None, seed=0xF16 + i)
    ts, ks = [], []
    for i in range(steps):
        t0 = time.perf_counter()
        eng.get_action(prob["state"], None, seed=0xF16 + warmup + i)
        ts.append(time.perf_counter() - t0)
        ks.append(eng.last_kernel_ms()[0])
    kern = eng.info()["kernel"]
    layout_name = eng.info()["layout"]
    # argmin agreement with the f32-grade split engine (within the fp32 envelope of the oracle:
    # tests/test_gpu_parity.py; against the oracle itself: tests/test_gpu_f16.py) over 16 seeds
    split = make_engine(wl, prob, device, "split")
    agree, regret = 0, []
    for sd in range(1, 17):
        rf = eng.get_action(prob["state"], None, seed=sd)
        rs = split.get_action(prob["state"], None, seed=sd, return_costs=True)
        agree += int(rf.best_index == rs.best_index)
        regret.append(float(rs.costs[rf.best_index] - rs.best_cost))
    split.close()
    eng.close()
    fpcs = flop_per_cand_step(wl["hidden"], wl["L"])
    tf = K * H * fpcs / (float(np.mean(ks)) / 1e3) / 1e12
    # the layout capi.cpp picks for this shape (the pipelined kernel at >= 2048 columns, BCMPC_F16_PP=0 off)
    pp = (os.environ.get("BCMPC_F16_PP", "") != "0" and not os.environ.get("BCMPC_F16_NC")
          and not os.environ.get("BCMPC_F16_NW") and wl["hidden"] in range(497, 513) and wl["L"] == 2
          and wl.get("act", "tanh") == "tanh" and K >= 2048 * 16)
    layout = (f"{layout_name} (two 64-candidate groups per workgroup, software-pipelined)" if pp
              else f"{layout_name} single-pass")
    traffic = None
    try:
        tr = json.load(open(os.path.join(REPO, "profiles", TRAFFIC_FILE))).get(f"{name}:f16:device")
        traffic = tr["hbm_bytes_per_launch"] if tr and pp else None
    except Exception:
        pass
    return {"precision": "f16 (one v_mfma_f32_16x16x32_f16 pass, f32 accumulate; f64 state / cost)",
            "kernel": kern, "layout": layout, "value": K * H / float(np.mean(ts)), "unit": "candidate-steps/s",
            "p50_ms": float(np.percentile(ts, 50) * 1e3), "kernel_ms_avg": float(np.mean(ks)),
            "roofline": {"bound": "mfma", "achieved": tf, "peak": F16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": tf / F16_MFMA_PEAK_TFLOPS, "traffic": traffic, "limiter": LIMITER["f16"],
                         "traffic_source": f"profiles/{TRAFFIC_FILE}"},
            "prewarm": pre,
            "argmin_agreement": {"seeds": 16, "top1_equal": agree,
                                 "reference": "the split (f32-grade) engine's argmin on the same actions",
                                 "regret_median": float(np.median(regret)), "regret_max": float(np.max(regret)),
                                 "regret_unit": "split-engine cost of the f16 choice minus its minimum"}}


def launch_plan(gpus, environ):
    """How this invocation gets its ranks (the driver's ``--gpus N`` contract):

    * ``"ranks"``  -- WORLD_SIZE is set (torch.distributed.run started this process): it must equal
      ``--gpus`` (a mismatch exits non-zero before anything is measured);
    * ``"single"`` -- ``--gpus 1`` and no WORLD_SIZE: one rank, no process group;
    * ``"spawn"``  -- ``--gpus N > 1`` and no WORLD_SIZE: this process starts the N ranks itself as a
      child ``torch.distributed.run`` (127.0.0.1, a free port) before it touches the GPU, waits for it
      and exits with its status (never an exec of this process)."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {gpus})")
    ws = environ.get("WORLD_SIZE", "")
    if ws != "":
        if int(ws) != gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={ws} but --gpus {gpus}: the launcher and the flag disagree")
        return "ranks"
    return "single" if gpus == 1 else "spawn"


def spawn_command(n, argv, port):
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def spawn_ranks(n, argv):
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, BCMPC_BENCH_LAUNCHER="bench.py --gpus (child torch.distributed.run)")
    return subprocess.run(spawn_command(n, argv, port), env=env).returncode


def workload_shard(K_wl, rank, world, scaling):
    """This rank's contiguous global candidate range (lo, hi) and the global K.
    strong: the workload's K is the GLOBAL K, split as distributed.shard_range splits it (the first K % N
    ranks one more; the north_star point: K = 65,536 over N GPUs); weak: every rank owns K_wl candidates
    of its own (global N * K_wl)."""
    if scaling == "weak":
        return rank * K_wl, (rank + 1) * K_wl, K_wl * world
    base, rem = divmod(int(K_wl), int(world))
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0), int(K_wl)


class RankCtx:
    """One rank's view: world / rank / device, the process group's backend, and the two primitives the
    timed loops need (barrier; max over ranks)."""

    def __init__(self, world, rank, local, backend):
        import torch
        self.world, self.rank, self.local, self.backend = world, rank, local, backend
        self.dev = torch.device("cuda", local)

    def barrier(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier()

    def allreduce(self, v, op="max"):
        if self.world == 1:
            return float(v)
        import torch
        import torch.distributed as dist
        t = torch.tensor([float(v)], dtype=torch.float64, device=self.dev if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op={"max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op])
        return float(t.item())

    def ranks(self):
        if self.world == 1:
            return 1
        import torch.distributed as dist
        return dist.get_world_size()


def timed_loop(ctx, step, steps, warmup, kernel_ms=None):
    """W untimed steps, then EXACTLY ``steps`` steps bracketed by a barrier + device synchronisation on
    both sides; the wall time is the max over ranks.  ``kernel_ms``: read after each step (HIP events of
    the rollout launch on its stream)."""
    import torch
    for i in range(warmup):
        step(i)
    ctx.barrier()
    torch.cuda.synchronize(ctx.dev)
    ts, ks = [], []
    t0 = time.perf_counter()
    for i in range(steps):
        t1 = time.perf_counter()
        step(warmup + i)
        ts.append(time.perf_counter() - t1)
        if kernel_ms is not None:
            ks.append(kernel_ms())
    torch.cuda.synchronize(ctx.dev)
    ctx.barrier()
    elapsed = ctx.allreduce(time.perf_counter() - t0, "max")
    return elapsed, ts, ks


def rollout_stepper(ctx, eng, state, lo, maximize, lib_comm=None):
    """One complete control step of a plain random-shooting workload on this rank's shard [lo, lo + K):
    1 rank -- bcmpc_get_action (state in the kernel arguments, in-kernel Philox actions, rollout + argmin,
    the result in mapped host memory, one synchronisation); N ranks -- the state H2D, bcmpc_rollout_async
    (result record on the device), then distributed.RecordExchange: one torch all-gather of the 144-byte
    records (RCCL over xGMI) + the library's device select + one D2H (or, with the library communicator
    attached -- BCMPC_LIBRARY_COMM=1 -- bcmpc_get_action with the exchange inside the library).
    Returns (step(i) -> (cost, index, first_action), carrier description)."""
    import torch
    if ctx.world == 1 or lib_comm is not None:
        def step(i):
            res = eng.get_action(state, None, seed=0xB0B + i, cand_offset=lo)
            return res.best_cost, res.best_index, res.first_action
        return step, ("none (1 rank)" if ctx.world == 1 else
                      "libbcmpc RCCL all-gather of the 144-byte result records + device np.argmin select, in "
                      "get_action (bcmpc_engine_set_comm)")
    from bc_mpc_amd import distributed as bdist
    ex = bdist.RecordExchange(ctx.local, maximize=maximize)
    h_state = torch.zeros(len(state), dtype=torch.float64).pin_memory()
    hs = h_state.numpy()
    d_state = torch.zeros(len(state), dtype=torch.float64, device=ctx.dev)
    d_costs = torch.empty(max(1, eng.num_paths), dtype=torch.float64, device=ctx.dev)
    stream = torch.cuda.current_stream(ctx.dev)

    def step(i):
        np.copyto(hs, state)
        with torch.cuda.stream(stream):
            d_state.copy_(h_state, non_blocking=True)
        eng.rollout_async(d_state.data_ptr(), 0, None, 0xB0B + i, lo, d_costs.data_ptr(), None,
                          ex.d_result.data_ptr(), stream.cuda_stream)
        return ex.exchange(stream)
    carrier = (f"torch {ctx.backend} all_gather_into_tensor of the 144-byte bcmpc_result records "
               f"({'RCCL over xGMI' if ctx.backend == 'nccl' else 'host memory'}) + bcmpc_select_results_async "
               "(device np.argmin select) + one D2H (distributed.RecordExchange)")
    return step, carrier


def cem_stepper(ctx, eng, wl, prob, lo, hi, K_global):
    """One CEMcontroller.get_action (cfg5): 1 rank -- bcmpc_cem_get_action (all iterations on the device);
    N ranks -- cem.cem_multi_rank over this rank's shard (per iteration one all-gather of the local top-E
    records, then the same global elite select + refit on every rank; one final min-loc)."""
    import torch
    from bc_mpc_amd.cem import cem_multi_rank
    cem = wl["cem"]
    H = wl["H"]
    iters = cem["iterations"]
    n_elite = max(1, int(round(cem["elite_frac"] * K_global)))
    mu0, sd0 = np.zeros((H, A_DIM)), np.full((H, A_DIM), 0.5)
    stream = torch.cuda.current_stream(ctx.dev)

    class _Shard:                                       # cem._EngineShard around this engine
        device = ctx.dev

        def rollout(self, d_state, d_mu, d_sigma, seed, it, lo_, k_global, d_costs, d_res, merge):
            eng.cem_rollout_async(d_state.data_ptr(), d_mu.data_ptr(), d_sigma.data_ptr(), seed, it, lo_,
                                  k_global, d_costs.data_ptr(), d_res.data_ptr(), merge, stream.cuda_stream)

        def check_status(self):
            eng.check_status()

        def select(self, d_pairs, d_costs, m, index_base, n, d_out, d_count):
            eng.select_async(d_pairs.data_ptr() if d_pairs is not None else None,
                             d_costs.data_ptr() if d_costs is not None else None, m, index_base, n,
                             d_out.data_ptr(), d_count.data_ptr(), stream.cuda_stream)

        def refit(self, d_elite, d_count, seed, it, alpha, d_mu, d_sigma):
            eng.cem_refit_async(d_elite.data_ptr(), d_count.data_ptr(), seed, it, alpha, d_mu.data_ptr(),
                                d_sigma.data_ptr(), stream.cuda_stream)

    def step(i):
        if ctx.world == 1:
            res, _, _ = eng.cem_get_action(prob["state"], mu0, sd0, iters, n_elite, cem["alpha"], 0xB0B + i)
            return res.best_cost, res.best_index, res.first_action
        return cem_multi_rank(_Shard(), prob["state"], mu0, sd0, iters, n_elite, cem["alpha"], 0xB0B + i, lo, hi,
                              K_global, A_DIM, prob["reward"])[:3]
    carrier = ("none (1 rank)" if ctx.world == 1 else
               f"torch {ctx.backend} all_gather of the local top-{n_elite} (cost, index) records per CEM iteration "
               "+ one final min-loc all-gather")
    return step, n_elite, carrier


def scale_line(ctx, name, K_global, steps, warmup, precision="auto", scaling="strong"):
    """A BASELINE config at this run's N (every rank takes part; rank 0 keeps the record): the global K split
    over the ranks (strong) or K per rank (weak), the same timed loop as the headline, value = the
    candidate-steps ALL ranks processed / the max-over-ranks wall time."""
    wl = dict(WORKLOADS[name], K=K_global)
    prob = synthetic_problem(wl)
    lo, hi, Kg = workload_shard(K_global, ctx.rank, ctx.world, scaling)
    eng = make_engine(wl, prob, ctx.local, precision, K=hi - lo)
    eng.set_timing(True)
    cem = wl.get("cem")
    iters = cem["iterations"] if cem else 1
    if cem:
        step, n_elite, carrier = cem_stepper(ctx, eng, wl, prob, lo, hi, Kg)
        kms = (lambda: eng.last_kernel_ms()[0]) if ctx.world == 1 else None
    else:
        step, carrier = rollout_stepper(ctx, eng, prob["state"], lo, prob["reward"])
        kms = lambda: eng.last_kernel_ms()[0]          # noqa: E731
    pre = prewarm(step, ctx)
    el, ts, ks = timed_loop(ctx, step, steps, warmup, kms)
    H = wl["H"]
    fpcs = flop_per_cand_step(wl["hidden"], wl["L"])
    # (multi-rank CEM: the HIP events see one pass at a time; the per-rank device share is the step's wall)
    kern = float(np.mean(ks)) if ks else float(np.median(ts) * 1e3)
    kern = ctx.allreduce(kern, "max")
    row = {"K_global": Kg, "K_per_gpu": hi - lo, "H": H, "scaling": scaling, "ranks": ctx.ranks(),
           "value": Kg * H * iters * steps / el, "unit": "candidate-steps/s", "steps": steps,
           "ms_per_step": el / steps * 1e3, "p50_ms": float(np.median(ts) * 1e3),
           "kernel": eng.info()["layout"], "precision": eng.precision,
           "kernel_ms": kern, "collective": carrier,
           "roofline": roofline_line(hi - lo, H, fpcs, kern, eng.precision, iters=iters), "prewarm": pre}
    row["roofline"]["per"] = "the slowest rank's shard launch (max over ranks)"
    if cem:
        row["cem"] = dict(cem, n_elite=n_elite)
    eng.close()
    return row


def exchange_cost(device, K=8192, H=20, calls=200, warmup=20, n_rec=8):
    """The N > 1 exchange's cost on ONE card at the north_star shard (K = 8192 per GPU of K = 65,536 over 8,
    H = 20, 2x500 tanh), the wire itself excepted (one GPU cannot all-gather with itself; the 144-byte
    all-gather over xGMI is the part SCALE measures): per control step p50, for
    * ``get_action``: the 1-rank step (bcmpc_get_action, result in mapped host memory);
    * ``host_staged``: the controller's default N > 1 tail (distributed.allgather_minloc): the result on
      the host, its record up to the device, ``n_rec`` records back down (the gathered buffer's D2H) and
      the host select (bcmpc_select_results);
    * ``device_select``: the bench's N > 1 tail (distributed.RecordExchange): state H2D, rollout_async with
      the record on the device, the ``n_rec`` records (a device copy standing in for the gather) reduced by
      bcmpc_select_results_async, one D2H.
    The overheads are the p50 differences to ``get_action``."""
    import ctypes
    import torch
    from bc_mpc_amd import _lib
    from bc_mpc_amd import distributed as bdist
    wl = dict(WORKLOADS["ns_shard"], K=K, H=H)
    prob = synthetic_problem(wl)
    state = prob["state"]
    eng = make_engine(wl, prob, device, "auto")
    dev = torch.device("cuda", device)
    stream = torch.cuda.current_stream(dev)
    lib = _lib.load()
    nb = ctypes.sizeof(_lib.Result)

    def p50(fn):
        for i in range(warmup):
            fn(i)
        ts = []
        for i in range(calls):
            t0 = time.perf_counter()
            fn(warmup + i)
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts) * 1e3)

    def ga(i):
        return eng.get_action(state, None, seed=0xE0 + i)

    n = 3 + A_DIM
    h_rec = torch.zeros(n, dtype=torch.float64).pin_memory()
    d_rec = torch.zeros(n, dtype=torch.float64, device=dev)
    d_out = torch.zeros(n_rec * n, dtype=torch.float64, device=dev)
    h_out = torch.zeros(n_rec * n, dtype=torch.float64).pin_memory()

    def host_staged(i):
        # (distributed.allgather_minloc's tail, its pinned staging buffers and vectorised select; a device
        #  copy of the record into n_rec slots stands in for the all-gather)
        r = eng.get_action(state, None, seed=0xE0 + i)
        rec = h_rec.numpy()
        rec[0], rec[1], rec[2], rec[3:] = 1.0, r.best_cost, float(r.best_index), r.first_action
        d_rec.copy_(h_rec, non_blocking=True)
        d_out.view(n_rec, n).copy_(d_rec.view(1, n).expand(n_rec, n))
        h_out.copy_(d_out, non_blocking=True)
        stream.synchronize()
        return bdist.select(h_out.numpy().reshape(n_rec, n))

    d_state = torch.zeros(S_DIM, dtype=torch.float64, device=dev)
    h_state = torch.zeros(S_DIM, dtype=torch.float64).pin_memory()
    d_costs = torch.empty(K, dtype=torch.float64, device=dev)
    d_res = torch.zeros(nb, dtype=torch.uint8, device=dev)
    d_all = torch.zeros(n_rec * nb, dtype=torch.uint8, device=dev)
    d_best = torch.zeros(nb, dtype=torch.uint8, device=dev)
    h_best = torch.zeros(nb, dtype=torch.uint8).pin_memory()

    def device_select(i):
        np.copyto(h_state.numpy(), state)
        d_state.copy_(h_state, non_blocking=True)
        eng.rollout_async(d_state.data_ptr(), 0, None, 0xE0 + i, 0, d_costs.data_ptr(), None, d_res.data_ptr(),
                          stream.cuda_stream)
        d_all.view(n_rec, nb).copy_(d_res.view(1, nb).expand(n_rec, nb))
        _lib.check(lib.bcmpc_select_results_async(ctypes.c_void_p(d_all.data_ptr()), n_rec, 0,
                                                  ctypes.c_void_p(d_best.data_ptr()),
                                                  ctypes.c_void_p(stream.cuda_stream)))
        h_best.copy_(d_best, non_blocking=True)
        stream.synchronize()
        return int(h_best.numpy()[:8].view(np.int64)[0])

    # the three tails pick the same winner
    assert device_select(7) == ga(7).best_index == int(host_staged(7)[2])
    prewarm(ga)
    out = {"K": K, "H": H, "records": n_rec, "get_action_p50_ms": p50(ga), "host_staged_p50_ms": p50(host_staged),
           "device_select_p50_ms": p50(device_select), "calls": calls}
    out["host_staged_overhead_us"] = (out["host_staged_p50_ms"] - out["get_action_p50_ms"]) * 1e3
    out["device_select_overhead_us"] = (out["device_select_p50_ms"] - out["get_action_p50_ms"]) * 1e3
    out["note"] = ("one card: the all-gather's wire time is not included (SCALE's N > 1 lines carry it); "
                   "host_staged = distributed.allgather_minloc's tail, device_select = distributed.RecordExchange")
    eng.close()
    return out


def summary_of(out):
    """value / p50_ms / roofline.frac of every line, compact, printed LAST in the JSON line so the driver's
    stdout tail keeps it."""
    def pick(d):
        if not isinstance(d, dict):
            return None
        r = {k: d[k] for k in ("value", "p50_ms", "ms_per_step") if isinstance(d.get(k), (int, float))}
        if isinstance(d.get("roofline"), dict) and "frac" in d["roofline"]:
            r["frac"] = round(float(d["roofline"]["frac"]), 4)
        for k in ("value", "p50_ms", "ms_per_step"):
            if k in r:
                r[k] = float(f"{r[k]:.4g}")
        return r or None
    s = {"headline": pick(out)}
    for key in ("cfg2", "ns_shard", "cfg4_shard", "cfg5", "f16_single_pass"):
        if out.get(key):
            s[key] = pick(out[key])
    for key, row in (out.get("scale") or {}).items():
        s["scale." + key] = pick(row)
    for key, row in (out.get("small_k") or {}).items():
        s["small_k." + key] = pick(row)
    if out.get("library_comm"):
        s["library_comm"] = pick(out["library_comm"]) or out["library_comm"].get("status")
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without WORLD_SIZE, N > 1 starts the N ranks itself")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="cfg3", choices=sorted(WORKLOADS))
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong (default): the workload's K is the GLOBAL K split over the ranks (cfg3: the "
                         "north_star point, K=65536 over N GPUs); weak: K per rank")
    ap.add_argument("--actions", default="device", choices=["hbm", "device"],
                    help="device: a complete get_action with in-kernel Philox actions (host state in, host result "
                         "out); hbm: the rollout alone on a [H,K,A] f64 action array resident in HBM (A/B)")
    ap.add_argument("--dropin-calls", type=int, default=20,
                    help="MPCcontroller.get_action calls (rng='numpy', the reference's draw) timed for "
                         "dropin_parity_p50_ms (0: skip)")
    ap.add_argument("--precision", default=os.environ.get("BCMPC_PRECISION", "auto"), choices=["auto", "fp32", "split", "f16"],
                    help="fp32: f32 MFMA (rollout_grp); split: f32-accurate hi/lo f16 MFMA (rollout_x3, tanh "
                         "NNDynamicsModel without LayerNorm; with a fused policy: hidden 449..1024); auto: split "
                         "where it applies, else fp32")
    ap.add_argument("--no-f16", action="store_true",
                    help="skip the f16_single_pass line (BASELINE cfg3's bf16-class GEMM on the f16 engine)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cfg2", action="store_true", help="skip the cfg2 line (BASELINE configs[1], K=4096)")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the ns_shard, cfg4_shard and cfg5 lines (the north_star's and configs[3]'s per-GPU "
                         "shards, configs[4] on 1 GPU)")
    ap.add_argument("--no-scale", action="store_true",
                    help="skip the `scale` lines (cfg4 at K_global=262144, cfg5 at K_global=65536, cfg3 weak) "
                         "that every N measures over all its ranks")
    ap.add_argument("--no-small-k", action="store_true",
                    help="skip the small-K get_action lines (ppo_defaults, runsh_recipe, cfg1: team vs slab kernel)")
    args = ap.parse_args()

    plan = launch_plan(args.gpus, os.environ)
    if plan == "spawn":                                # before any GPU call: N ranks in a child launcher
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (N ranks on one GPU): BCMPC_DIST_BACKEND=gloo BCMPC_BENCH_DEVICE=0
    backend = os.environ.get("BCMPC_DIST_BACKEND", "nccl")
    if "BCMPC_BENCH_DEVICE" not in os.environ and local >= torch.cuda.device_count():
        raise SystemExit(f"bench.py: rank {rank} needs GPU {local} but {torch.cuda.device_count()} are visible "
                         f"(one rank per GPU; a rehearsal on one card sets BCMPC_BENCH_DEVICE=0 and "
                         f"BCMPC_DIST_BACKEND=gloo)")
    local = int(os.environ.get("BCMPC_BENCH_DEVICE", local))
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    ctx = RankCtx(world, rank, local, backend)

    from bc_mpc_amd import distributed as bdist

    wl = WORKLOADS[args.workload]
    H, hidden, L, act = wl["H"], wl["hidden"], wl["L"], wl["act"]
    lo, hi, K_global = workload_shard(wl["K"], rank, world, args.scaling)
    K = hi - lo                                        # this rank's shard (precision "auto": engine.py's rule)

    prob = synthetic_problem(wl)
    kernels, biases, ln_g, ln_b, norm, state = (prob[k] for k in ("kernels", "biases", "ln_g", "ln_b", "norm", "state"))
    reward, ln, gamma, policy, pol_arrays = (prob[k] for k in ("reward", "ln", "gamma", "policy", "pol_arrays"))
    eng = make_engine(wl, prob, local, args.precision, K=K)
    eng.set_timing(True)                               # the roofline's HIP events inside the timed region
    info = eng.info()
    kernel_name = {"solo": "rollout_fp32", "group4": "rollout_grp<NW=4>",
                   "group8": "rollout_grp<NW=8>", "split1": "rollout_x3<NC=1>", "split2": "rollout_x3<NC=2>",
                   "split4": "rollout_x3<NC=4>",
                   "team": "rollout_team (weights in registers, one column per team of workgroups)"}.get(
        info["kernel"], info["kernel"]) + f" (hidden padded {info['hidden_padded']}, {act})"
    if info["layout"].startswith("rollout_pp"):
        kernel_name = info["layout"] + f" (hidden padded {info['hidden_padded']}, {act})"
    lib_comm = None
    if (world > 1 and backend == "nccl" and not wl.get("cem") and args.actions == "device"
            and os.environ.get("BCMPC_LIBRARY_COMM", "0") == "1"):
        # opt-in (BCMPC_LIBRARY_COMM=1): the library's own communicator -- get_action all-gathers the ranks'
        # result records over RCCL and selects on the device (csrc/comm.hip); torch.distributed only carried
        # its RCCL id.  Default: distributed.RecordExchange (torch all-gather + device select)
        lib_comm = bdist.LibraryComm(local)
        eng.set_comm(lib_comm)
    cem = wl.get("cem")
    iters = cem["iterations"] if cem else 1
    n_elite = None
    if cem:
        step, n_elite, carrier = cem_stepper(ctx, eng, wl, prob, lo, hi, K_global)
    elif args.actions == "device":
        step, carrier = rollout_stepper(ctx, eng, state, lo, reward, lib_comm)
    else:
        # A/B: the rollout alone on a resident [H, K, A] f64 action array, the exchange as above
        d_state = torch.from_numpy(state).to(dev)
        host = np.random.RandomState(1234 + rank).uniform(-1, 1, (H, K, A_DIM))
        d_actions = torch.from_numpy(host).to(dev)
        del host
        d_costs = torch.empty(K, dtype=torch.float64, device=dev)
        ex = bdist.RecordExchange(local, maximize=reward)
        stream = torch.cuda.current_stream(dev)

        def step(i):
            eng.rollout_async(d_state.data_ptr(), 0, d_actions.data_ptr(), 0xB0B + i, lo, d_costs.data_ptr(), None,
                              ex.d_result.data_ptr(), stream.cuda_stream)
            return ex.exchange(stream)
        carrier = "none (1 rank)" if world == 1 else f"torch {backend} all-gather + device select"

    kms = (lambda: eng.last_kernel_ms()[0]) if not (cem and world > 1) else None
    pre = prewarm(step, ctx)                           # (untimed: the GPU's clock ramp after idle, see prewarm)
    elapsed, step_s, kern_ms = timed_loop(ctx, step, args.steps, args.warmup, kms)

    scale = None
    if not args.no_scale and args.workload == "cfg3" and args.scaling == "strong":
        # BASELINE's global configs at this N (every rank takes part): configs[3] K=262144, configs[4]
        # K=65536 CEM x4, and cfg3 weak-scaled (65536 per GPU; at N=1 the headline itself)
        scale = {"cfg4": scale_line(ctx, "cfg4_shard", 262144, steps=10, warmup=2),
                 "cfg5": scale_line(ctx, "cfg5", 65536, steps=3, warmup=1)}
        scale["cfg3_weak"] = (scale_line(ctx, "cfg3", 65536, steps=20, warmup=3, scaling="weak") if world > 1 else
                              "= the headline (N=1)")

    lib_line = None
    if world > 1 and lib_comm is None and not cem and args.actions == "device":
        lib_line = library_comm_line(eng, state, lo, K, H, args.steps, args.warmup, world, local, backend)

    dropin = None
    if args.dropin_calls > 0 and not (cem or policy or reward):
        dropin = dropin_parity_p50(K_global, H, hidden, L, act, ln, kernels, biases, ln_g, ln_b, norm, state,
                                   local, args.dropin_calls, world)

    value = K_global * H * iters * args.steps / elapsed
    fpcs = flop_per_cand_step(hidden, L, policy=policy, reward=reward)
    if cem and world > 1:                              # per-launch device time: the wall-clock share
        kern_ms = [t * 1e3 for t in step_s]
    kern_avg_s = ctx.allreduce(float(np.mean(kern_ms)), "max") / 1e3
    peak = {"fp32": FP32_MFMA_PEAK_TFLOPS, "f16": F16_MFMA_PEAK_TFLOPS}.get(eng.precision, SPLIT_PEAK_TFLOPS)
    achieved_tflops = K * H * iters * fpcs / kern_avg_s / 1e12
    ns = args.workload == "cfg3" and args.scaling == "strong"
    out = {
        "metric": "candidate-steps/sec (K x H per get_action), HalfCheetah dims",
        # CEM workloads count every iteration's K x H candidate-steps (iterations x K x H per get_action)
        "value": value,
        "unit": "candidate-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": {"fp32": "f32", "f16": "f16 (one MFMA pass, f32 accumulate; not the fp32 tolerance)"}.get(
            eng.precision, "f32 (hi/lo f16 split operands, 3 MFMA passes, f32 accumulate)"),
        "data": f"synthetic (HalfCheetah dims s=20,a=6; random-init {'two-head reward net' if reward else 'dynamics MLP'}; "
                f"actions {'resident in HBM as [H,K,6] f64, rollout only' if args.actions == 'hbm' else 'drawn in-kernel (Philox); step = complete get_action, host state in, host result out'})",
        "config": {"workload": ("north_star: " if ns else "") + f"{args.workload}: K_global={K_global} "
                               + (f"({K} per GPU)" if args.scaling == "weak" else f"over {world} GPU(s), {K} on rank 0")
                               + f", H={H}, "
                               + (f"reward net {hidden} trunk + 2x{hidden} heads tanh, argmax sum r*{gamma}^h"
                                  if reward else f"{L}x{hidden} {act}" + (" + LayerNorm" if ln else ""))
                               + (f" + fused policy {policy[1]}x{policy[0]} tanh "
                                  f"({wl.get('policy_mode', 'explore')})" if policy else "")
                               + (f" + CEM {iters} iterations, {n_elite} elites, alpha {cem['alpha']}" if cem else "")
                               + {"fp32": ", fp32 MFMA", "f16": ", single-pass f16 MFMA"}.get(
                                   eng.precision, ", split-f16 MFMA (f32-accurate)")
                               + (f", {world} ranks: 1 all-gather min-loc per step"
                                  + (" (+1 all-gather of the local top-E per CEM iteration)" if cem else "")
                                  if world > 1 else ", 1 GPU (no collective)"),
                   "K_per_gpu": K, "K_global": K_global, "horizon": H, "hidden": hidden, "n_layers": L,
                   "activation": act, "actions": args.actions, "parallelism": f"candidate-shard x{world}",
                   "ranks": ctx.ranks(), "launcher": os.environ.get("BCMPC_BENCH_LAUNCHER", "external" if world > 1
                                                                    else "none (1 rank)"),
                   "collective": carrier},
        "p50_ms": float(np.percentile(step_s, 50) * 1e3),
        "dropin_parity_p50_ms": dropin["p50_ms"] if dropin else None,
        "dropin_parity": dropin if dropin else "n/a (MPCcontroller drop-in is timed for the plain delta-net "
                                                "workloads; policy / reward / CEM controllers: tools/bench_dropin.py)",
        "p90_ms": float(np.percentile(step_s, 90) * 1e3),
        "kernel_ms_avg": kern_avg_s * 1e3,
        "roofline": {"bound": "mfma", "achieved": achieved_tflops, "peak": peak,
                     "unit": "TFLOP/s", "frac": achieved_tflops / peak, "traffic": None,
                     "peak_note": {"fp32": "fp32 matrix peak (v_mfma_f32_16x16x4_f32)",
                                   "f16": "f16 dense MFMA peak (one pass per product)"}.get(
                                       eng.precision, "f16 dense MFMA peak 2516.6 / 3 passes per f32 product "
                                                      "(f32-equivalent)"),
                     "kernel": kernel_name + (" x CEM iterations + select/refit (HIP events around the "
                                              "whole device-side CEM call)" if cem else ""),
                     "flop_per_launch": K * H * fpcs,
                     "flop_per_cand_step": fpcs,
                     "limiter": LIMITER.get("cfg3" if (args.workload == "cfg3" and world == 1) else
                                            "ns_shard" if (args.workload == "cfg3" and K <= 8192) else
                                            args.workload, ""),
                     "per": "one rank's shard launch (the slowest rank's, max over ranks)"},
        "cpu_baseline": None,
        "small_k": None,
        "prewarm": dict(pre, note="untimed control steps of the same workload before the W warmup steps: the GPU's "
                                  "clocks ramp over the first ~40 ms of work after idle (profiles/r06_cold_ramp.txt)"),
    }
    if scale is not None:
        out["scale"] = scale
    if lib_line is not None:
        out["library_comm"] = lib_line
    # PMC HBM traffic per launch of THIS round's kernels (tools/gpu_validate.sh traffic: rocprofv3 --pmc FETCH_SIZE /
    # WRITE_SIZE in separate passes, the gfx950 FETCH_SIZE x2 correction calibrated on the action tensor)
    prof = os.path.join(REPO, "profiles", TRAFFIC_FILE)
    out["roofline"]["traffic_source"] = f"profiles/{TRAFFIC_FILE}"
    # (N > 1: the rank's shard is measured by the 1-GPU line of the same 2x500 tanh net at that K, if any)
    shard_wl = args.workload if world == 1 else {65536: "cfg3", 32768: "cfg4_shard", 8192: "ns_shard",
                                                 4096: "cfg2"}.get(K) if args.workload == "cfg3" else None
    if os.path.exists(prof) and shard_wl:
        try:
            key = shard_wl + {"fp32": "", "f16": ":f16"}.get(eng.precision, ":split") + \
                (":device" if args.actions == "device" else "")
            out["roofline"]["traffic_key"] = key
            tr = json.load(open(prof)).get(key)
            if tr:
                out["roofline"]["traffic"] = tr["hbm_bytes_per_launch"]
        except Exception:
            pass
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import mpc_oracle as orc
        w = orc.RewardMLPWeights(kernels, biases, ln_g, ln_b) if reward else orc.MLPWeights(kernels, biases, act, ln_g, ln_b)
        out["cpu_baseline"] = cpu_baseline(w, norm, state, H, args.cpu_baseline_seconds, K, net_label(wl, prob),
                                           pol_arrays, wl.get("explore", 0.5), gamma, cem)
    if rank == 0 and world == 1 and not args.no_small_k:
        out["small_k"] = small_k_lines(local, with_cpu=not args.no_cpu_baseline)
    if rank == 0 and world == 1 and not args.no_cfg2 and args.workload == "cfg3" and not args.no_small_k:
        out["cfg2"] = cfg2_line(local, with_cpu=not args.no_cpu_baseline)
    if rank == 0 and world == 1 and not args.no_extra and args.workload == "cfg3":
        out["ns_shard"] = workload_line("ns_shard", local, steps=50, warmup=5, with_cpu=not args.no_cpu_baseline)
        out["ns_shard"]["exchange_cost"] = exchange_cost(local)
        out["cfg4_shard"] = workload_line("cfg4_shard", local, with_cpu=not args.no_cpu_baseline)
        out["cfg5"] = workload_line("cfg5", local, steps=5, warmup=1, cpu_seconds=4.0,
                                    with_cpu=not args.no_cpu_baseline)
    if (rank == 0 and world == 1 and not args.no_f16 and not (cem or policy or reward or ln) and act == "tanh"
            and eng.precision != "f16"):
        out["f16_single_pass"] = f16_line(wl, prob, local, name=args.workload)
    out["summary"] = summary_of(out)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if lib_comm is not None:
        eng.set_comm(None)
        lib_comm.close()
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
