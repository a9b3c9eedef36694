"""NNDynamicsModel / NNDynamicsRewardModel weight containers (dynamics.py:7-238 API).

The reference builds a TF1 graph (dynamics.py:54-71) whose variables the
rollout engine must read.  This class is the MI355X-side container: the
same constructor signature, the dense kernels in TF layout ``[in, out]`` held
as torch tensors (PyTorch-ROCm is used as the weight store only), the
normalization stats of dynamics.py:41, and a ``version`` stamp that the
controller's re-sync hook compares.

``predict`` (dynamics.py:106-119) runs one horizon step of the same HIP
kernel in per-candidate-state mode; it never computes on the host.
``fit`` (dynamics.py:81-104, Adam on normalized deltas) runs on the GPU
(``bc_mpc_amd/fit.py``), off the control-step path.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np

from .engine import MLPSpec, RolloutEngine
from .weights import _act_name


class NNDynamicsModel():
    def __init__(self,
                 env,
                 n_layers,
                 size,
                 activation,
                 output_activation,
                 normalization,
                 batch_size,
                 iterations,
                 learning_rate,
                 sess=None,
                 layer_norm: bool = False,
                 seed: int = 0,
                 device: Optional[int] = None):
        import torch
        if output_activation is not None:
            raise ValueError("output_activation must be None (train_mpc_ppo.py:540)")
        self.env = env
        S = int(np.prod(env.observation_space.shape))
        A = int(np.prod(env.action_space.shape))
        self.state_dim, self.action_dim = S, A
        self.n_layers, self.size = int(n_layers), int(size)
        self.activation = _act_name(activation)
        self.layer_norm = bool(layer_norm)
        (self.mean_obs, self.std_obs, self.mean_action, self.std_action, self.mean_reward, self.std_reward,
         self.mean_nxt_state, self.std_nxt_state, self.mean_deltas, self.std_deltas) = normalization
        self.batch_size, self.iterations, self.learning_rate, self.sess = batch_size, iterations, learning_rate, sess
        self.device = device
        dims = [S + A] + [self.size] * self.n_layers + [S]
        g = torch.Generator().manual_seed(seed)
        # tf.layers.dense defaults: glorot_uniform kernel, zero bias
        self.kernels = []
        for i in range(len(dims) - 1):
            lim = float(np.sqrt(6.0 / (dims[i] + dims[i + 1])))
            self.kernels.append((torch.rand(dims[i], dims[i + 1], generator=g) * 2 - 1) * lim)
        self.biases = [torch.zeros(d) for d in dims[1:]]
        self.ln_gamma = [torch.ones(self.size) for _ in range(self.n_layers)] if self.layer_norm else None
        self.ln_beta = [torch.zeros(self.size) for _ in range(self.n_layers)] if self.layer_norm else None
        self.version = 1
        self._engines = {}

    # ------------------------------------------------------------ weights I/O
    def load_weights(self, kernels: Sequence, biases: Sequence, ln_gamma: Optional[Sequence] = None,
                     ln_beta: Optional[Sequence] = None) -> None:
        """Replace the weights (e.g. after an external fit); bumps ``version``."""
        import torch
        if len(kernels) != self.n_layers + 1 or len(biases) != self.n_layers + 1:
            raise ValueError("expected n_layers + 1 kernels and biases")
        for i, (k, b) in enumerate(zip(kernels, biases)):
            k = torch.as_tensor(np.asarray(k, dtype=np.float32))
            b = torch.as_tensor(np.asarray(b, dtype=np.float32))
            if k.shape != self.kernels[i].shape or b.shape != self.biases[i].shape:
                raise ValueError(f"layer {i}: shape {tuple(k.shape)} != {tuple(self.kernels[i].shape)}")
            self.kernels[i], self.biases[i] = k.clone(), b.clone()
        if self.layer_norm:
            if ln_gamma is None or ln_beta is None:
                raise ValueError("layer_norm model needs ln_gamma / ln_beta")
            self.ln_gamma = [torch.as_tensor(np.asarray(x, dtype=np.float32)).clone() for x in ln_gamma]
            self.ln_beta = [torch.as_tensor(np.asarray(x, dtype=np.float32)).clone() for x in ln_beta]
        self.version += 1

    def mlp_spec(self) -> MLPSpec:
        f = lambda t: t.detach().cpu().numpy().astype(np.float32)  # noqa: E731
        return MLPSpec([f(k) for k in self.kernels], [f(b) for b in self.biases], self.activation,
                       [f(x) for x in self.ln_gamma] if self.layer_norm else None,
                       [f(x) for x in self.ln_beta] if self.layer_norm else None)

    def normalization(self) -> List[np.ndarray]:
        return [self.mean_obs, self.std_obs, self.mean_action, self.std_action, self.mean_reward,
                self.std_reward, self.mean_nxt_state, self.std_nxt_state, self.mean_deltas, self.std_deltas]

    # ------------------------------------------------------------ dynamics.py:106-119
    def predict(self, unnormalized_state, unnormalized_action):
        import torch
        s = np.ascontiguousarray(unnormalized_state, dtype=np.float64)
        a = np.ascontiguousarray(unnormalized_action, dtype=np.float64)
        if s.ndim != 2 or a.ndim != 2 or s.shape[0] != a.shape[0]:
            raise ValueError("predict expects states [K, S] and actions [K, A]")
        K = s.shape[0]
        dev_index = self.device if self.device is not None else torch.cuda.current_device()
        eng = self._engines.get(K)
        if eng is None:
            eng = RolloutEngine(self.state_dim, self.action_dim, self.size, self.n_layers, self.activation,
                                self.layer_norm, 1, K, device=dev_index, cost="none")
            self._engines[K] = eng
        eng.set_weights(self.mlp_spec(), self.normalization(), self.version)
        dev = torch.device("cuda", dev_index)
        d_s = torch.from_numpy(s).to(dev)
        d_a = torch.from_numpy(a).to(dev).reshape(1, K, self.action_dim)
        d_traj = torch.empty((2, K, self.state_dim), dtype=torch.float64, device=dev)
        eng.rollout_async(d_s.data_ptr(), self.state_dim, d_a.data_ptr(), 0, 0, None, d_traj.data_ptr(), None,
                          torch.cuda.current_stream(dev).cuda_stream)
        out = d_traj[1].cpu().numpy()
        eng.check_status()
        return out

    def fit(self, data):  # dynamics.py:81-104
        """``iterations`` Adam steps on the GPU (bc_mpc_amd/fit.py, csrc/fit.hip) on batches drawn
        exactly as DataBufferGeneral.sample draws them; returns (last loss, 0) like the reference."""
        import torch
        from .fit import GPUFitter, buffer_arrays, sample_batches
        dev = self.device if self.device is not None else torch.cuda.current_device()
        if getattr(self, "_fitter", None) is None:
            self._fitter = GPUFitter(self.state_dim, self.action_dim, self.size, self.n_layers, self.activation,
                                     self.layer_norm, int(self.batch_size), float(self.learning_rate), dev)
            self._fit_version = None
        if self._fit_version != self.version:               # weights changed outside fit: re-upload
            self._fitter.set_params(self.mlp_spec(), self.normalization())
        states, actions, deltas = buffer_arrays(data)
        self._fitter.set_data(states, actions, deltas)
        size = int(getattr(data, "size", states.shape[0]))
        print("Model fitting for ", self.iterations, "times ... ")   # dynamics.py:88
        losses = self._fitter.run(sample_batches(size, int(self.batch_size), int(self.iterations)))
        ks, bs, gs, bes = self._fitter.get_params()
        self.load_weights(ks, bs, gs if self.layer_norm else None, bes if self.layer_norm else None)
        self._fit_version = self.version
        return (float(losses[-1]) if len(losses) else None), 0


class NNDynamicsRewardModel():
    """Two-head learned-reward net (dynamics.py:121-238 API) for the engine.

    Same constructor as the reference (no n_layers / size / activation: the net
    is hard-wired to a 500-wide tanh trunk and two 500-wide tanh heads,
    dynamics.py:150-177; ``size`` is exposed for smaller test nets).  Weights
    are held in TF creation order dense .. dense_4 (+ LayerNorm, _1, _2).
    ``predict`` returns ``(next_state [K,S] f64, reward [K,1] f64)`` computed by
    the HIP kernel (one horizon step, per-candidate states)."""

    def __init__(self,
                 env,
                 normalization,
                 batch_size,
                 iterations,
                 learning_rate,
                 sess=None,
                 layer_norm: bool = False,
                 size: int = 500,
                 seed: int = 0,
                 device: Optional[int] = None):
        import torch
        self.env = env
        S = int(np.prod(env.observation_space.shape))
        A = int(np.prod(env.action_space.shape))
        self.state_dim, self.action_dim, self.size = S, A, int(size)
        self.layer_norm = bool(layer_norm)
        (self.mean_obs, self.std_obs, self.mean_action, self.std_action, self.mean_reward, self.std_reward,
         self.mean_nxt_state, self.std_nxt_state, self.mean_deltas, self.std_deltas) = normalization
        self.batch_size, self.iterations, self.learning_rate, self.sess = batch_size, iterations, learning_rate, sess
        self.device = device
        h = self.size
        shapes = [(S + A, h), (h, h), (h, S), (h, h), (h, 1)]
        g = torch.Generator().manual_seed(seed)
        self.kernels = [(torch.rand(*sh, generator=g) * 2 - 1) * float(np.sqrt(6.0 / sum(sh))) for sh in shapes]
        self.biases = [torch.zeros(sh[1]) for sh in shapes]
        self.ln_gamma = [torch.ones(h) for _ in range(3)] if self.layer_norm else None
        self.ln_beta = [torch.zeros(h) for _ in range(3)] if self.layer_norm else None
        self.version = 1
        self._engines = {}

    def load_weights(self, kernels: Sequence, biases: Sequence, ln_gamma: Optional[Sequence] = None,
                     ln_beta: Optional[Sequence] = None) -> None:
        """Replace the weights (TF order dense .. dense_4); bumps ``version``."""
        import torch
        if len(kernels) != 5 or len(biases) != 5:
            raise ValueError("expected 5 kernels and biases (dense .. dense_4)")
        for i, (k, b) in enumerate(zip(kernels, biases)):
            k = torch.as_tensor(np.asarray(k, dtype=np.float32))
            b = torch.as_tensor(np.asarray(b, dtype=np.float32))
            if k.shape != self.kernels[i].shape or b.shape != self.biases[i].shape:
                raise ValueError(f"layer {i}: shape {tuple(k.shape)} != {tuple(self.kernels[i].shape)}")
            self.kernels[i], self.biases[i] = k.clone(), b.clone()
        if self.layer_norm:
            if ln_gamma is None or ln_beta is None or len(ln_gamma) != 3 or len(ln_beta) != 3:
                raise ValueError("layer_norm reward model needs 3 ln_gamma / ln_beta arrays")
            self.ln_gamma = [torch.as_tensor(np.asarray(x, dtype=np.float32)).clone() for x in ln_gamma]
            self.ln_beta = [torch.as_tensor(np.asarray(x, dtype=np.float32)).clone() for x in ln_beta]
        self.version += 1

    def mlp_spec(self) -> MLPSpec:
        f = lambda t: t.detach().cpu().numpy().astype(np.float32)  # noqa: E731
        return MLPSpec([f(k) for k in self.kernels], [f(b) for b in self.biases], "tanh",
                       [f(x) for x in self.ln_gamma] if self.layer_norm else None,
                       [f(x) for x in self.ln_beta] if self.layer_norm else None, model="reward")

    def normalization(self) -> List[np.ndarray]:
        return [self.mean_obs, self.std_obs, self.mean_action, self.std_action, self.mean_reward,
                self.std_reward, self.mean_nxt_state, self.std_nxt_state, self.mean_deltas, self.std_deltas]

    # dynamics.py:225-238
    def predict(self, unnormalized_state, unnormalized_action):
        import torch
        s = np.ascontiguousarray(unnormalized_state, dtype=np.float64)
        a = np.ascontiguousarray(unnormalized_action, dtype=np.float64)
        if s.ndim != 2 or a.ndim != 2 or s.shape[0] != a.shape[0]:
            raise ValueError("predict expects states [K, S] and actions [K, A]")
        K = s.shape[0]
        dev_index = self.device if self.device is not None else torch.cuda.current_device()
        eng = self._engines.get(K)
        if eng is None:
            eng = RolloutEngine(self.state_dim, self.action_dim, self.size, 2, "tanh", self.layer_norm, 1, K,
                                device=dev_index, cost="reward", model="reward")
            self._engines[K] = eng
        eng.set_weights(self.mlp_spec(), self.normalization(), self.version)
        dev = torch.device("cuda", dev_index)
        d_s = torch.from_numpy(s).to(dev)
        d_a = torch.from_numpy(a).to(dev).reshape(1, K, self.action_dim)
        d_traj = torch.empty((2, K, self.state_dim), dtype=torch.float64, device=dev)
        d_r = torch.empty(K, dtype=torch.float64, device=dev)        # reward * gamma**0
        eng.rollout_async(d_s.data_ptr(), self.state_dim, d_a.data_ptr(), 0, 0, d_r.data_ptr(), d_traj.data_ptr(),
                          None, torch.cuda.current_stream(dev).cuda_stream)
        out = d_traj[1].cpu().numpy(), d_r.cpu().numpy().reshape(K, 1)
        eng.check_status()
        return out

    def fit(self, data):  # dynamics.py:195-219
        """``iterations`` Adam steps on the GPU (bc_mpc_amd/fit.py, csrc/fit.hip, model "reward") on the
        sum loss_dynamic + loss_reward (dynamics.py:153-157), batches drawn exactly as
        DataBufferGeneral.sample draws them; returns the last step's (model_loss, reward_loss) like the
        reference (:219)."""
        import torch
        from .fit import GPUFitter, buffer_arrays_reward, sample_batches
        dev = self.device if self.device is not None else torch.cuda.current_device()
        if getattr(self, "_fitter", None) is None:
            self._fitter = GPUFitter(self.state_dim, self.action_dim, self.size, 2, "tanh", self.layer_norm,
                                     int(self.batch_size), float(self.learning_rate), dev, model="reward")
            self._fit_version = None
        if self._fit_version != self.version:               # weights changed outside fit: re-upload
            self._fitter.set_params(self.mlp_spec(), self.normalization())
        states, actions, rewards, deltas = buffer_arrays_reward(data)
        self._fitter.set_data(states, actions, deltas)
        self._fitter.set_rewards(rewards)
        size = int(getattr(data, "size", states.shape[0]))
        print("Model fitting for ", self.iterations, "times ... ")   # dynamics.py:185
        iters = int(self.iterations)
        losses = self._fitter.run(sample_batches(size, int(self.batch_size), iters))
        rlosses = self._fitter.reward_losses(iters)
        ks, bs, gs, bes = self._fitter.get_params()
        self.load_weights(ks, bs, gs if self.layer_norm else None, bes if self.layer_norm else None)
        self._fit_version = self.version
        if not iters:
            return None, None
        return float(losses[-1]), float(rlosses[-1])
