"""ES-NSRA (evolution strategies with novelty-seeking and adaptive reward weight) on
the device — the reference's evolution_strategies.py API (EvolutionStrategy,
FeedForwardNetwork) over libppox kernels (csrc/es.hip).

Reference: evolution_strategies.py:22-101 (FeedForwardNetwork), :103-384
(EvolutionStrategy).  What runs where:
  * population perturbations eps (P x n_params, float64): ppox_es_noise, a Philox stream
    keyed by (global member, generation) — the reference draws np.random.randn per
    member and layer (:176-186); sharding members over ranks never changes the stream;
  * fitness of every perturbed policy (:137-174 evaluate/_get_rewards): ppox_es_evaluate,
    one wave per member running its whole episode (arctan MLP + tanh head, the env step)
    in registers/LDS;
  * the ES update (:224-246): reward normalisation on the host exactly as numpy does it,
    then the P^T c GEMV on the device (ppox_es_update);
  * novelty (:201-222, :273-297): behaviour characterisation from a device episode,
    kNN distance / probabilities / brain choice on the host (numpy RNG as the reference).
The reference evaluates MuJoCo envs through gym (unavailable offline); the episodes
here run the synthetic 'SwimmerLike' dynamics of oracle/es.py (state dim and action
dim of the env_id, Box actions; behaviour = final state[0:2], standing in for qpos[0:2]).
Multi-GPU: members sharded by index across ranks; fitness all-gathered, the partial
update all-reduced (one n_params float64 message per generation).
"""
import time
from collections import deque

import numpy as np
import torch

import logger
import native
from dist import DistContext
from env import VECTOR_ENVS, Box


class FeedForwardNetwork:
    """evolution_strategies.py:22-101: weights list of (in, out) float64 matrices drawn with
    np.random.randn (same draws as the reference for the same numpy seed), no biases."""

    def __init__(self, env, hidden_sizes):
        self.env = env
        self.action_space = env.action_space.__class__.__name__
        layer_sizes = [env.observation_space.shape[0], *hidden_sizes, self.num_actions]
        self.weights = [np.random.randn(layer_sizes[i], layer_sizes[i + 1]) for i in range(len(layer_sizes) - 1)]

    @property
    def num_actions(self):
        if self.action_space == "Discrete":
            return self.env.action_space.n
        return self.env.action_space.shape[0]

    def predict(self, inp):
        """:50-63 (Box): tanh(arctan-MLP(obs)); host numpy, for inspection / tests."""
        out = np.expand_dims(np.asarray(inp, np.float64).flatten(), 0)
        for w in self.weights[:-1]:
            out = np.arctan(np.dot(out, w))
        return np.tanh(np.dot(out, self.weights[-1]).astype(float)).astype(np.double)

    def get_weights(self):
        return self.weights

    def set_weights(self, weights):
        self.weights = weights


class _EnvSpec:
    def __init__(self, env_id):
        d, space, max_len = VECTOR_ENVS.get(env_id, (8, Box((2,)), 1000))
        if space.__class__.__name__ != "Box":
            raise NotImplementedError("ES-NSRA runs Box action spaces (the reference's MuJoCo tasks)")
        self.observation_space = Box((d,))
        self.action_space = space
        self.max_len = max_len


def _flat(weights):
    return np.concatenate([w.reshape(-1) for w in weights])


class EvolutionStrategy:
    """evolution_strategies.py:103-384 with the reference's constructor signature
    (+ seed / episode_len / device keywords of this build)."""

    def __init__(self, env_id, hidden_sizes, nsr_plateu=1.5, nsr_range=[0, 1], nsr_update=0.05, population_size=50,
                 sigma=0.1, learning_rate=0.01, decay=0.9995, novelty_param=0.5, num_threads=1, seed=0,
                 episode_len=None, device=None):
        if len(hidden_sizes) != 2 or max(hidden_sizes) > 64:
            raise ValueError("device ES policy: two hidden layers of at most 64 units")
        self.env_id = env_id
        self.env = _EnvSpec(env_id)
        self.hidden_sizes = list(hidden_sizes)
        self.model = FeedForwardNetwork(self.env, hidden_sizes=hidden_sizes)
        self.weights = self.model.get_weights()
        self.POPULATION_SIZE = population_size
        self.SIGMA = sigma
        self.learning_rate = learning_rate
        self.decay = decay
        self.num_threads = num_threads  # API parity; the device evaluates every member at once
        self.rewards = deque(maxlen=50)
        self.novelty_param = novelty_param
        self.K = 10
        self.nsr_plateu, self.nsr_range, self.nsr_update = nsr_plateu, nsr_range, nsr_update
        self.dist = DistContext.current()
        self.device = torch.device(device or "cuda")
        native.lib()  # fail loudly without the HIP library / a GPU
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.env_seed = (self.seed * 0x9E3779B97F4A7C15 + 1) & 0xFFFFFFFFFFFFFFFF
        self.T = int(episode_len or self.env.max_len)
        self.sizes = [self.env.observation_space.shape[0], *hidden_sizes, self.model.num_actions]
        self.n_params = int(sum(a * b for a, b in zip(self.sizes[:-1], self.sizes[1:])))
        P, g, G = population_size, self.dist.rank, self.dist.world
        self.m0, self.m1 = P * g // G, P * (g + 1) // G  # this rank's members
        self.generation = 0
        self.xi = torch.empty(self.T * self.sizes[0], dtype=torch.float64, device=self.device)
        native.es_env_noise(self.T, self.sizes[0], self.env_seed, self.xi)

    # ---------------------------------------------------------------- pieces
    def _get_weights_try(self, w, p):
        """:137-145 (reference-format population member)."""
        return [wi + self.SIGMA * pi for wi, pi in zip(w, p)]

    def get_weights(self):
        return self.weights

    def _dev_weights(self, weights):
        return torch.from_numpy(_flat(weights)).to(self.device)

    def _evaluate_dev(self, weights, eps=None, P=1, bc=False):
        D, H1, H2, A = self.sizes
        fit = torch.empty(P, dtype=torch.float64, device=self.device)
        b = torch.empty(P, 2, dtype=torch.float64, device=self.device) if bc else None
        w = weights if torch.is_tensor(weights) else self._dev_weights(weights)
        native.es_evaluate(w, eps, self.SIGMA, P, D, H1, H2, A, self.T, self.env_seed, self.xi, fit, b)
        return fit, b

    def evaluate(self, weights, env=None):
        """:147-165: total reward of one episode of `weights` (device episode)."""
        return float(self._evaluate_dev(weights)[0].item())

    def _get_population(self):
        """:167-177 -> this rank's perturbations, (P_local, n_params) float64 on the device."""
        P = self.m1 - self.m0
        eps = torch.empty(P, self.n_params, dtype=torch.float64, device=self.device)
        native.es_noise(P, self.n_params, self.m0, self.generation, self.seed, eps)
        return eps

    def _get_rewards(self, pool, population):
        """:179-195: fitness of every perturbation -> (P,) numpy (all ranks' members)."""
        fit, _ = self._evaluate_dev(self._dev_weights(self.weights), population, population.shape[0])
        if self.dist.enabled:  # members in rank order (shards may differ by one when P % world != 0)
            P, G = self.POPULATION_SIZE, self.dist.world
            fit = self.dist.all_gather_rows(fit, [P * (g + 1) // G - P * g // G for g in range(G)])
        return fit.cpu().numpy()

    def get_behavior_char(self, weights, env=None):
        """:248-271: final state[0:2] of an episode (the qpos[0:2] analogue) -> (1, 2)."""
        _, b = self._evaluate_dev(weights, bc=True)
        return b.cpu().numpy()

    def get_kNN(self, archive, bc, n_neighbors):
        """:273-289: sum of the n_neighbors smallest Euclidean distances (brute force, as
        sklearn's exact NearestNeighbors)."""
        arch = np.concatenate(archive)
        d = np.sqrt(((arch - np.asarray(bc).reshape(1, -1)) ** 2).sum(axis=1))
        return float(np.sort(d)[:n_neighbors].sum())

    def get_novelty(self, p, archive):
        """:201-222."""
        S = np.minimum(self.K, len(archive))
        novelty = self.get_kNN(archive, self.get_behavior_char(p), S) / S
        return 5e-3 if novelty <= 1e-3 else novelty

    def calc_noveltiy_distribution(self, novelties):
        """:291-297 (the reference's spelling)."""
        return [round((novel / (sum(novelties))), 4) for novel in novelties]

    def _update_weights(self, rewards, population, novelty=None):
        """:224-246.  population: this rank's device perturbations (P_local, n) — or the
        reference's list-of-lists format (host numpy path, as the reference computes it)."""
        std = rewards.std()
        if std == 0:
            return
        r = (rewards - rewards.mean()) / std
        update_factor = self.learning_rate / (self.POPULATION_SIZE * self.SIGMA)
        if not torch.is_tensor(population):  # reference format: (P, in, out) per layer
            for index, w in enumerate(self.weights):
                lp = np.array([p[index] for p in population])
                if novelty is not None:
                    nov = np.full(r.shape, novelty)
                    score = ((1 - self.novelty_param) * np.dot(lp.T, r).T
                             + self.novelty_param * np.dot(lp.T, nov).T) / 2
                else:
                    score = np.dot(lp.T, r).T
                self.weights[index] = w + update_factor * score
            self.learning_rate *= self.decay
            return
        # device: delta = sum_p c_p eps_p, c_p = ((1 - nu) r_p + nu * novelty) / 2
        coef = ((1 - self.novelty_param) * r + self.novelty_param * novelty) / 2 if novelty is not None else r
        c = torch.from_numpy(np.ascontiguousarray(coef[self.m0:self.m1], dtype=np.float64)).to(self.device)
        P = population.shape[0]
        ws = torch.empty(native.es_update_workspace_bytes(P, self.n_params) // 8 + 1, dtype=torch.float64,
                         device=self.device)
        delta = torch.empty(self.n_params, dtype=torch.float64, device=self.device)
        native.es_update(population, c, P, self.n_params, ws, delta)
        if self.dist.enabled:
            self.dist.all_reduce_(delta)
        d = (update_factor * delta).cpu().numpy()
        off = 0
        for index, w in enumerate(self.weights):
            k = w.size
            self.weights[index] = w + d[off:off + k].reshape(w.shape)
            off += k
        self.learning_rate *= self.decay

    # ------------------------------------------------------------------ run
    def run(self, total_timesteps, reward_target=None, log_interval=1, log_to_file=False):
        """:299-384 (total_timesteps counts generations, as in the reference)."""
        quiet = self.dist.rank != 0
        logger.configure("ES", self.env_id, log_to_file and not quiet, quiet=quiet)
        MPS = 2
        meta_population = [FeedForwardNetwork(self.env, hidden_sizes=self.hidden_sizes) for _ in range(MPS)]
        start_time = time.time()
        archive = []
        delta_reward_buffer = deque(maxlen=10)
        novelties = []
        for iteration in range(int(total_timesteps)):
            self.generation = iteration
            population = self._get_population()
            if len(archive) > 0:
                novelties = []
                S = np.minimum(self.K, len(archive))
                for model in meta_population:
                    distance = self.get_kNN(archive, self.get_behavior_char(model.get_weights()), S)
                    novelty = distance / S
                    if novelty <= 1e-3:
                        novelty = 5e-3
                    novelties.append(novelty)
                probs = np.array(self.calc_noveltiy_distribution(novelties))
                probs /= probs.sum()
                brain_idx = np.random.choice(list(range(MPS)), p=probs)
                novelty = novelties[brain_idx]
            else:
                brain_idx = np.random.randint(0, MPS)
                novelty = 1
            self.weights = [w.copy() for w in meta_population[brain_idx].get_weights()]
            rewards = self._get_rewards(None, population)
            self._update_weights(rewards, population, novelty)
            meta_population[brain_idx].set_weights([w.copy() for w in self.weights])

            mean_reward_batch = np.mean(rewards)
            # the reference takes np.mean of the (first: empty) deque -> nan, so the first
            # schedule step always lowers the novelty weight
            reward_gradient_mean = np.mean(delta_reward_buffer) if len(delta_reward_buffer) else np.nan
            r_koeff = abs(mean_reward_batch - reward_gradient_mean)
            if iteration % 5 == 0:
                if r_koeff < self.nsr_plateu:
                    self.novelty_param = np.minimum(self.nsr_range[1], self.novelty_param + self.nsr_update)
                else:
                    self.novelty_param = np.maximum(self.nsr_range[0], self.novelty_param - self.nsr_update)
            delta_reward_buffer.append(mean_reward_batch)
            archive.append(self.get_behavior_char(self.weights))
            self.rewards.extend([self.evaluate(self.weights)])
            if (iteration + 1) % log_interval == 0:
                logger.record("iteration", iteration + 1)
                logger.record("reward", np.mean(self.rewards))
                logger.record("novelty", np.mean(novelties) if len(novelties) else np.nan)
                logger.record("n_koeff", self.novelty_param)
                logger.record("total_time", time.time() - start_time)
                logger.dump(step=iteration + 1)
            if reward_target is not None and np.mean(self.rewards) > reward_target:
                logger.record("iteration", iteration + 1)
                logger.record("reward", np.mean(self.rewards))
                logger.record("total_time", time.time() - start_time)
                logger.dump(step=iteration + 1)
                break
        return self
