"""Torch-CPU restatement of the reference networks and distribution heads.

Test infrastructure only (see oracle/__init__.py).

Reference architectures (construction order == torch RNG consumption order,
so a given torch seed reproduces the reference's initial weights bit-exactly):
  * MLP actor-critic            models.py:137-170 (MlpNetwork)
  * MLP actor-critic + int head models.py:173-213 (MlpIntrinsic)
  * orthogonal(sqrt 2)/zero init models.py:130-134
  * RND MLP, constant init      models.py:216-267
  * ICM MLP                     models.py:270-320
  * NatureCNN actor-critic      .ipynb_checkpoints/models-checkpoint.py:48-90
Distribution heads: models.py:30-124 (Categorical from softmax probs; Normal
with tanh mean and exp(log_std)).
"""
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.distributions as D


def _mlp(sizes, act):
    layers = []
    for i in range(len(sizes) - 1):
        layers.append(nn.Linear(sizes[i], sizes[i + 1]))
        if i < len(sizes) - 2:
            layers.append(act())
    return nn.Sequential(*layers)


def orthogonal_init(module, gain=math.sqrt(2)):
    """models.py:130-134 (and the CNN's conv+linear variant, checkpoint :74-77)."""
    for m in module.modules():
        if isinstance(m, (nn.Linear, nn.Conv2d)):
            nn.init.orthogonal_(m.weight, gain)
            nn.init.constant_(m.bias, 0)


class MlpAC(nn.Module):
    """MlpNetwork / MlpIntrinsic (models.py:137-213)."""

    def __init__(self, d_in, n_out, hidden=128, intrinsic=False):
        super().__init__()
        self.actor = _mlp([d_in, hidden, hidden, n_out], nn.Tanh)
        self.critic = _mlp([d_in, hidden, hidden, 1], nn.Tanh)
        if intrinsic:
            self.int_critic = _mlp([d_in, hidden, hidden, 1], nn.Tanh)
        self.intrinsic = intrinsic
        self.action_log_std = nn.Parameter(torch.zeros(1, n_out))
        orthogonal_init(self)

    def heads(self, x, box=False):
        """Returns (actor_out, log_std_or_None, value, int_value_or_None) with the
        reference's raw head shapes (value (B,1))."""
        a = self.actor(x)
        ls = None
        if box:
            a = a.tanh()
            ls = self.action_log_std.expand_as(a)
        iv = self.int_critic(x) if self.intrinsic else None
        return a, ls, self.critic(x), iv


class NatureCNN(nn.Module):
    """checkpoint models-checkpoint.py:48-90; optional intrinsic value head
    (parallel to extra_layer/critic_ext, this build's RND extension)."""

    def __init__(self, in_ch=4, n_actions=4, hidden=512, intrinsic=False):
        super().__init__()
        self.feature_extractor = nn.Sequential(
            nn.Conv2d(in_ch, 32, 8, 4), nn.ReLU(), nn.Conv2d(32, 64, 4, 2), nn.ReLU(),
            nn.Conv2d(64, 64, 3, 1), nn.ReLU(), nn.Flatten(), nn.Linear(7 * 7 * 64, hidden), nn.ReLU())
        self.actor = nn.Sequential(nn.Linear(hidden, n_actions))
        self.extra_layer = nn.Sequential(nn.Linear(hidden, hidden), nn.ReLU())
        self.critic_ext = nn.Linear(hidden, 1)
        self.intrinsic = intrinsic
        if intrinsic:
            self.int_extra_layer = nn.Sequential(nn.Linear(hidden, hidden), nn.ReLU())
            self.critic_int = nn.Linear(hidden, 1)
        orthogonal_init(self)

    def heads(self, x, box=False):
        f = self.feature_extractor(x)
        iv = self.critic_int(self.int_extra_layer(f)) if self.intrinsic else None
        return self.actor(f), None, self.critic_ext(self.extra_layer(f)), iv


class RndMLP(nn.Module):
    """models.py:216-267 — predictor/target MLPs with constant init."""

    def __init__(self, d_in, hidden=32):
        super().__init__()
        self.predictor = nn.Sequential(
            nn.Linear(d_in, hidden), nn.LeakyReLU(), nn.Linear(hidden, hidden), nn.LeakyReLU(),
            nn.Linear(hidden, hidden), nn.ELU(), nn.Linear(hidden, 1))
        self.target = nn.Sequential(
            nn.Linear(d_in, hidden), nn.LeakyReLU(), nn.Linear(hidden, hidden), nn.LeakyReLU(),
            nn.Linear(hidden, 1))
        for n, p in self.target.named_parameters():
            nn.init.constant_(p, 1.0 if "bias" in n else 0.01)
        for n, p in self.predictor.named_parameters():
            nn.init.constant_(p, 0.01 if "bias" in n else 1.0)
        for p in self.target.parameters():
            p.requires_grad = False

    def forward(self, x):
        return self.predictor(x), self.target(x)

    def int_reward(self, x):
        p, t = self(x)
        return (p - t).pow(2).squeeze()


class IcmMLP(nn.Module):
    """models.py:270-320."""

    def __init__(self, d_in, n_actions, discrete, hidden):
        super().__init__()
        self.discrete = discrete
        self.feature_size = hidden
        self.state_encoder = nn.Sequential(nn.Linear(d_in, hidden), nn.LeakyReLU(), nn.Linear(hidden, hidden))
        self.forward_model = nn.Sequential(nn.Linear(n_actions + hidden, hidden), nn.LeakyReLU(),
                                           nn.Linear(hidden, hidden))
        self.inverse_model = nn.Sequential(nn.Linear(2 * hidden, hidden), nn.LeakyReLU(),
                                           nn.Linear(hidden, n_actions))
        self.action_encoder = nn.Embedding(n_actions, n_actions) if discrete else nn.Linear(n_actions, n_actions)
        orthogonal_init(self)

    def _enc_action(self, a, squeeze):
        if self.discrete:
            a = a.squeeze().long() if squeeze else a.long()
            return self.action_encoder(a)
        return self.action_encoder(a.float())

    def forward(self, s, s_next, a):
        """models.py:300-309 -> (action_hat, next_state_hat, next_state_ft)."""
        ae = self._enc_action(a, True)
        f = self.state_encoder(s)
        fn = self.state_encoder(s_next).view(-1, self.feature_size)
        return self.inverse_model(torch.cat((f, fn), 1)), self.forward_model(torch.cat((f, ae), 1)), fn

    def int_reward(self, s, s_next, a):
        """models.py:311-320."""
        ae = self._enc_action(a, False)
        f = self.state_encoder(s)
        fn = self.state_encoder(s_next)
        nh = self.forward_model(torch.cat((f, ae), 1))
        return torch.clamp((nh - fn).pow(2).mean(dim=-1), -5, 5)


# ---------------------------------------------------------------------------
# distribution heads (models.py:30-124)
# ---------------------------------------------------------------------------
def categorical(logits):
    """Categorical(probs=softmax(logits)) as the reference builds it."""
    return D.Categorical(F.softmax(logits, dim=-1))


def act(net, obs, box=False):
    """models.py:30-50 / 75-99 -> actions, values, [int_values], log_probs."""
    a, ls, v, iv = net.heads(torch.as_tensor(obs, dtype=torch.float32), box)
    v = v.squeeze()
    iv = iv.squeeze() if iv is not None else None
    if box:
        dist = D.Normal(a, torch.exp(ls))
        actions = dist.sample()
        lp = dist.log_prob(actions)
    else:
        dist = categorical(a)
        actions = dist.sample().squeeze()
        lp = dist.log_prob(actions).squeeze()
    return actions, v, iv, lp


def evaluate(net, obs, actions, box=False, dtype=torch.float32):
    """models.py:52-73 / 101-124 -> values, [int_values], log_probs, entropy.
    dtype float64: the same program in exact-er arithmetic (conditioning checks)."""
    a, ls, v, iv = net.heads(torch.as_tensor(obs, dtype=dtype), box)
    v = v.squeeze()
    iv = iv.squeeze() if iv is not None else None
    if box:
        dist = D.Normal(a, torch.exp(ls))
        lp = dist.log_prob(actions)
    else:
        dist = categorical(a)
        lp = dist.log_prob(actions.flatten()).unsqueeze(1)
    return v, iv, lp, dist.entropy()
