"""Numerics utilities on the device (reference: util.py).

RunningMeanStd keeps the reference's interface (util.py:9-44: `update(arr)`,
`update_from_moments(m, v, n)`, attributes mean / var / count) with the state
resident in HBM as float64 and the batch moments computed by libppox
(ppox_rms_update_u8 / _f32); count stays a host float like the reference's.
ActionConverter is the reference's action-space adapter (util.py:47-79).
"""
import numpy as np
import torch
import torch.nn as nn

import native


class RunningMeanStd:
    """util.py:9-44 on the device.  `shape=()` broadcasts to per-feature state
    on the first update, like the reference's numpy broadcasting."""

    def __init__(self, epsilon=1e-4, shape=(), device="cuda"):
        self.device = torch.device(device)
        self.shape = tuple(shape)
        self.count = epsilon
        self._mean = torch.zeros(self.shape, dtype=torch.float64, device=self.device)
        self._var = torch.ones(self.shape, dtype=torch.float64, device=self.device)
        self._ws = None

    # reference attribute names (numpy on the host in the reference)
    @property
    def mean(self):
        return self._mean

    @property
    def var(self):
        return self._var

    def _features(self, n):
        if self._mean.numel() != n:
            if self._mean.dim() != 0:
                raise ValueError(f"RunningMeanStd has {self._mean.numel()} features, batch has {n}")
            self._mean = self._mean.expand(n).contiguous()
            self._var = self._var.expand(n).contiguous()

    def update(self, arr):
        """Batch moments over axis 0 of a (rows, ...) device tensor (u8 or f32)."""
        if not isinstance(arr, torch.Tensor):
            arr = torch.as_tensor(np.asarray(arr))
        arr = arr.to(self.device)
        rows = arr.shape[0]
        x = arr.reshape(rows, -1)
        cols = x.shape[1]
        if arr.dim() == 1:  # scalar stream (int_rew_rms): (N,) -> shape () state
            x = arr.contiguous()
            if x.dtype != torch.float32:
                x = x.float()
            native.rms_update_f32(x, rows, 1, 1, self._mean, self._var, self.count)
        elif x.dtype == torch.uint8:
            self._features(cols)
            need = native.rms_u8_workspace_bytes(rows, cols)
            if self._ws is None or self._ws.numel() < need:
                self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
            native.rms_update_u8(x, rows, cols, x.stride(0), self._mean, self._var, self.count, self._ws)
        else:
            x = x if x.dtype == torch.float32 else x.float()
            self._features(cols)
            if cols == 1:
                x = x.reshape(rows).contiguous()
            native.rms_update_f32(x, rows, cols, x.stride(0) if cols > 1 else 1, self._mean, self._var, self.count)
        self.count = rows + self.count

    def update_from_moments(self, batch_mean, batch_var, batch_count):
        """util.py:30-44 (used to merge moments gathered from other ranks)."""
        bm = torch.as_tensor(batch_mean, dtype=torch.float64, device=self.device)
        bv = torch.as_tensor(batch_var, dtype=torch.float64, device=self.device)
        if self._mean.dim() == 0 and bm.dim() > 0:
            self._features(bm.numel())
        delta = bm - self._mean
        tot = self.count + batch_count
        new_mean = self._mean + delta * batch_count / tot
        m2 = self._var * self.count + bv * batch_count + torch.square(delta) * self.count * batch_count / (
            self.count + batch_count)
        self._mean = new_mean
        self._var = m2 / (self.count + batch_count)
        self.count = batch_count + self.count


class ActionConverter:
    """util.py:47-79."""

    def __init__(self, action_space):
        self.action_type = action_space.__class__.__name__
        if self.action_type == "Discrete":
            self.num_actions = action_space.n
            self.action_output = 1
        elif self.action_type == "Box":
            self.num_actions = action_space.shape[0]
            self.action_output = self.num_actions
        else:
            raise ValueError(f"unsupported action space {self.action_type}")

    def get_loss(self):
        return nn.CrossEntropyLoss() if self.action_type == "Discrete" else nn.MSELoss()

    def action(self, action):
        return action.squeeze().long() if self.action_type == "Discrete" else action.float()
