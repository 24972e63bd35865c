"""PPO_ICM's Intrinsic Curiosity Module on libppox (K11, csrc/icm.hip) for image observations.

The reference's module (models.py:270-320) is a torch MLP trained by autograd
(ppo.py:684-699) and evaluated per collect step (ppo.py:629-630).  On Atari frames
its state encoder's first layer, Linear(4*84*84 -> 32), reads every minibatch row's
28,224-byte frame stack twice (forward, weight gradient), and the rest of the module is
~30 small 32-wide ops.  NativeIcm runs the same math as six kernels per minibatch:
  ppox_icm_pack_w1 (once per optimizer step), ppox_icm_encode (split-f16 MFMA encoder
  straight off the uint8 rollout rows + the per-row rest of the encoder),
  ppox_icm_pair_backward (inverse / forward model, both losses and their backward for the
  pairs (row j, row j + 1), ppo.py:684), ppox_icm_row_backward, ppox_icm_grad_reduce
  (every gradient but W1's, written into the ICM's flat gradient segment) and
  ppox_icm_enc_wgrad (W1's gradient, split-f16 MFMA) — and collect as ppox_icm_encode +
  ppox_icm_int_reward.  All gradients are overwritten (no zero fill), deterministic.

Supported: Discrete actions (<= 32), feature size 32, uint8 observations of K bytes,
K % 64 == 0 — the Atari configuration.  Other PPO_ICM setups (vector observations, Box
actions) keep the torch module (ppo.icm_loss_sharded).
"""
import numpy as np
import torch

import native

H = 32


def _param_order(icm):
    se, fm, im = icm.state_encoder, icm.forward_model, icm.inverse_model
    return [se[0].weight, se[0].bias, se[2].weight, se[2].bias, fm[0].weight, fm[0].bias, fm[2].weight, fm[2].bias,
            im[0].weight, im[0].bias, im[2].weight, im[2].bias, icm.action_encoder.weight]


def supported(icm, flat, obs_shape, obs_dtype):
    """True when the kernels cover this module and its parameters sit in `flat` as the
    kernels expect (W1, then the ppox_icm_param_elems segment, contiguous, module order)."""
    if not (icm.discrete and icm.feature_size == H and 1 <= icm.n_actions <= 32 and obs_dtype == torch.uint8):
        return False
    K = int(np.prod(obs_shape))
    if K % 64 != 0 or icm.state_encoder[0].weight.shape != (H, K):
        return False
    ps = _param_order(icm)
    if [p.data_ptr() for p in flat.params] != [p.data_ptr() for p in ps]:
        return False
    base = flat.data.data_ptr()
    off = 0
    for p in ps:
        if p.data_ptr() != base + 4 * off or not p.is_contiguous():
            return False
        off += p.numel()
    return off == flat.n == H * K + native.icm_param_elems(icm.n_actions)


class NativeIcm:
    """Binds an IntrinsicCuriosityModule whose parameters live in a FlatParams (`flat`)."""

    def __init__(self, icm, flat, K):
        self.icm, self.flat, self.K = icm, flat, int(K)
        self.A = icm.n_actions
        w1 = icm.state_encoder[0].weight
        self.w1, self.w1_grad = w1, w1.grad
        n = native.icm_param_elems(self.A)
        off = H * self.K
        self.seg, self.gseg = flat.data[off:off + n], flat.grad[off:off + n]
        self.q = torch.empty(native.icm_w1_pack_elems(self.K), dtype=torch.int16, device=flat.device)
        self._version = None
        self._bufs = {}
        self._captured = set()

    def _buf(self, name, shape, dtype=torch.float32):
        """A named workspace, grown on demand.  A buffer first handed out while a graph is
        being captured (the collect graph's c0 / c1 / ir tags) is pinned: the replayed graph
        writes into it, so a later request that would replace it raises instead."""
        n = int(np.prod(shape))
        b = self._bufs.get(name)
        if torch.cuda.is_current_stream_capturing():
            self._captured.add(name)
        if b is None or b.numel() < n or b.dtype != dtype:
            if b is not None and name in self._captured:
                raise RuntimeError(f"ICM workspace '{name}' is captured by the collect graph and cannot grow "
                                   f"({b.numel()} -> {n} elements, {b.dtype} -> {dtype})")
            b = torch.empty(max(n, 1), dtype=dtype, device=self.flat.device)
            self._bufs[name] = b
        return b[:n].view(shape)

    def pack(self):
        """Split W1 into its f16 planes once per optimizer step."""
        v = (self.flat.step_count, self.flat.data.data_ptr())
        if v != self._version:
            native.icm_pack_w1(self.w1.detach(), self.q)
            self._version = v

    def _src(self, obs):
        """(frames, idx, T, N, rows) of a convs.RolloutRows or a contiguous (rows, ...) uint8 tensor."""
        if hasattr(obs, "idx"):
            return obs.frames, obs.idx, obs.T, obs.N, obs.shape[0]
        assert obs.dtype == torch.uint8 and obs.is_contiguous()
        return obs, None, 0, 0, obs.shape[0]

    def encode(self, obs, tag="enc", rowno=False):
        """-> (pre1, phi[, rowno]) of the observation rows (phi = state_encoder(obs))."""
        self.pack()
        x, idx, T, N, rows = self._src(obs)
        pre1 = self._buf(tag + "_pre1", (rows, H))
        phi = self._buf(tag + "_phi", (rows, H))
        rn = self._buf(tag + "_rowno", (rows,), torch.int32) if rowno else None
        # a workspace per tag: the collect graph captures its tags' buffers, which a training
        # encode of another row count must never replace
        ws = self._buf(tag + "_ws", (max(native.icm_encode_workspace_bytes(rows, self.K), 1),), torch.uint8)
        native.icm_encode(x, rows, idx, T, N, self.K, self.q, self.seg, ws, pre1, phi, rn)
        return (pre1, phi, rn) if rowno else (pre1, phi)

    def int_reward(self, phi_s, phi_n, actions, rewards, eta, out):
        """Collect (ppo.py:629-631): out = int_reward(s, s', a); rewards mixed in place."""
        native.icm_int_reward(phi_s, phi_n, actions, phi_s.shape[0], self.A, self.seg, eta, rewards, out)

    def train_minibatch(self, obs, actions, pos, B, beta, ctx, loss_accum):
        """ICM loss of one global minibatch of B rows + its backward into the ICM's flat
        gradient (overwritten).  obs: this rank's rows (RolloutRows or uint8 rows), actions:
        the int32 action array that the rows' frame-row numbers index (the rollout's (T, N)
        actions for RolloutRows, per-row actions otherwise), pos: their minibatch positions
        (world > 1; None in one process).  loss_accum[0] += this rank's loss share."""
        x, _, _, _, Bl = self._src(obs)
        A = self.A
        pre1 = phi = rowno = None
        if Bl > 0:
            pre1, phi, rowno = self.encode(obs, "mb", rowno=True)
        partials = self._buf("partials", (max(native.icm_partials_bytes(max(Bl, 1), A) // 4, 1),))
        g1q = self._buf("g1q", (max(native.icm_g1_pack_elems(Bl), 1),), torch.int16)
        if not ctx.enabled:
            dS, dN = self._buf("dS", (B, H)), self._buf("dN", (B, H))
            native.icm_pair_backward(phi, B, actions, rowno, None, B - 1, B - 1, A, beta, self.seg, dS, dN, partials)
            native.icm_row_backward(dS, dN, None, Bl, pre1, self.seg, A, g1q, partials)
            native.icm_grad_reduce(partials, Bl, B - 1, A, beta, B - 1, self.gseg, loss_accum)
            native.icm_enc_wgrad(x, rowno, Bl, self.K, g1q, self.w1_grad)
            return
        # world > 1: the pairs cross rank boundaries (ppo.icm_loss_sharded) — features and actions
        # are summed into minibatch positions, each rank evaluates the pairs whose first row it
        # owns, and dL/dphi is summed back (same collective sequence on every rank)
        # features and actions (as f32: small integers, exact) at their positions in one buffer (one
        # launch: zero-fill + scatter), one all-reduce
        fa = self._buf("fa", (B * (H + 1),))
        native.icm_scatter_positions(phi, actions.reshape(-1), rowno, pos, Bl, B, fa)
        ctx.all_reduce_(fa)
        dS, dN = self._buf("dS", (B, H)), self._buf("dN", (B, H))
        if Bl > 0:
            # the pair list is every owned position: the kernel skips the one at B - 1 (no pair), so
            # the host never waits for a compaction's count; the actions are fa's f32 tail (NULL)
            native.icm_pair_backward(fa, B, None, None, pos, Bl, B - 1, A, beta, self.seg, dS, dN, partials)
        g = ctx.all_reduce_(dS.add_(dN)) if Bl > 0 else ctx.all_reduce_(dS.zero_())
        if Bl == 0:
            self.gseg.zero_()
            self.w1_grad.zero_()
            return
        native.icm_row_backward(g, None, pos, Bl, pre1, self.seg, A, g1q, partials)
        native.icm_grad_reduce(partials, Bl, Bl, A, beta, B - 1, self.gseg, loss_accum)
        native.icm_enc_wgrad(x, rowno, Bl, self.K, g1q, self.w1_grad)
