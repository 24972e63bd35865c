"""Networks of the PPO + exploration path, with parameters packed in ONE flat
device buffer per optimiser (so the data-parallel gradient all-reduce is one
bucket and the Adam step one streaming kernel, libppox ppox_adam_step).

Architectures (reference file:line):
  MlpNetwork / MlpIntrinsic   models.py:137-213 (tanh MLPs, orthogonal sqrt(2) init :130-134)
  RndNetwork                  models.py:216-267 (constant init, target frozen)
  IntrinsicCuriosityModule    models.py:270-320
  CnnActorCritic (NatureCNN)  .ipynb_checkpoints/models-checkpoint.py:48-90; the
                              intrinsic value head (RND) mirrors MlpIntrinsic's
                              extra critic.
Modules are constructed on the CPU first so that a given torch seed yields the
reference's exact initial weights (same construction order => same torch RNG
consumption), then re-homed into the flat device buffers.
The NatureCNN convolutions run on the libppox MFMA implicit-GEMM kernels when
available (see convs.py); the small linear layers use PyTorch-ROCm (rocBLAS).
"""
import contextlib
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

import native


def orthogonal_init(module, gain=math.sqrt(2)):
    for m in module.modules():
        if isinstance(m, (nn.Linear, nn.Conv2d)):
            nn.init.orthogonal_(m.weight, gain)
            nn.init.constant_(m.bias, 0)


def _seq(sizes, act):
    layers = []
    for i in range(len(sizes) - 1):
        layers.append(nn.Linear(sizes[i], sizes[i + 1]))
        if i < len(sizes) - 2:
            layers.append(act())
    return nn.Sequential(*layers)


class MlpNetwork(nn.Module):
    """models.py:137-170 (+ MlpIntrinsic :173-213 with intrinsic=True)."""

    def __init__(self, input_size, output_size, hidden_size=128, intrinsic=False):
        super().__init__()
        self.actor = _seq([input_size, hidden_size, hidden_size, output_size], nn.Tanh)
        self.critic = _seq([input_size, hidden_size, hidden_size, 1], nn.Tanh)
        if intrinsic:
            self.int_critic = _seq([input_size, hidden_size, hidden_size, 1], nn.Tanh)
        self.intrinsic = intrinsic
        self.action_log_std = nn.Parameter(torch.zeros(1, output_size))
        orthogonal_init(self)

    def forward(self, x):
        """-> (actor output, value (B,), int value (B,) or None)."""
        x = x.float()
        iv = self.int_critic(x).squeeze(-1) if self.intrinsic else None
        return self.actor(x), self.critic(x).squeeze(-1), iv


# dW = d^T x of the 512-wide hidden layers: split-K (WGRAD_SPLIT row chunks as one batched
# GEMM + an ordered sum) from WGRAD_SPLIT_MIN rows — the single GEMM has only 64 output tiles
# of 64x64 for a 512x512 result and leaves most CUs idle over K = 16384 rows (tools/
# gemm_split_probe.py: 104 -> 67 us at 16384 rows, no gain at 2048)
WGRAD_SPLIT, WGRAD_SPLIT_MIN = 8, 8192
# the heads' backward to the fc output in one launch (ppox_head_backward; PPOX_HBW=0: the two-launch form)
HEAD_BWD_FUSED = native.ab_env("PPOX_HBW", "1") != "0"


def weight_grad(d, x, out, part=None):
    """out = d^T x (rows summed), d (B, m), x (B, n) contiguous; part: (WGRAD_SPLIT, m, n) scratch."""
    B = d.shape[0]
    if B >= WGRAD_SPLIT_MIN and B % WGRAD_SPLIT == 0 and part is not None:
        S = WGRAD_SPLIT
        torch.bmm(d.view(S, B // S, d.shape[1]).transpose(1, 2), x.view(S, B // S, x.shape[1]), out=part)
        torch.sum(part, 0, out=out)
    else:
        torch.mm(d.t(), x, out=out)


def linear_relu(x, weight, bias):
    """relu(x W^T + b) as one library GEMM with a bias+ReLU epilogue (hipBLASLt through
    torch._addmm_activation: bitwise equal to addmm().relu_(), one launch instead of two)."""
    return torch._addmm_activation(bias, x, weight.t())


class CnnActorCritic(nn.Module):
    """NatureCNN actor-critic (checkpoint models-checkpoint.py:48-90)."""

    def __init__(self, input_size=4, output_size=4, hidden_size=512, intrinsic=False):
        super().__init__()
        self.feature_extractor = nn.Sequential(
            nn.Conv2d(input_size, 32, 8, 4), nn.ReLU(), nn.Conv2d(32, 64, 4, 2), nn.ReLU(),
            nn.Conv2d(64, 64, 3, 1), nn.ReLU(), nn.Flatten(), nn.Linear(7 * 7 * 64, hidden_size), nn.ReLU())
        self.actor = nn.Sequential(nn.Linear(hidden_size, output_size))
        self.extra_layer = nn.Sequential(nn.Linear(hidden_size, hidden_size), nn.ReLU())
        self.critic_ext = nn.Linear(hidden_size, 1)
        self.intrinsic = intrinsic
        if intrinsic:
            self.int_extra_layer = nn.Sequential(nn.Linear(hidden_size, hidden_size), nn.ReLU())
            self.critic_int = nn.Linear(hidden_size, 1)
        orthogonal_init(self)
        self.conv_impl = None  # set by convs.attach()

    def trunk(self, x):
        return self._trunk_am(x)[0]

    def _trunk_am(self, x, table=None, actor=False):
        """(f, the pass's amax table or None[, the actor's logits or None when `actor`]); table: a zeroed
        amax table for the pass (convs.NatureConvs.forward_acts)"""
        if self.conv_impl is not None and self.conv_impl.math != "f32" and not torch.is_grad_enabled():
            # inference (collect): the split-f16 fc GEMM straight off the conv trunk (the split-K form's
            # reduce also runs the actor head)
            h1, h2, h3, am = self.conv_impl.forward_acts(x.contiguous(), table=table)
            if actor:
                f, logits = self.conv_impl.fc_forward(h3, am, actor=(self.actor[0].weight, self.actor[0].bias))
                return f, am, logits
            return self.conv_impl.fc_forward(h3, am), am
        if self.conv_impl is not None:
            h = self.conv_impl(x)
        else:
            fe = self.feature_extractor
            h = F.relu(fe[0](x.float()))
            h = F.relu(fe[2](h))
            h = F.relu(fe[4](h))
        fc = self.feature_extractor[7]
        f = F.relu(F.linear(h.flatten(1), fc.weight, fc.bias))
        return (f, None, None) if actor else (f, None)

    def forward(self, x, value_out=None, table=None):
        """(actor logits, value, int value).  Inference (collect) only: value_out, a (B,) float32 buffer the value
        is written to (the rollout's row: no copy), table a zeroed amax table for the pass."""
        if not torch.is_grad_enabled():  # collect: the same head kernels as forward_train
            f, am, logits = self._trunk_am(x, table, actor=True)
            return self._heads(f, am, out=logits, value_out=value_out)[:3]
        f, am = self._trunk_am(x)
        v = self.critic_ext(self.extra_layer(f)).squeeze(-1)
        iv = self.critic_int(self.int_extra_layer(f)).squeeze(-1) if self.intrinsic else None
        return self.actor(f), v, iv

    # ---- explicit training forward/backward (no autograd graph): the same layer math as
    # forward() (addmm = F.linear, relu), with every parameter gradient written straight
    # into its .grad view of the flat gradient buffer (weights: GEMMs with out=, conv kernels
    # and ppox_head_grads overwrite theirs), so a minibatch with rows needs no zero-fill of
    # the buffer (ppo.BaseAlgorithm._zero_policy_grad).  Each parameter is used once per forward.
    def forward_train(self, x):
        """-> (actor out, value (B,), int value or None, ctx for backward_train)."""
        with torch.no_grad():
            x = x.contiguous()
            h1, h2, h3, am = self.conv_impl.forward_acts(x, train=True)
            hf = h3.view(h3.shape[0], -1)
            fc = self.feature_extractor[7]
            logits = None
            if self.conv_impl.math != "f32":  # (the small-batch fc form also runs the actor head)
                f, logits = self.conv_impl.fc_forward(h3, am, actor=(self.actor[0].weight, self.actor[0].bias))
            else:
                f = linear_relu(hf, fc.weight, fc.bias)
            out, v, iv, e, ie = self._heads(f, am, out=logits)
        return out, v, iv, (x, h1, h2, h3, f, e, ie, am)

    def _heads(self, f, am=None, out=None, value_out=None):
        """actor logits (unless `out` already holds them), value (into value_out when given), int value, and
        the hidden activations (no autograd): fused bias+ReLU GEMMs for the 512-wide layers (the extra layer
        on the split-f16 kernel for large batches: f's amax in am), skinny-row kernels for the narrow heads."""
        a, el, ce = self.actor[0], self.extra_layer[0], self.critic_ext
        if out is None:
            out = native.head_linear(f, a.weight, a.bias)
        cv = self.conv_impl
        v = None
        if am is not None and cv is not None and cv.split_head(f.shape[0]):
            import convs as _convs
            cv.pack(f.shape[0])
            e = torch.empty_like(f)
            native.head_hidden_fwd(f, cv.qh[0], el.bias, e, amax_f=am[_convs.AM_F])
        elif am is not None and cv is not None and cv.split_head_fwd(f.shape[0]) and f.is_contiguous() \
                and f.data_ptr() % 16 == 0:
            # small batches: split over K, the critic head fused into the reduce when its weight is aligned
            import convs as _convs
            B = f.shape[0]
            cv.pack(B)
            e = torch.empty_like(f)
            fuse = ce.weight.is_contiguous() and ce.weight.data_ptr() % 16 == 0
            v = (value_out if value_out is not None else torch.empty(B, device=f.device)) if fuse else None
            native.head_hidden_fwd_splitk(f, cv.qh[0], el.bias, cv.head_fwd_ws(B), e, amax_f=am[_convs.AM_F],
                                          critic=(ce.weight, ce.bias) if fuse else None, value=v)
        else:
            e = linear_relu(f, el.weight, el.bias)
        if v is None:
            v = native.head_linear(e, ce.weight, ce.bias).squeeze(-1)
            if value_out is not None:
                value_out.copy_(v)
                v = value_out
        ie = iv = None
        if self.intrinsic:
            il, ci = self.int_extra_layer[0], self.critic_int
            ie = linear_relu(f, il.weight, il.bias)
            iv = native.head_linear(ie, ci.weight, ci.bias).squeeze(-1)
        return out, v, iv, e, ie

    def _fc_grad_buf(self, w):
        buf = getattr(self, "_fcg", None)
        if buf is None or buf.device != w.device:
            buf = torch.empty_like(w)
            self._fcg = buf
        return buf

    def _wgrad_part(self, w):
        buf = getattr(self, "_wgp", None)
        if buf is None or buf.device != w.device:
            buf = torch.empty((WGRAD_SPLIT,) + tuple(w.shape), device=w.device)
            self._wgp = buf
        return buf

    def _fc_wgrad_ws(self, rows):
        need = native.nature_fc_wgrad_workspace_bytes(rows)
        ws = getattr(self, "_fcw_ws", None)
        if ws is None or ws.numel() < need or ws.device != self.actor[0].weight.device:
            ws = torch.empty(max(need, 1), dtype=torch.uint8, device=self.actor[0].weight.device)
            self._fcw_ws = ws
        return ws

    def _head_wgrad_ws(self, rows):
        need = native.head_hidden_wgrad_workspace_bytes(rows)
        ws = getattr(self, "_hh_ws", None)
        if ws is None or ws.numel() < need or ws.device != self.actor[0].weight.device:
            ws = torch.empty(max(need, 16), dtype=torch.uint8, device=self.actor[0].weight.device)
            self._hh_ws = ws
        return ws

    def _head_ws(self, rows, h, n_actions):
        need = native.head_grads_workspace_bytes(rows, h, n_actions, self.intrinsic)
        ws = getattr(self, "_hg_ws", None)
        if ws is None or ws.numel() < need or ws.device != self.actor[0].weight.device:
            ws = torch.empty(need, dtype=torch.uint8, device=self.actor[0].weight.device)
            self._hg_ws = ws
        return ws

    def backward_train(self, ctx, dout, dv, div=None, dense_ready=None):
        """Accumulate dL/dparams for upstream grads (dout (B,A), dv (B,), div (B,)).
        `dense_ready()` is called once every non-conv gradient (fc + heads) is enqueued,
        before the conv backward (ppo.BaseAlgorithm._bwd_reduce overlaps its all-reduce)."""
        x, h1, h2, h3, f, e, ie, am = ctx
        B = x.shape[0]
        with torch.no_grad():
            hf = h3.view(B, -1)
            a, fc = self.actor[0], self.feature_extractor[7]
            dout = dout.contiguous()
            heads = [(self.extra_layer[0], self.critic_ext, e, dv)]
            if self.intrinsic:
                heads.append((self.int_extra_layer[0], self.critic_int, ie, div))
            import convs as _convs
            side = _convs.side_stream(dout.device) if _convs.BWD_STREAMS and dout.is_cuda else None
            cur = _convs.current_stream(dout.device) if side is not None else None
            cv = self.conv_impl
            split = cv.split_head_bwd(B)  # the extra layer's dgrad / weight gradient on the split-f16 kernels
            des = []
            # FORK_MERGE: the hidden layers' weight gradients go to the side stream with the fc weight
            # gradient's fork (one event record on the main stream fewer) instead of a fork of their own
            merge = (side is not None and _convs.FORK_MERGE and split and cv.nhwc3
                     and B >= _convs.FC_WGRAD_SPLIT_MIN_BATCH)
            deferred = []
            # round 5: with the split hidden layer and no intrinsic head, the actor's input grad, the critic's
            # ReLU-layer grad and the hidden layer's dgrad (fc ReLU applied) in one launch (ppox_head_backward)
            # (the kernel reads w_actor as 16-B vectors; w_critic, whose flat-buffer offset depends on the action
            # count, by dwords)
            fused = (split and not self.intrinsic and HEAD_BWD_FUSED and dout.shape[1] <= 8
                     and a.weight.is_contiguous() and a.weight.data_ptr() % 16 == 0)
            if fused:
                df, de0 = torch.empty_like(f), torch.empty_like(e)
                native.head_backward(dout, a.weight, dv.contiguous().view(B), self.critic_ext.weight, e, f, cv.qh[1],
                                     df, de0, am[_convs.AM_DE], am[_convs.AM_DF])
            else:
                # the actor head's input grad and the extra layer's dv * w_critic * ReLU' in one launch
                df, de0 = native.head_dgrad_outer(dout, a.weight, dv.contiguous().view(B), self.critic_ext.weight, e,
                                                  amax_de=am[_convs.AM_DE] if split else None)
            for hid, crit, act, d in heads:
                d = d.contiguous().view(B, 1)
                sp = split and hid is self.extra_layer[0]
                if hid is self.extra_layer[0]:
                    de = de0
                else:
                    de = torch.empty_like(act)
                    native.outer_relu_backward(d, crit.weight, act, de)  # dv * w, ReLU'
                if merge and sp:
                    deferred.append((de, hid))
                else:
                    if side is not None:  # the hidden layer's weight gradient beside the dgrad chain
                        _convs.fork(side, cur)
                    with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
                        if sp:
                            native.head_hidden_wgrad(de, f, self._head_wgrad_ws(B), hid.weight.grad,
                                                     amax_de=am[_convs.AM_DE], amax_f=am[_convs.AM_F])
                        else:
                            weight_grad(de, f, hid.weight.grad, self._wgrad_part(hid.weight))
                if not sp:
                    df.addmm_(de, hid.weight)
                des.append((de, d))
            if split and not fused:  # df = (f > 0) ? df + de W : 0, recording df's amax (the fc layer's operand)
                native.head_hidden_dgrad(des[0][0], cv.qh[1], f, df, amax_de=am[_convs.AM_DE], amax_df=am[_convs.AM_DF])
            # every column-reduction gradient (actor W/b, critic W/b, extra-layer b, fc b) in one pass; without
            # the split hidden layer it first applies the fc ReLU's backward to df (in place, df's amax recorded)
            ws = self._head_ws(B, f.shape[1], dout.shape[1])
            (de, d), intr = des[0], des[1] if self.intrinsic else (None, None)
            dfp = None
            if cv.px_df(B) and isinstance(am, _convs.PassState):  # df's planes for the fc dgrad and weight gradient
                am.px[_convs.EX_DF] = True
                dfp = torch.empty((B, 2 * f.shape[1]), dtype=torch.int16, device=df.device)
            # with the split hidden layer df is final here (its amax recorded by the heads' backward): its planes are
            # written by the same pass (round 6; the separate ppox_px_split otherwise, after the fc ReLU's backward)
            fuse_px = dfp is not None and split
            native.head_grads(f, e, dout, d, de, df, ws, a.weight.grad, a.bias.grad, self.critic_ext.weight.grad,
                              self.critic_ext.bias.grad, self.extra_layer[0].bias.grad, fc.bias.grad,
                              ie=ie, div=intr[1], die=intr[0],
                              w_critic_int=self.critic_int.weight.grad if self.intrinsic else None,
                              b_critic_int=self.critic_int.bias.grad if self.intrinsic else None,
                              b_int_extra=self.int_extra_layer[0].bias.grad if self.intrinsic else None,
                              relu_df=not split, amax_df=am[_convs.AM_DF] if (cv.nhwc3 and not split) else None,
                              df_planes=dfp if fuse_px else None, df_planes_amax=am[_convs.AM_DF] if fuse_px else None,
                              df_planes_exp=am.exp(_convs.EX_DF) if fuse_px else None)
            if dfp is not None and not fuse_px:
                native.px_split(df, am[_convs.AM_DF], dfp, am.exp(_convs.EX_DF))
            if cv._diag is not None:  # (tests: the backward's intermediates)
                cv._diag.update(df=df, dfp=dfp, de=de0)
            if cv.nhwc3 and B >= _convs.FC_WGRAD_SPLIT_MIN_BATCH:  # split-f16 kernel, Flatten-order dW
                h3_exp = am.exp(_convs.EX_H3)  # (PX h3: its planes)
                df_exp = am.exp(_convs.EX_DF) if dfp is not None else None
                dfw = dfp if dfp is not None else df
                if side is None:
                    native.nature_fc_wgrad(dfw, B, h3, self._fc_wgrad_ws(B), fc.weight.grad, amax_df=am[_convs.AM_DF],
                                           amax_h3=am[_convs.AM_H3], h3_exp=h3_exp, df_exp=df_exp)
                    if dense_ready is not None:
                        dense_ready()
                else:
                    # on the side stream, beside the fc dgrad and the conv backward; the dense
                    # gradients' all-reduce is started from there (ordered after it and, through the
                    # fork, after every head gradient); backward_acts joins the side stream
                    _convs.fork(side, cur)
                    for de_, hid_ in deferred:
                        native.head_hidden_wgrad(de_, f, self._head_wgrad_ws(B), hid_.weight.grad,
                                                 amax_de=am[_convs.AM_DE], amax_f=am[_convs.AM_F], stream=side)
                    native.nature_fc_wgrad(dfw, B, h3, self._fc_wgrad_ws(B), fc.weight.grad, amax_df=am[_convs.AM_DF],
                                           amax_h3=am[_convs.AM_H3], h3_exp=h3_exp, df_exp=df_exp, stream=side)
                    if dense_ready is not None:
                        with torch.cuda.stream(side):
                            dense_ready()
            else:
                if cv.nhwc3:  # NHWC features: library GEMM in NHWC order, permuted back to Flatten order
                    dwp = self._fc_grad_buf(fc.weight)
                    torch.mm(df.t(), hf, out=dwp)
                    fc.weight.grad.view(fc.weight.shape[0], 64, 49).copy_(dwp.view(-1, 49, 64).transpose(1, 2))
                else:
                    torch.mm(df.t(), hf, out=fc.weight.grad)
                if side is not None:
                    _convs.join(side, cur)  # the hidden-layer weight gradients, before their all-reduce
                if dense_ready is not None:
                    dense_ready()
            fe = self.feature_extractor
            if cv.nhwc3 and B < _convs.FC_DGRAD_FUSED_MAX_BATCH:  # masked NHWC grad directly
                dh3, g3 = None, cv.fc_dgrad_g3(df, h3, am, dfp)
            elif cv.nhwc3:  # library GEMM on the permuted weight: NHWC order, then the ReLU mask
                torch.index_select(fc.weight, 1, cv.fc_perm, out=cv.wfc_nhwc)
                g3 = torch.mm(df, cv.wfc_nhwc).view(B, 7, 7, 64)
                native.relu_backward_(g3, h3, amax=am[_convs.AM_G3])
                dh3 = None
            else:
                dh3, g3 = torch.mm(df, fc.weight), None
            # conv grads are written by the trunk kernels; the flat buffer was zeroed per minibatch
            self.conv_impl.backward_acts(x, h1, h2, h3, dh3, fe[0].weight.grad, fe[0].bias.grad, fe[2].weight.grad,
                                         fe[2].bias.grad, fe[4].weight.grad, fe[4].bias.grad, g3=g3, am=am)


class RndNetwork(nn.Module):
    """models.py:216-267: predictor 3 hidden (LeakyReLU, LeakyReLU, ELU) -> 1,
    target 2 hidden -> 1, constant init (target W=0.01 b=1; predictor W=1 b=0.01)."""

    def __init__(self, input_size, hidden_size=32):
        super().__init__()
        self.predictor = nn.Sequential(
            nn.Linear(input_size, hidden_size), nn.LeakyReLU(), nn.Linear(hidden_size, hidden_size), nn.LeakyReLU(),
            nn.Linear(hidden_size, hidden_size), nn.ELU(), nn.Linear(hidden_size, 1))
        self.target = nn.Sequential(
            nn.Linear(input_size, hidden_size), nn.LeakyReLU(), nn.Linear(hidden_size, hidden_size), nn.LeakyReLU(),
            nn.Linear(hidden_size, 1))
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
        return (p - t).pow(2).squeeze(-1)


class IntrinsicCuriosityModule(nn.Module):
    """models.py:270-320."""

    def __init__(self, input_size, action_converter, hidden_size):
        super().__init__()
        self.action_converter = action_converter
        self.discrete = action_converter.action_type == "Discrete"
        self.feature_size = hidden_size
        self.n_actions = action_converter.num_actions
        self.state_encoder = nn.Sequential(nn.Linear(input_size, hidden_size), nn.LeakyReLU(),
                                           nn.Linear(hidden_size, hidden_size))
        self.forward_model = nn.Sequential(nn.Linear(self.n_actions + hidden_size, hidden_size), nn.LeakyReLU(),
                                           nn.Linear(hidden_size, hidden_size))
        self.inverse_model = nn.Sequential(nn.Linear(2 * hidden_size, hidden_size), nn.LeakyReLU(),
                                           nn.Linear(hidden_size, self.n_actions))
        if self.discrete:
            self.action_encoder = nn.Embedding(self.n_actions, self.n_actions)
        else:
            self.action_encoder = nn.Linear(self.n_actions, self.n_actions)
        orthogonal_init(self)

    def encode_action(self, a):
        if self.discrete:
            # nn.Embedding's lookup as one_hot(a) @ W: the same rows exactly (1 * w + exact zeros),
            # and a GEMM for the weight gradient (torch's embedding backward kernel on ROCm took
            # 193 us per minibatch of 2048 rows, 16 % of a per-rank PPO_ICM iteration)
            W = self.action_encoder.weight
            return F.one_hot(a.reshape(-1).long(), self.n_actions).to(W.dtype) @ W
        return self.action_encoder(a.float())

    def forward(self, state, next_state, action):
        """models.py:300-309 -> (action_hat, next_state_hat, next_state_ft)."""
        ae = self.encode_action(action)
        f = self.state_encoder(state)
        fn = self.state_encoder(next_state).view(-1, self.feature_size)
        return self.inverse_model(torch.cat((f, fn), 1)), self.forward_model(torch.cat((f, ae), 1)), fn

    def int_reward(self, state, next_state, action):
        """models.py:311-320: clamp(mean((phi_hat(s,a) - phi(s'))^2), -5, 5)."""
        return self.int_reward_features(self.state_encoder(state), self.state_encoder(next_state), action)

    def int_reward_features(self, f, fn, action):
        """int_reward from already encoded phi(s), phi(s') (the collect loop encodes each
        observation once: s_{t+1} of step t is s_t of step t + 1)."""
        ae = self.encode_action(action)
        nh = self.forward_model(torch.cat((f, ae), 1))
        return torch.clamp((nh - fn).pow(2).mean(dim=-1), -5, 5)


class FlatParams:
    """Re-homes a module's trainable parameters into one contiguous f32 device
    buffer (+ gradient and Adam moment buffers of the same layout).  Autograd
    accumulates straight into the flat gradient buffer."""

    def __init__(self, module, device="cuda"):
        self.module = module
        self.device = torch.device(device)
        self.params = [p for p in module.parameters() if p.requires_grad]
        frozen = [p for p in module.parameters() if not p.requires_grad]
        sizes = [p.numel() for p in self.params]
        self.n = int(sum(sizes))
        npad = (self.n + 63) // 64 * 64
        self.data = torch.zeros(npad, device=self.device)
        self.grad = torch.zeros(npad, device=self.device)
        self.exp_avg = torch.zeros(npad, device=self.device)
        self.exp_avg_sq = torch.zeros(npad, device=self.device)
        self.norm_partials = torch.zeros(native.NORM_PARTIALS, dtype=torch.float64, device=self.device)
        off = 0
        with torch.no_grad():
            for p in self.params:
                k = p.numel()
                self.data[off:off + k].copy_(p.detach().reshape(-1))
                p.data = self.data[off:off + k].view(p.shape)
                p.grad = self.grad[off:off + k].view(p.shape)
                off += k
            for p in frozen:
                p.data = p.data.to(self.device)
        for b in module.buffers():
            b.data = b.data.to(self.device)
        self.step_count = 0
        # the NatureCNN weight packing whose amax pass the Adam step records (convs.WmaxLink; round 6)
        self.wmax = None

    def zero_grad(self):
        self.grad.zero_()

    def adam_step(self, lr, max_grad_norm, betas=(0.9, 0.999), eps=1e-8):
        """clip_grad_norm_(max_grad_norm) + Adam.step (ppo.py:243-244)."""
        self.step_count += 1
        if max_grad_norm is not None and max_grad_norm > 0:
            native.grad_sumsq(self.grad, self.norm_partials)
        lk = self.wmax
        if lk is not None and lk.ready(self):
            native.adam_step_wmax(self.data, self.grad, self.exp_avg, self.exp_avg_sq, self.norm_partials,
                                  max_grad_norm if max_grad_norm else 0.0, lr, betas[0], betas[1], eps,
                                  self.step_count, lk.ranges, lk.recording())
            lk.recorded(self)
        else:
            native.adam_step(self.data, self.grad, self.exp_avg, self.exp_avg_sq, self.norm_partials,
                             max_grad_norm if max_grad_norm else 0.0, lr, betas[0], betas[1], eps, self.step_count)

    def state_dict(self):
        return {k: v.detach() for k, v in self.module.state_dict().items()}
