"""Float64 re-evaluation of one NatureCNN PPO minibatch for the parity tests (test infrastructure):
the reference's loss (ppo.py:216-238, restated in oracle.algos.ppo_loss) backward through the
checkpoint NatureCNN (models-checkpoint.py:48-90, oracle.models.NatureCNN) in float64, either with its
own ReLU decisions or with the ReLU decisions of a device pass, plus the ReLU decisions that differ.

A pre-activation within a rounding of 0 lands on either side in two f32 computations; each such flip
moves the downstream gradients by a whole term, and is a sign decision, not arithmetic error (round 6:
the reference's own f32 first minibatch of the 16,384-row fixture differs from float64 in 8 / 11 / 7 / 3 /
1 ReLU decisions of conv1 / conv2 / conv3 / fc / the heads' hidden layer, and with those decisions applied
float64 reproduces its gradient to 1.7e-7 of each tensor's largest entry; tools/flip_analysis.py).
"""
import torch
import torch.nn.functional as F

from oracle import models as OM
from oracle.algos import ppo_loss

LAYERS = ("conv1", "conv2", "conv3", "fc", "hidden")
GEO = ((400, 32, 20, 20), (81, 64, 9, 9), (49, 64, 7, 7))


def _unpack_bits(words, B, P, C, H, W):
    """one int32 per 32 channels of a pixel, bit c = channel c > 0 -> (B, C, H, W) bool"""
    w = words.view(B, P, C // 32).long() & 0xFFFFFFFF
    bits = (w.unsqueeze(-1) >> torch.arange(32, device=w.device)) & 1
    return bits.reshape(B, H, W, C).permute(0, 3, 1, 2).bool()


def pass_masks(ctx):
    """The device pass's own ReLU decisions (bool, NCHW / rows, on the device) from its training ctx
    (models.CnnActorCritic.forward_train): the conv layers' from the bitmasks the split forwards wrote,
    else from their f32 activations; fc output f and the hidden layer e from their f32 values."""
    x, h1, h2, h3, f, e, _, am = ctx
    B = x.shape[0]
    out = []
    for i, h in enumerate((h1, h2, h3)):
        P, C, H, W = GEO[i]
        bits = getattr(am, "bits", (None, None, None))[i] if am is not None else None
        if bits is not None:
            out.append(_unpack_bits(bits, B, P, C, H, W))
        elif h.dtype == torch.float32 and tuple(h.shape[1:]) == (C, H, W):
            out.append(h > 0)
        elif h.dtype == torch.float32 and tuple(h.shape[1:]) == (H, W, C):
            out.append((h > 0).permute(0, 3, 1, 2))
        else:
            raise ValueError(f"layer {i + 1}: no bitmask and no f32 activation to read the ReLU from")
    return out + [f > 0, e > 0]


def minibatch_grads(init, x, mb, n_actions, masks=None, dtype=torch.float64, clip=0.2, ent_coef=0.01, vf_coef=1.0):
    """(gradients by parameter name, pre-activations of the 5 ReLUs) of the PPO loss of one minibatch.
    init: the weights (name -> tensor); x (B, 4, 84, 84) frames; mb: the minibatch's fields as tensors
    (advantages (B, 1), returns, old_values, old_log_probs (B, 1), actions (B, 1)); masks: the ReLU
    decisions to apply instead of the dtype's own (pass_masks order)."""
    dev = x.device
    net = OM.NatureCNN(4, n_actions).to(device=dev, dtype=dtype)
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(init[k].to(device=dev, dtype=dtype))
    fe = net.feature_extractor
    pre = []

    def act(z, i):
        pre.append(z.detach())
        return F.relu(z) if masks is None else z * masks[i].to(device=dev, dtype=dtype)
    h = act(fe[0](x.to(dtype)), 0)
    h = act(fe[2](h), 1)
    h = act(fe[4](h), 2)
    fo = act(fe[7](h.flatten(1)), 3)
    logits = net.actor(fo)
    v = net.critic_ext(act(net.extra_layer[0](fo), 4)).squeeze()
    dist = OM.categorical(logits)
    lp = dist.log_prob(mb["actions"].flatten()).unsqueeze(1)
    m = {k: (t.to(device=dev, dtype=dtype) if t.is_floating_point() else t.to(dev)) for k, t in mb.items()}
    loss = ppo_loss(v, lp, dist.entropy(), m, clip, ent_coef, vf_coef)[0]
    loss.backward()
    return {k: q.grad.detach().clone() for k, q in net.named_parameters()}, pre


def flips(masks, pre64):
    """per layer: how many of the pass's ReLU decisions differ from float64's"""
    return {n: int((m.to(p.device) != (p > 0)).sum()) for n, m, p in zip(LAYERS, masks, pre64)}
