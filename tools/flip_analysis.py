"""Where the heads' first-minibatch gradient error comes from in the 16,384-row reference fixture
(tests/golden/train_cnn_big.npz).  CPU only, oracle arithmetic (test infrastructure):
the first minibatch forward + loss backward in float32 (torch-CPU, the reference's own arithmetic) and in
float64, with every ReLU's pre-activation recorded, then
  * the ReLU decisions that differ between the two (per layer),
  * the float64 gradient recomputed with the float32 run's ReLU decisions ("own masks"),
  * for each differing decision of the heads' hidden layer, its share of the extra layer's gradient.
  python tools/flip_analysis.py [threads] [--write]
--write records the reference's own decomposition as tests/golden/train_cnn_big_flips.npz (per tensor the max
|g32 - g64(f32 masks)| and |g64(f32 masks) - g64| relative to the tensor's largest float64 entry; the ReLU
decisions that differ per layer): the oracle's float32 pass here is the reference's arithmetic bitwise (pinned
against the fixture's recorded g32 above), so this is the reference run's own error, split into its parts, that
tests/test_product_gpu.py holds the product's split against.
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import models as OM  # noqa: E402
from oracle.algos import _tensors, ppo_loss  # noqa: E402
from oracle.philox import SyntheticAtari  # noqa: E402
from oracle.storage import Rollout  # noqa: E402


def frames(f, p, N, T, A, env_seed):
    env = SyntheticAtari(N, env_seed, n_actions=A, p_done=float(f[p + "p_done"]))
    obs = np.empty((T, N, 4, 84, 84), np.uint8)
    o = env.reset()
    for t in range(T):
        obs[t] = o
        o = env.step(f[p + "roll_actions"][t].reshape(N))[0]
    return obs


def first_minibatch(f, p, obs, dt, masks=None):
    """(loss grads by parameter name, pre-activations of the 5 ReLUs, v, logits) of minibatch 0 in dtype dt;
    masks: use these ReLU decisions instead of the dtype's own"""
    N, T, B, E_, A, seed, net_seed, env_seed = (int(x) for x in f[p + "cfg"])
    np.random.seed(seed)
    ro = Rollout(T, N, (4, 84, 84), 1)
    ro.obs[:] = obs
    ro.actions[:] = f[p + "roll_actions"].reshape(ro.actions.shape)
    ro.rewards[:], ro.values[:], ro.masks[:] = f[p + "roll_rewards"], f[p + "roll_values"], f[p + "roll_masks"]
    ro.log_probs[:] = f[p + "roll_action_log_probs"].reshape(ro.log_probs.shape)
    ro.pos = T
    ro.finish(f[p + "roll_values"][T - 1], f[p + "roll_masks"][T - 1])
    idx, mb = next(ro.minibatches(B))
    mb = _tensors(mb, dt)
    net = OM.NatureCNN(4, A).to(dt)
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.from_numpy(f[p + "init_" + k]).to(dt))
    fe = net.feature_extractor
    pre = []

    def act(z, i):
        pre.append(z.detach())
        return F.relu(z) if masks is None else z * masks[i].to(dt)
    x = mb["observations"].to(dt)
    h = act(fe[0](x), 0)
    h = act(fe[2](h), 1)
    h = act(fe[4](h), 2)
    fo = act(fe[7](h.flatten(1)), 3)
    logits = net.actor(fo)
    e = act(net.extra_layer[0](fo), 4)
    v = net.critic_ext(e).squeeze()
    dist = OM.categorical(logits)
    lp = dist.log_prob(mb["actions"].flatten()).unsqueeze(1)
    loss = ppo_loss(v, lp, dist.entropy(), mb, 0.2, 0.01, 1.0)[0]
    loss.backward()
    grads = {k: q.grad.detach().double().clone() for k, q in net.named_parameters()}
    return grads, pre, v.detach().double(), logits.detach().double(), idx


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    torch.set_num_threads(int(args[0]) if args else os.cpu_count())
    f = np.load(os.path.join(ROOT, "tests", "golden", "train_cnn_big.npz"))
    p = "big_"
    N, T, B, E_, A, seed, net_seed, env_seed = (int(x) for x in f[p + "cfg"])
    obs = frames(f, p, N, T, A, env_seed)
    g32, pre32, v32, l32, idx = first_minibatch(f, p, obs, torch.float32)
    g64, pre64, v64, l64, _ = first_minibatch(f, p, obs, torch.float64)
    # pin: this recomputation is the fixture's (sampled entries)
    for key in ("extra_layer.0.weight", "feature_extractor.0.weight"):
        i = f[p + "w1idx_" + key]
        for tag, g in (("g32_", g32), ("g64_", g64)):
            d = np.abs(g[key].flatten().numpy()[i] - f[p + tag + key]).max() / np.abs(f[p + tag + key]).max()
            print(f"pin {tag}{key}: max rel diff vs fixture {d:.2e}")
    names = ["conv1", "conv2", "conv3", "fc (f)", "hidden (e)"]
    m32 = [(z > 0) for z in pre32]
    for n, a, b in zip(names, m32, pre64):
        diff = a != (b > 0)
        print(f"ReLU decisions f32 != f64 in {n}: {int(diff.sum())} of {diff.numel()}")
    g64own, _, _, _, _ = first_minibatch(f, p, obs, torch.float64, masks=m32)
    for key in g64:
        s = g64[key].abs().max()
        print(f"{key}: |g32 - g64| {float((g32[key] - g64[key]).abs().max() / s):.3g}  "
              f"|g32 - g64(f32 masks)| {float((g32[key] - g64own[key]).abs().max() / s):.3g}  "
              f"|g64(f32 masks) - g64| {float((g64own[key] - g64[key]).abs().max() / s):.3g}")
    # one hidden-unit flip's share of the extra layer's weight gradient: row j gains de[b, j] f[b, :]
    e64 = pre64[4]
    d = (m32[4] != (e64 > 0)).nonzero().tolist()
    gw = g64["extra_layer.0.weight"]
    print("hidden flips (row b, unit j, pre-activation f64, f32):")
    for b, j in d[:20]:
        print(f"  {b} {j} {float(e64[b, j]):.3e} {float(pre32[4][b, j]):.3e}")
    print(f"max |extra_layer.0.weight grad| (f64) {float(gw.abs().max()):.4g}; 2/B = {2 / B:.3g}")
    if "--write" in sys.argv:
        out = {"flips": np.array([int((a != (b > 0)).sum()) for a, b in zip(m32, pre64)], np.int64)}
        for key in g64:
            s_ = g64[key].abs().max()
            out["arith_" + key] = np.float64((g32[key] - g64own[key]).abs().max() / s_)
            out["relu_" + key] = np.float64((g64own[key] - g64[key]).abs().max() / s_)
        path = os.path.join(ROOT, "tests", "golden", "train_cnn_big_flips.npz")
        np.savez(path, **out)
        print("wrote", path)


if __name__ == "__main__":
    main()
