"""ES-NSRA (evolution_strategies.py): oracle vs the reference's recorded outputs (CPU),
device kernels and the EvolutionStrategy class vs the oracle (GPU)."""
import numpy as np
import pytest
import torch

from oracle import es as O


@pytest.fixture(scope="module")
def golden():
    import os
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "es.npz"))


def test_oracle_predict_matches_reference(golden):
    w = [golden["pred_w0"], golden["pred_w1"], golden["pred_w2"]]
    np.testing.assert_allclose(O.predict(w, golden["pred_obs"]), golden["pred_act"], rtol=0, atol=1e-14)


@pytest.mark.parametrize("tag", ["a", "b"])
def test_oracle_update_matches_reference(golden, tag):
    meta = golden[f"upd_{tag}_meta"]
    wb = [golden[f"upd_{tag}_w{i}_before"] for i in range(3)]
    pops = [golden[f"upd_{tag}_pop{i}"] for i in range(3)]
    new = O.update_weights(wb, pops, golden[f"upd_{tag}_rewards"], meta[0], meta[1], meta[2], int(meta[3]), meta[4])
    for i in range(3):  # bit-exact: same numpy program
        assert np.array_equal(new[i], golden[f"upd_{tag}_w{i}_after"])


def test_oracle_knn_and_probs_match_reference(golden):
    for n in (1, 3, 10, 57):
        d = O.knn_distance(golden[f"knn_{n}_archive"], golden[f"knn_{n}_bc"], min(10, n))
        assert abs(d - float(golden[f"knn_{n}_dist"])) <= 1e-12 * max(1.0, abs(d))
    assert O.novelty_probs(list(golden["probs_in"])) == list(golden["probs_out"])


# ---------------------------------------------------------------------------- GPU
def _es(P=24, hidden=(16, 12), T=40, seed=3):
    import evolution_strategies as ES
    np.random.seed(seed)
    return ES.EvolutionStrategy("Swimmer-v3", hidden_sizes=list(hidden), population_size=P, sigma=0.1,
                                learning_rate=0.01, seed=seed, episode_len=T)


@pytest.mark.gpu
def test_es_noise_matches_oracle_and_shards():
    import native
    P, n = 37, 301
    eps = torch.empty(P, n, dtype=torch.float64, device="cuda")
    native.es_noise(P, n, 0, 5, 77, eps)
    ref = O.perturbations(77, 5, np.arange(P), n)
    np.testing.assert_allclose(eps.cpu().numpy(), ref, rtol=1e-13, atol=1e-13)
    part = torch.empty(10, n, dtype=torch.float64, device="cuda")
    native.es_noise(10, n, 20, 5, 77, part)        # members 20..29 of the same generation
    assert torch.equal(part, eps[20:30])


@pytest.mark.gpu
@pytest.mark.parametrize("hidden", [(16, 12), (64, 64)])
def test_es_evaluate_matches_oracle(hidden):
    es = _es(P=6, hidden=hidden, T=30)
    eps = es._get_population()
    fit, bc = es._evaluate_dev(es.weights, eps, eps.shape[0], bc=True)
    e = eps.cpu().numpy()
    members = []
    for p in range(6):
        off, ws = 0, []
        for w in es.weights:
            ws.append(w + es.SIGMA * e[p, off:off + w.size].reshape(w.shape))
            off += w.size
        members.append(ws)
    f_ref, b_ref = O.evaluate(members, es.env_seed, 30)
    np.testing.assert_allclose(fit.cpu().numpy(), f_ref, rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(bc.cpu().numpy(), b_ref, rtol=1e-10, atol=1e-10)


@pytest.mark.gpu
def test_es_device_update_matches_reference_rule():
    es = _es(P=40)
    eps = es._get_population()
    rewards = np.random.RandomState(1).randn(40) * 2 + 0.5
    before = [w.copy() for w in es.weights]
    es.novelty_param = 0.3
    es._update_weights(rewards, eps, 0.42)
    e = eps.cpu().numpy()
    pops, off = [], 0
    for w in before:
        pops.append(e[:, off:off + w.size].reshape(40, *w.shape))
        off += w.size
    ref = O.update_weights(before, pops, rewards, 0.42, 0.3, 0.01, 40, 0.1)
    for a, b in zip(es.weights, ref):
        np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-14)
    assert abs(es.learning_rate - 0.01 * 0.9995) < 1e-18


@pytest.mark.gpu
def test_es_class_host_pieces_match_reference(golden):
    """The class's reference-format _update_weights / get_kNN / probabilities reproduce the
    reference's recorded outputs."""
    es = _es(P=40, hidden=(16, 12))
    meta = golden["upd_a_meta"]
    es.weights = [golden[f"upd_a_w{i}_before"].copy() for i in range(3)]
    es.novelty_param, es.learning_rate = meta[1], meta[2]
    pop = [[golden[f"upd_a_pop{i}"][p] for i in range(3)] for p in range(40)]
    es._update_weights(golden["upd_a_rewards"], pop, meta[0])
    for i in range(3):
        assert np.array_equal(es.weights[i], golden[f"upd_a_w{i}_after"])
    for n in (3, 57):
        arch = [golden[f"knn_{n}_archive"][i:i + 1] for i in range(n)]
        assert abs(es.get_kNN(arch, golden[f"knn_{n}_bc"], min(10, n)) - float(golden[f"knn_{n}_dist"])) < 1e-12
    assert es.calc_noveltiy_distribution(list(golden["probs_in"])) == list(golden["probs_out"])


@pytest.mark.gpu
def test_es_gradient_steps_improve_fitness():
    """Plain ES steps (novelty=None branch of :243-244) on the device raise the fitness."""
    es = _es(P=256, hidden=(32, 32), T=60, seed=2)
    es.weights = [w * 0.3 for w in es.weights]  # start away from the optimum (|B a| -> 2)
    es.learning_rate = 0.05
    f0 = es.evaluate(es.weights)
    for g in range(8):
        es.generation = g
        pop = es._get_population()
        es._update_weights(es._get_rewards(None, pop), pop, None)
    assert es.evaluate(es.weights) > f0 + 10.0


@pytest.mark.gpu
def test_es_run_smoke():
    es = _es(P=128, hidden=(32, 32), T=40, seed=4)
    es.run(6, log_interval=100)
    assert len(es.rewards) == 6 and np.isfinite(list(es.rewards)).all()
    assert 0.0 <= es.novelty_param <= 1.0
