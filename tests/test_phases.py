"""phases.py (SURVEY.md §5 Tracing): ranges nest and return values pass through on a host
without a GPU; the product's phase names are the ones bench.py reports."""
import phases


def test_phase_passthrough_and_nesting():
    phases.enable_timers()

    @phases.traced("outer")
    def f(x):
        with phases.phase("inner"):
            return x + 1

    assert f(1) == 2
    # no GPU here: nothing is recorded, summary() is empty rather than raising
    assert phases.summary() == {} or set(phases.summary()) <= {"outer", "inner"}
    phases.enable_timers(False)
    assert phases.summary() == {}


def test_product_phases_are_traced():
    import buffer
    import ppo
    for cls in (ppo.PPO, ppo.PPO_RND, ppo.PPO_ICM):
        assert cls.collect_samples.__wrapped__ is not None and cls.train.__wrapped__ is not None
    assert buffer.RolloutStorage.compute_returns_and_advantages.__wrapped__ is not None
