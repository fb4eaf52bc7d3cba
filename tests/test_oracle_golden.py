"""The oracle pinned against the reference's own code (tests/golden, made by
oracle/make_golden.py from /root/reference): n-step targets, the frame-stack /
auto-reset / episode-info semantics, and the MultiEnvAgent layout."""
import json
import os
import sys
import zlib

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, 'golden')
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'oracle'))
import oracle  # noqa: E402


def _returns_cases():
    d = np.load(os.path.join(GOLD, 'returns.npz'))
    meta = json.loads(str(d['meta']))
    for i, m in enumerate(meta):
        yield m, {k[len('c{}_'.format(i)):]: d[k] for k in d.files if k.startswith('c{}_'.format(i))}


def test_gamma_tables_are_the_reference_matrices_bit_for_bit():
    for m, c in _returns_cases():
        gp, bp = oracle.gamma_tables(0.99, m['T'])
        D, bf = c['D'], c['boot_factors']
        for n in range(m['N']):
            for i in range(m['T']):
                for j in range(i + 1):
                    if D[n, i, j] != 0:
                        assert D[n, i, j] == gp[i - j]
            for t in range(m['T']):
                if bf[n, t] != 0:
                    assert bf[n, t] == bp[m['T'] - t]
                    assert not c['terminals'][n, t:].any()
                else:
                    assert c['terminals'][n, t:].any()


def test_targets_f32_within_4ulp_of_reference_closures():
    # tolerance: <= 4 ulp of max |target| against the reference closures
    # with np.matmul standing in for tf.matmul
    for m, c in _returns_cases():
        got = oracle.targets_f32(c['rewards'], c['terminals'], c['v_boot'], 0.99)
        ref = c['targets_f32']
        ulp = np.spacing(np.float32(np.abs(ref).max()))
        assert np.abs(got - ref).max() <= 4 * ulp, m
        exact = oracle.targets_f64(c['rewards'], c['terminals'], c['v_boot'], 0.99)
        assert np.abs(exact - c['targets_f64']).max() <= 1e-4 * max(1.0, np.abs(exact).max())


def test_framestack_autoreset_trace_matches_reference_wrappers():
    rec = json.load(open(os.path.join(GOLD, 'framestack_autoreset.json')))
    for e in rec['envs']:
        r = rec['env{}'.format(e)]
        env = oracle.SyntheticAtari(rec['seed'], e)
        o = env.reset()
        assert zlib.crc32(o.tobytes()) == r['crc'][0]
        saw_terminal = False
        kept = np.load(os.path.join(GOLD, 'framestack_env{}.npz'.format(e)))
        for t, a in enumerate(r['actions']):
            o, rw, d, ep = env.step(a)
            assert zlib.crc32(o.tobytes()) == r['crc'][t + 1], t
            assert rw == r['rewards'][t] and d == r['terminals'][t]
            key = 'obs_t{}'.format(t + 1)
            if key in kept.files:
                np.testing.assert_array_equal(o, kept[key])
            if d:
                saw_terminal = True
                # terminal observation is [0, 0, 0, frame] (wrappers.py:226-229)
                assert not o[..., :3].any()
        assert saw_terminal


def test_episode_rewards_match_reference_info_batch():
    rec = json.load(open(os.path.join(GOLD, 'framestack_autoreset.json')))
    ep_ref = rec['episode_rewards']
    for row, e in zip(ep_ref, rec['envs']):
        env = oracle.SyntheticAtari(rec['seed'], e)
        env.reset()
        for t, a in enumerate(rec['env{}'.format(e)]['actions']):
            _, _, _, ep = env.step(a)
            if row[t] is None:
                assert np.isnan(ep)
            else:
                assert ep == pytest.approx(row[t])


def test_agent_layout_matches_reference(monkeypatch):
    from actorcritic.agents import MultiEnvAgent, transpose_list
    gold = json.load(open(os.path.join(GOLD, 'agent_layout.json')))
    assert transpose_list([[1, 2, 3, 4], [5, 6, 7, 8], [9, 10, 11, 12]]) == gold['transpose_list']

    class FakeMultiEnv:
        batched = None

        def __init__(self, n):
            self.n, self.t = n, 0

        def reset(self):
            return ['obs(e{},t0)'.format(e) for e in range(self.n)]

        def step(self, actions):
            self.t += 1
            obs = ['obs(e{},t{})'.format(e, self.t) for e in range(self.n)]
            return obs, [float(a) for a in actions], [a % 3 == 0 for a in actions], [{'a': a} for a in actions]

    class FakeModel:
        def __init__(self):
            self.batches = []

        def sample_actions(self, batch, session):
            self.batches.append(batch)
            return [10 * i + len(self.batches) for i in range(len(batch))]

    model = FakeModel()
    agent = MultiEnvAgent(FakeMultiEnv(3), model, 4)
    first = [list(x) for x in agent.interact(None)]
    second = [list(x) for x in agent.interact(None)]
    assert json.loads(json.dumps(model.batches)) == gold['sample_batches']
    assert json.loads(json.dumps(first)) == gold['first']
    assert json.loads(json.dumps(second)) == gold['second']


def test_single_env_agent_matches_reference():
    """SingleEnvAgent.interact (agents.py:50-131) against the reference class run on
    the same fakes: [[obs]] sample batches, [1, steps] outputs, [next_obs], and the
    last observation carried into the next call (no reset in between)."""
    from actorcritic.agents import SingleEnvAgent
    gold = json.load(open(os.path.join(GOLD, 'agent_layout.json')))

    class FakeEnv:
        def __init__(self):
            self.t, self.resets = 0, 0

        def reset(self):
            self.resets += 1
            return 'obs(r{},t{})'.format(self.resets, self.t)

        def step(self, action):
            self.t += 1
            return 'obs(r{},t{})'.format(self.resets, self.t), 0.5 * action, action % 2 == 1, {'t': self.t}

    class FakeModel:
        def __init__(self):
            self.batches = []

        def sample_actions(self, batch, session):
            self.batches.append(batch)
            return [10 * i + len(self.batches) for i in range(len(batch))]

    model = FakeModel()
    agent = SingleEnvAgent(FakeEnv(), model, 3)
    first = [list(x) for x in agent.interact(None)]
    second = [list(x) for x in agent.interact(None)]
    assert json.loads(json.dumps(model.batches)) == gold['single_sample_batches']
    assert json.loads(json.dumps(first)) == gold['single_first']
    assert json.loads(json.dumps(second)) == gold['single_second']


def test_gae_lambda1_reduces_to_reference_targets():
    """GAE(lambda = 1) targets equal the reference's n-step targets (exact
    arithmetic; float32 differs by rounding of the telescoping V terms): pins the
    GAE restatement (an option beyond the reference) at lambda = 1."""
    rng = np.random.default_rng(3)
    for m, c in _returns_cases():
        v = rng.normal(0, 1, size=(m['N'], m['T'])).astype(np.float32)
        tg, adv = oracle.gae_f32(c['rewards'], c['terminals'], v, c['v_boot'], 0.99, 1.0)
        ref = c['targets_f32']
        scale = max(1.0, np.abs(ref).max(), np.abs(v).max())
        assert np.abs(tg - ref).max() <= 4 * m['T'] * np.spacing(np.float32(scale)), m
        assert np.array_equal(adv, (tg - v).astype(np.float32)) or np.abs(adv - (tg - v)).max() <= 2 * np.spacing(
            np.float32(scale))


@pytest.mark.parametrize('lam', [0.0, 0.5, 0.95])
def test_gae_f32_matches_float64(lam):
    rng = np.random.default_rng(7)
    N, T = 6, 20
    r = rng.choice([-1.0, 0.0, 1.0], size=(N, T)).astype(np.float32)
    d = rng.random((N, T)) < 0.1
    d[0, 0] = d[1, T - 1] = True
    d[2, :] = True
    v = rng.normal(0, 1, size=(N, T)).astype(np.float32)
    vb = rng.normal(0, 1, size=N).astype(np.float32)
    t32, a32 = oracle.gae_f32(r, d, v, vb, 0.99, lam)
    t64, a64 = oracle.gae_f64(r, d, v, vb, 0.99, lam)
    assert np.abs(a32 - a64).max() <= 1e-5 * max(1.0, np.abs(a64).max())
    assert np.abs(t32 - t64).max() <= 1e-5 * max(1.0, np.abs(t64).max())
    # lambda = 0: one-step TD error; an all-terminal row is r - V
    if lam == 0.0:
        assert np.allclose(a64[2], r[2] - v[2])


def test_normalize_advantages_moments():
    a = np.random.default_rng(1).normal(3.0, 2.0, size=1000)
    n = oracle.normalize_advantages(a)
    assert abs(n.mean()) < 1e-12 and abs(n.std() - 1.0) < 1e-6
