"""GPU parity of the HIP path against the oracle (oracle/oracle.py) and the golden
fixtures of the reference (tests/golden).  Everything calls libacmi through the
C-ABI (directly or through the actorcritic API).  Tolerances:
  * integer / byte work (stepper, sampling with given uniforms, schedule): bit-exact,
  * n-step targets: bit-exact vs the float32 oracle, <= 4 ulp vs the reference closures,
  * logits / values / losses: rel 1e-5 (fp32 vs float64),
  * K-FAC factors: rel 2e-5; inverses rel 1e-4; preconditioned gradients rel-L2 <= 1e-3
    (north_star), eigenvalues rel 1e-4.
"""
import ctypes
import json
import os
import sys
import zlib

import numpy as np
import pytest
import torch

from actorcritic import _lib

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, 'golden')
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'oracle'))
import oracle  # noqa: E402

pytestmark = pytest.mark.gpu


def dev(x, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def test_returns_kernel_matches_golden(lib, cuda):
    d = np.load(os.path.join(GOLD, 'returns.npz'))
    meta = json.loads(str(d['meta']))
    for i, m in enumerate(meta):
        c = {k[len('c{}_'.format(i)):]: d[k] for k in d.files if k.startswith('c{}_'.format(i))}
        N, T = m['N'], m['T']
        gp, bp = oracle.gamma_tables(0.99, T)
        r, te, v, vb = dev(c['rewards']), dev(c['terminals'].astype(np.uint8)), dev(c['values']), dev(c['v_boot'])
        gp_d, bp_d = dev(gp), dev(bp)
        tg = torch.zeros(N, T, device=cuda)
        adv = torch.zeros(N, T, device=cuda)
        _lib.call('acmi_returns', _lib.ptr(r), _lib.ptr(te), _lib.ptr(v), _lib.ptr(vb), N, T, _lib.ptr(gp_d),
                  _lib.ptr(bp_d), _lib.ptr(tg), _lib.ptr(adv), _lib.stream_handle())
        got = tg.cpu().numpy()
        mine = oracle.targets_f32(c['rewards'], c['terminals'], c['v_boot'], 0.99)
        np.testing.assert_array_equal(got, mine)  # bit-exact vs the float32 restatement
        ulp = np.spacing(np.float32(np.abs(c['targets_f32']).max()))
        assert np.abs(got - c['targets_f32']).max() <= 4 * ulp, m
        np.testing.assert_array_equal(adv.cpu().numpy(), (got - c['values']).astype(np.float32))


@pytest.mark.parametrize('lam', [0.0, 0.95, 1.0])
def test_gae_kernel_bit_exact_vs_oracle(lib, cuda, lam):
    """acmi_gae (an option beyond the reference) is bit-exact with the float32
    restatement: terminals at t = 0 and T-1, an all-terminal row, none."""
    rng = np.random.default_rng(11)
    N, T = 37, 20
    r = rng.choice([-1.0, 0.0, 1.0], size=(N, T)).astype(np.float32)
    te = rng.random((N, T)) < 0.08
    te[0, 0] = te[1, T - 1] = True
    te[2, :] = True
    te[3, :] = False
    v = rng.normal(0, 1, size=(N, T)).astype(np.float32)
    vb = rng.normal(0, 1, size=N).astype(np.float32)
    tg = torch.zeros(N, T, device=cuda)
    adv = torch.zeros(N, T, device=cuda)
    rd, ted, vd, vbd = dev(r), dev(te.astype(np.uint8)), dev(v), dev(vb)
    _lib.call('acmi_gae', _lib.ptr(rd), _lib.ptr(ted), _lib.ptr(vd), _lib.ptr(vbd), N, T, 0.99, lam,
              _lib.ptr(tg), _lib.ptr(adv), _lib.stream_handle())
    t_ref, a_ref = oracle.gae_f32(r, te, v, vb, 0.99, lam)
    np.testing.assert_array_equal(tg.cpu().numpy(), t_ref)
    np.testing.assert_array_equal(adv.cpu().numpy(), a_ref)


def test_advantage_normalization_matches_oracle(lib, cuda):
    M = 10240 + 37
    a = np.random.default_rng(5).normal(0.3, 2.5, size=M).astype(np.float32)
    ad = dev(a)
    ws = torch.zeros(int(lib.acmi_adv_moments_ws_doubles(M)), dtype=torch.float64, device=cuda)
    mom = torch.zeros(2, dtype=torch.float64, device=cuda)
    _lib.call('acmi_adv_moments', _lib.ptr(ad), M, _lib.ptr(ws), _lib.ptr(mom), _lib.stream_handle())
    m = mom.cpu().numpy()
    assert m[0] == pytest.approx(a.astype(np.float64).sum(), rel=1e-12)
    assert m[1] == pytest.approx((a.astype(np.float64) ** 2).sum(), rel=1e-12)
    _lib.call('acmi_adv_normalize', _lib.ptr(ad), M, _lib.ptr(mom), float(M), 1e-8, _lib.stream_handle())
    ref = oracle.normalize_advantages(a)
    np.testing.assert_allclose(ad.cpu().numpy(), ref, rtol=0, atol=2e-6)


def test_gae_and_normalized_advantages_through_objective(lib, cuda):
    """A2CObjective(gae_lambda=0.95, normalize_advantages=True): targets, advantages
    and the losses match the float64 oracle of the same options."""
    from actorcritic import session as sess
    from actorcritic.objectives import A2CObjective
    N, T = 4, 5
    env, model, agent, obj, gs, opt, op, params = _build(N, T)
    obj2 = A2CObjective(model, gae_lambda=0.95, normalize_advantages=True)
    with sess.Session() as s:
        data = agent.interact(s)
        feed = _feed(model, data)
        tg, adv, pl, bl = s.run([obj2.target_values, obj2.advantage, obj2.policy_loss, obj2.baseline_loss],
                                feed_dict=feed)
    obs, act, rew, term, nxt, _ = data
    full = oracle.forward(params, obs.cpu().numpy().reshape(-1, 84, 84, 4), 4, 32)
    vb = oracle.forward(params, nxt.cpu().numpy(), 4, 32)['value']
    t_ref, a_ref = oracle.gae_f64(rew.cpu().numpy(), term.cpu().numpy(), full['value'].reshape(N, T), vb, 0.99, 0.95)
    a_ref = oracle.normalize_advantages(a_ref)
    scale = max(1.0, np.abs(t_ref).max())
    assert np.abs(tg - t_ref).max() <= 1e-5 * scale
    assert np.abs(adv - a_ref).max() <= 1e-4
    ref = oracle.a2c_loss_and_head_grads(full['logits'], full['value'], act.cpu().numpy().reshape(-1),
                                         t_ref.reshape(-1), adv=a_ref)
    assert pl == pytest.approx(ref['policy_loss'], rel=1e-4, abs=1e-6)
    assert bl == pytest.approx(ref['baseline_loss'], rel=1e-4)


def test_stepper_matches_reference_wrapper_trace(lib, cuda):
    from actorcritic.envs.atari.wrappers import SyntheticAtariEnvs
    rec = json.load(open(os.path.join(GOLD, 'framestack_autoreset.json')))
    envs = rec['envs']
    N = max(envs) + 1
    env = SyntheticAtariEnvs(N, num_actions=4, seed=rec['seed'], env_offset=0)
    obs = env.reset().cpu().numpy()
    for e in envs:
        assert zlib.crc32(obs[e].tobytes()) == rec['env{}'.format(e)]['crc'][0]
    steps = len(rec['env{}'.format(envs[0])]['actions'])
    ep_seen = {e: [] for e in envs}
    for t in range(steps):
        a = np.zeros(N, np.int32)
        for e in envs:
            a[e] = rec['env{}'.format(e)]['actions'][t]
        o, r, d, info = env.step(a)
        o, r, d = o.cpu().numpy(), r.cpu().numpy(), d.cpu().numpy()
        ep = info.episode_rewards.cpu().numpy()[:, 0]
        for e in envs:
            g = rec['env{}'.format(e)]
            assert zlib.crc32(o[e].tobytes()) == g['crc'][t + 1], (e, t)
            assert r[e] == g['rewards'][t] and bool(d[e]) == g['terminals'][t], (e, t)
            ep_seen[e].append(None if np.isnan(ep[e]) else float(ep[e]))
    for row, e in zip(rec['episode_rewards'], envs):
        assert ep_seen[e] == [None if v is None else pytest.approx(v) for v in row]


def test_mixed_game_stepper_matches_oracle(lib, cuda):
    """Atari-57 mixed batch (BASELINE configs[4]): 64 envs, global ids 40.. so the game
    index wraps, 18 actions (illegal ones step as NOOP), 300 steps -- several episodes of
    the short games, auto-resets included -- bit-exact against the oracle envs."""
    from actorcritic.envs.atari.wrappers import ATARI57, SyntheticAtariEnvs
    N, off, seed = 64, 40, 77
    env = SyntheticAtariEnvs(N, num_actions=18, seed=seed, env_offset=off, games='atari57')
    games = [(off + n) % 57 for n in range(N)]
    assert env.games.cpu().tolist() == games
    ref = [oracle.SyntheticAtari(seed, off + n, game=g) for n, g in enumerate(games)]
    o = env.reset().cpu().numpy()
    for n in range(N):
        np.testing.assert_array_equal(o[n], ref[n].reset())
    rng = np.random.default_rng(1)
    n_term = 0
    for t in range(300):
        a = rng.integers(0, 18, N).astype(np.int32)
        ob, r, d, info = env.step(a)
        ob, r, d = ob.cpu().numpy(), r.cpu().numpy(), d.cpu().numpy()
        ep = info.episode_rewards.cpu().numpy()[:, 0]
        for n in range(N):
            rob, rr, rd, rep = ref[n].step(int(a[n]))
            assert zlib.crc32(ob[n].tobytes()) == zlib.crc32(rob.tobytes()), (n, t)
            assert r[n] == rr and bool(d[n]) == rd, (n, t, ATARI57[games[n]])
            assert (np.isnan(ep[n]) and np.isnan(rep)) or ep[n] == rep
            n_term += rd
    assert n_term > 0


def test_mixed_game_rollout_matches_oracle_env(lib, cuda):
    """The fused rollout tail steps mixed games like the standalone stepper."""
    from actorcritic import session as sess
    from actorcritic.agents import MultiEnvAgent
    from actorcritic.envs.atari.model import AtariModel
    from actorcritic.envs.atari.wrappers import SyntheticAtariEnvs
    from actorcritic.multi_env import MultiEnv
    sess.reset_default_graph()
    N, T, A = 6, 8, 18
    env = MultiEnv(SyntheticAtariEnvs(N, num_actions=A, seed=9, env_offset=50, games='atari57'))
    model = AtariModel(env.observation_space, env.action_space, 32, params=oracle.init_params(A, 32, seed=1),
                       random_seed=3)
    agent = MultiEnvAgent(env, model, T)
    with sess.Session() as s:
        obs, act, rew, term, nxt, _ = agent.interact(s)
    o = obs.cpu().numpy()
    for n in range(N):
        ref = oracle.SyntheticAtari(9, 50 + n, game=(50 + n) % 57)
        np.testing.assert_array_equal(o[n, 0], ref.reset())
        for t in range(T):
            ob, r, d, _ = ref.step(int(act[n, t]))
            np.testing.assert_array_equal(o[n, t + 1] if t + 1 < T else nxt[n].cpu().numpy(), ob)
            assert float(rew[n, t]) == r and bool(term[n, t]) == d


def test_sampling_exact_with_given_uniforms_and_calibrated(lib, cuda):
    rng = np.random.default_rng(3)
    B, A = 4096, 6
    logits = (rng.standard_normal((B, A)) * 2).astype(np.float32)
    u = rng.random(B).astype(np.float32)
    lg, ud = dev(logits), dev(u)
    out = torch.zeros(B, dtype=torch.int32, device=cuda)
    bad = torch.zeros(1, dtype=torch.int32, device=cuda)
    _lib.call('acmi_sample_actions', _lib.ptr(lg), A, B, A, 0, 0, 0, _lib.ptr(ud), 0, _lib.ptr(out), _lib.ptr(bad),
              _lib.stream_handle())
    np.testing.assert_array_equal(out.cpu().numpy(), oracle.sample_f32(logits, u))
    # counter RNG: exactly the oracle's uniforms, and calibrated frequencies
    _lib.call('acmi_sample_actions', _lib.ptr(lg), A, B, A, 5, 1, 9, None, 0, _lib.ptr(out), _lib.ptr(bad),
              _lib.stream_handle())
    np.testing.assert_array_equal(out.cpu().numpy(),
                                  oracle.sample_f32(logits, oracle.sample_uniforms(5, 1, 9, B)))
    z = np.zeros((B, A), np.float32)
    _lib.call('acmi_sample_actions', _lib.ptr(dev(z)), A, B, A, 5, 1, 10, None, 0, _lib.ptr(out), _lib.ptr(bad),
              _lib.stream_handle())
    counts = np.bincount(out.cpu().numpy(), minlength=A)
    chi2 = ((counts - B / A) ** 2 / (B / A)).sum()
    assert chi2 < 25.0  # df=5, p ~ 1e-4
    # mode and NaN detection
    _lib.call('acmi_sample_actions', _lib.ptr(lg), A, B, A, 0, 0, 0, None, 1, _lib.ptr(out), _lib.ptr(bad),
              _lib.stream_handle())
    np.testing.assert_array_equal(out.cpu().numpy(), logits.argmax(1))
    logits[7, 2] = np.nan
    _lib.call('acmi_sample_actions', _lib.ptr(dev(logits)), A, B, A, 0, 0, 0, None, 0, _lib.ptr(out),
              _lib.ptr(bad), _lib.stream_handle())
    assert int(bad.item()) == 1 and int(out[7].item()) == -1


def test_a2c_loss_and_categorical_match_oracle(lib, cuda):
    rng = np.random.default_rng(4)
    M, A = 1000, 18
    logits = rng.standard_normal((M, A)).astype(np.float32)
    values = rng.standard_normal(M).astype(np.float32)
    actions = rng.integers(0, A, M).astype(np.int32)
    targets = rng.standard_normal(M).astype(np.float32)
    adv = (targets - values).astype(np.float32)
    ldh = 20
    dhead = torch.zeros(M, ldh, device=cuda)
    ws = torch.zeros(lib.acmi_a2c_loss_ws_floats(M), device=cuda)
    out = torch.zeros(4, device=cuda)
    L, V, AC, TG, AD = dev(logits), dev(values), dev(actions), dev(targets), dev(adv)
    _lib.call('acmi_a2c_loss', _lib.ptr(L), A, _lib.ptr(V), _lib.ptr(AC), _lib.ptr(TG), _lib.ptr(AD), M, A,
              0.01, 0.5, 1.0, _lib.ptr(dhead), ldh, _lib.ptr(ws), _lib.ptr(out), _lib.stream_handle())
    ref = oracle.a2c_loss_and_head_grads(logits, values, actions, targets)
    got = out.cpu().numpy()
    assert got[0] == pytest.approx(ref['policy_loss'], rel=1e-5, abs=1e-7)
    assert got[1] == pytest.approx(ref['baseline_loss'], rel=1e-5)
    assert got[2] == pytest.approx(ref['mean_entropy'], rel=1e-5)
    dh = dhead.cpu().numpy()
    np.testing.assert_allclose(dh[:, :A], ref['dlogits'], rtol=1e-4, atol=1e-9)
    np.testing.assert_allclose(dh[:, A], ref['dvalue'], rtol=1e-5, atol=1e-10)
    assert not dh[:, A + 1:].any()
    ent = torch.zeros(M, device=cuda)
    lp = torch.zeros(M, device=cuda)
    _lib.call('acmi_categorical', _lib.ptr(L), A, M, A, _lib.ptr(AC), _lib.ptr(ent), _lib.ptr(lp),
              _lib.stream_handle())
    np.testing.assert_allclose(ent.cpu().numpy(), oracle.entropy(logits.astype(np.float64)), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(lp.cpu().numpy(),
                               oracle.log_softmax(logits.astype(np.float64))[np.arange(M), actions], rtol=1e-5,
                               atol=1e-6)


def test_first_order_optimizers_match_oracle(lib, cuda):
    rng = np.random.default_rng(6)
    n = 100003
    p = rng.standard_normal(n).astype(np.float32)
    g = rng.standard_normal(n).astype(np.float32)
    acc = rng.standard_normal(n).astype(np.float32)
    ws = torch.zeros(lib.acmi_opt_ws_floats(n), device=cuda)
    norm = torch.zeros(1, device=cuda)
    P, G, ACC = dev(p), dev(g), dev(acc)
    _lib.call('acmi_momentum_apply', _lib.ptr(P), _lib.ptr(ACC), _lib.ptr(G), n, 3e-4, 0.9, 0.5, _lib.ptr(ws),
              _lib.ptr(norm), _lib.stream_handle())
    rp, racc = oracle.momentum_apply(p.astype(np.float64), acc.astype(np.float64), g.astype(np.float64), 3e-4, 0.9,
                                     0.5)
    np.testing.assert_allclose(P.cpu().numpy(), rp, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(ACC.cpu().numpy(), racc, rtol=1e-5, atol=1e-7)
    assert norm.item() == pytest.approx(np.linalg.norm(g.astype(np.float64)), rel=1e-5)
    P, G = dev(p), dev(g)
    ms = torch.ones(n, device=cuda)
    mom = torch.zeros(n, device=cuda)
    _lib.call('acmi_rmsprop_apply', _lib.ptr(P), _lib.ptr(ms), _lib.ptr(mom), _lib.ptr(G), n, 7e-4, 0.9, 0.0, 1e-10,
              0.5, _lib.ptr(ws), _lib.ptr(norm), _lib.stream_handle())
    rp, rms, rmom = oracle.rmsprop_apply(p.astype(np.float64), np.ones(n), np.zeros(n), g.astype(np.float64), 7e-4,
                                         0.5)
    np.testing.assert_allclose(P.cpu().numpy(), rp, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(ms.cpu().numpy(), rms, rtol=1e-5)


def _build(N=3, T=4, A=4, C3=32, seed=5, games=None):
    from actorcritic import session as sess
    from actorcritic.agents import MultiEnvAgent
    from actorcritic.envs.atari.model import AtariModel
    from actorcritic.envs.atari.wrappers import SyntheticAtariEnvs
    from actorcritic.examples.atari.a2c_acktr import create_optimizer
    from actorcritic.multi_env import MultiEnv
    from actorcritic.nn import linear_decay
    from actorcritic.objectives import A2CObjective
    sess.reset_default_graph()
    kw = {} if games is None else dict(games=games)
    env = MultiEnv(SyntheticAtariEnvs(N, num_actions=A, seed=seed, **kw))
    params = oracle.init_params(A, C3, seed=1)
    model = AtariModel(env.observation_space, env.action_space, C3, params=params, random_seed=3)
    agent = MultiEnvAgent(env, model, T)
    obj = A2CObjective(model)
    gs = sess.get_or_create_global_step()
    opt = create_optimizer(C3 == 32, model, linear_decay(0.25, 0.025, gs, 1000) if C3 == 32 else 7e-4)
    op = obj.optimize_shared(opt, 0.5, global_step=gs)
    return env, model, agent, obj, gs, opt, op, params


def _feed(model, data):
    obs, act, rew, term, nxt, _ = data
    return {model.observations_placeholder: obs, model.bootstrap_observations_placeholder: nxt,
            model.actions_placeholder: act, model.rewards_placeholder: rew, model.terminals_placeholder: term}


def test_rollout_matches_oracle_env_and_tower(lib, cuda):
    from actorcritic import session as sess
    N, T, A = 3, 6, 4
    env, model, agent, obj, gs, opt, op, params = _build(N, T, A)
    with sess.Session() as s:
        data = agent.interact(s)
    obs, act, rew, term, nxt, infos = [x for x in data]
    o = obs.cpu().numpy()
    # the stepper: replay the sampled actions through the oracle envs
    envs = [oracle.SyntheticAtari(5, e) for e in range(N)]
    for e in range(N):
        np.testing.assert_array_equal(o[e, 0], envs[e].reset())
        for t in range(T):
            ob, r, d, ep = envs[e].step(int(act[e, t]))
            nxt_ref = ob
            if t + 1 < T:
                np.testing.assert_array_equal(o[e, t + 1], ob)
            assert float(rew[e, t]) == r and bool(term[e, t]) == d
        np.testing.assert_array_equal(nxt[e].cpu().numpy(), nxt_ref)
    # the tower activations cached by the rollout (row n*T + t)
    fwd = model.engine.lookup_rollout(obs)
    ref = oracle.forward(params, o.reshape(-1, 84, 84, 4), A, 32)
    for name, got in (('logits', fwd.flat_logits), ('value', fwd.flat_value), ('a4', fwd.acts.a4),
                      ('a1', fwd.acts.a1)):
        r = ref[name].reshape(got.shape)
        rel = np.abs(got.cpu().double().numpy() - r).max() / np.abs(r).max()
        assert rel < 1e-5, (name, rel)
    # at N = 3 the rollout's towers ran split (step 0: tower_split_kernel, steps 1..:
    # rollout_tail_split_kernel, each image over 7 workgroups; towersplit.hpp): bit
    # for bit the one-block tower's activations and ReLU' words on the same
    # observations inside a 72-image batch (B > kSplitMaxB)
    M = N * T
    rep = torch.from_numpy(np.concatenate([o.reshape(M, 84, 84, 4)] * 4)).to(cuda)
    one, _ = model.engine.forward_obs(rep, key='one-block')
    torch.cuda.synchronize()
    for k in ('a1', 'a2', 'a3', 'm1', 'm2', 'm3'):
        assert torch.equal(getattr(fwd.acts, k)[:M], getattr(one, k)[:M]), k
    # the actions are the oracle's inverse-CDF draws of the rollout's counters
    lg = fwd.flat_logits.cpu().numpy().reshape(N, T, A)
    for t in range(T):
        u = oracle.sample_uniforms(3, 0, t, N)
        np.testing.assert_array_equal(act[:, t].cpu().numpy(), oracle.sample_f32(lg[:, t], u))


_UPDATE_CASES = [
    # (N, T, A, games, forward)
    (3, 5, 4, None, 'f32'),
    (32, 20, 4, None, 'f32'),
    (32, 20, 18, 'atari57', 'f32'),
    (32, 20, 18, 'atari57', 'bf16'),
]


@pytest.fixture
def forward_mode(lib):
    """Sets acmi_set_forward_mode for one test and restores the previous mode."""
    prev = lib.acmi_get_forward_mode()
    yield lambda m: _lib.call('acmi_set_forward_mode', _lib.FWD_BF16 if m == 'bf16' else _lib.FWD_F32)
    _lib.call('acmi_set_forward_mode', prev)


def _blocks(A, C3):
    """[(name, lo, hi)] of the six K-FAC blocks ([W; b] contiguous) in the flat layout."""
    off, n = oracle.param_offsets(A, C3)
    names = ['conv1', 'conv2', 'conv3', 'fc4', 'fc_policy', 'fc_baseline']
    return [(names[l], off[2 * l], off[2 * l + 2] if l < 5 else n) for l in range(6)]


@pytest.mark.parametrize('N,T,A,games,fwd', _UPDATE_CASES,
                         ids=['toy', 'configs2-32x20', 'configs4-a18-atari57', 'configs4-a18-atari57-bf16fwd'])
def test_acktr_update_matches_oracle(lib, cuda, forward_mode, N, T, A, games, fwd):
    """One steady-state ACKTR update at gs=40 (covariance update + inverse + apply)
    against the float64 oracle on the same rollout -- at a toy size, at the
    reference's own ACKTR config, BASELINE configs[2] (32 envs x 20 steps, C3 = 32,
    a2c_acktr.py:306-310, :51-53), and at the configs[4] action space (A = 18, mixed
    Atari-57 games): A/G factors, the damped inverses, the preconditioned gradients
    (north_star rel-L2 1e-3) and the parameter step, all PER K-FAC BLOCK (the value
    head's 513 and the policy head's 19 x 18 entries are < 0.3 % of the vector; a
    global norm could hide them), and the trust-region coefficient.

    A = 18 runs the policy head's categorical G factor at 18 x 18
    (policies.py:146-158), the heads' weight gradient + A factor with 19 dY columns,
    and the K-FAC step's narrow first product for A % 4 != 0 (kfac.hip
    kfac_narrow_kernel).  The bf16 case runs the rollout tower on bf16 MFMAs
    (BASELINE configs[4] "bf16 forward / fp32 KFAC"); the update behind it is f32.

    The oracle's backward, factors and step are fed the GPU's own forward --
    activations, logits, values, targets (a2c_acktr.py:243-247) -- after that forward
    is checked against the float64 oracle forward (rel 1e-5, bf16: 1e-2): what is
    compared is the update's arithmetic on identical inputs.  (With the float64
    forward's own ReLU masks, a pre-activation within f32 rounding of zero takes the
    other branch; at 640 rows x 12800 conv1 outputs such flips move conv1's G factor
    by ~1e-4, more than the update's rounding.)"""
    from actorcritic import session as sess
    forward_mode(fwd)
    C3 = 32
    env, model, agent, obj, gs, opt, op, params = _build(N, T, A, C3, games=games)
    gs.assign(40)
    with sess.Session() as s:
        data = agent.interact(s)
        feed = _feed(model, data)
        fwd_out = model.engine.lookup_rollout(data[0])
        logits32 = fwd_out.flat_logits.cpu().numpy().copy()
        p_before = model.params.cpu().numpy().astype(np.float64)
        acts = fwd_out.acts
        M = N * T
        gpu = dict(a1=acts.a1[:M], a2=acts.a2[:M], a3=acts.a3[:M], a4=acts.a4[:M],
                   logits=fwd_out.flat_logits, value=fwd_out.flat_value)
        gpu = {k: v.cpu().double().numpy() for k, v in gpu.items()}
        tg_gpu = s.run(obj.target_values, feed_dict=feed)
        s.run(op, feed_dict=feed)
        torch.cuda.synchronize()
    obs, act, rew, term, nxt, _ = [x for x in data]
    M = N * T
    # the GPU forward and targets against float64 (f32: rel 1e-5; the bf16 tower
    # within 1e-2, test_bf16_forward_mode)
    ref_fwd = oracle.forward(p_before, obs.cpu().numpy().reshape(M, 84, 84, 4), A, C3)
    vb = oracle.forward(p_before, nxt.cpu().numpy(), A, C3)['value']
    tg_ref = oracle.targets_f64(rew.cpu().numpy(), term.cpu().numpy(), vb, 0.99).reshape(-1)
    ftol = 1e-2 if fwd == 'bf16' else 1e-5
    for k in ('a1', 'a2', 'a3', 'a4', 'logits', 'value'):
        r = ref_fwd[k].reshape(gpu[k].shape)
        rel = np.abs(gpu[k] - r).max() / np.abs(r).max()
        assert rel < ftol, ('forward', k, rel)
    tg = np.asarray(tg_gpu, np.float64).reshape(-1)
    assert np.abs(tg - tg_ref).max() <= (1e-2 if fwd == 'bf16' else 1e-5) * max(1.0, np.abs(tg_ref).max())
    # the update's inputs: the GPU's own forward
    full = dict(gpu, x=obs.cpu().numpy().reshape(M, 84, 84, 4).astype(np.float64) / 255.0)
    full['a3f'] = full['a3'].reshape(M, -1)
    lg = oracle.a2c_loss_and_head_grads(full['logits'], full['value'], act.cpu().numpy().reshape(-1), tg)
    grads, _, afac = oracle.backward(p_before, full, lg['dlogits'], lg['dvalue'], A, C3, with_a_factors=True)
    g_pi, g_v, y = oracle.sampled_head_grads(logits32, 0x4b464143, 0, 40)
    if games is not None:
        assert len(np.unique(y)) > 4  # the draws reach actions beyond Breakout's four
    gfac = oracle.g_factors(p_before, full, g_pi, g_v, A, C3)
    st = opt.state
    L = model.engine.layout
    fac = st['factors'].cpu().numpy().astype(np.float64)
    for f in range(5):
        d = L.din[f]
        got = fac[L.stat_off[f]:L.stat_off[f] + d * d].reshape(d, d)
        rel = np.abs(got - afac[f]).max() / np.abs(afac[f]).max()
        assert rel < 2e-5, ('A', f, rel)  # first EMA step with zero-debias == the batch statistics
    for l in range(6):
        d = L.dout[l]
        got = fac[L.stat_off[5 + l]:L.stat_off[5 + l] + d * d].reshape(d, d)
        rel = np.abs(got - gfac[l]).max() / np.abs(gfac[l]).max()
        assert rel < 5e-5, ('G', l, rel)
    assert L.dout[4] == A
    inv = oracle.damped_inverses(afac, gfac, 0.01)
    # the damped inverses, each against the float64 inverse of the oracle's factors
    # (their difference is the f32 factors' rounding seen through the damped
    # condition number: the relative error is bounded by cond * 2e-5)
    inv_got = st['inv']
    for l in range(6):
        for m, ref in ((2 * l, inv[l][0]), (2 * l + 1, inv[l][1])):
            got = L.inverse_block(inv_got, m).cpu().numpy().astype(np.float64)
            rel = np.abs(got - ref).max() / np.abs(ref).max()
            print('inverse', l, m % 2, 'rel %.2e' % rel)
            assert rel < 1e-3, ('inverse', l, m % 2, rel)
    new_p, vel, precon, coeff = oracle.kfac_step(p_before, np.zeros_like(p_before), grads, inv,
                                                 oracle.linear_decay(0.25, 0.025, 40, 1000), 0.9, 1e-4, A, C3)
    got_pre = st['precon'].cpu().numpy().astype(np.float64)
    got_p = model.params.cpu().numpy().astype(np.float64)
    rel_l2 = np.linalg.norm(got_pre - precon) / np.linalg.norm(precon)
    assert rel_l2 < 1e-3, rel_l2  # north_star: preconditioned gradients within 1e-3 rel-L2
    # ... and per K-FAC block, so a wrong head block cannot hide in the global norm
    for name, lo, hi in _blocks(A, C3):
        e_pre = np.linalg.norm(got_pre[lo:hi] - precon[lo:hi]) / np.linalg.norm(precon[lo:hi])
        e_step = np.linalg.norm(got_p[lo:hi] - new_p[lo:hi]) / np.linalg.norm(new_p[lo:hi] - p_before[lo:hi])
        print('block %-11s precon rel-L2 %.2e  step rel-L2 %.2e' % (name, e_pre, e_step))
        assert e_pre < 1e-3, (name, 'precon', e_pre)
        assert e_step < 1e-3, (name, 'step', e_step)
    assert float(st['coeff'][0]) == pytest.approx(coeff, rel=1e-3)
    assert np.linalg.norm(got_p - new_p) / np.linalg.norm(new_p - p_before) < 1e-3
    assert gs.value == 41


@pytest.mark.parametrize('fwd', ['f32', 'bf16'])
def test_acktr_update_end_to_end_vs_float64_forward(lib, cuda, forward_mode, fwd):
    """End to end at BASELINE configs[2] (32 envs x 20 steps, A = 4): the float64
    oracle runs its OWN forward on the rollout's observations (oracle.forward) and
    everything after it -- targets, losses, backward, A / G factors, damped
    inverses, the K-FAC step -- so the forward's error is carried into the update
    (test_acktr_update_matches_oracle feeds the oracle the GPU's forward instead
    and checks the update's arithmetic alone).  The sampled-loss draws are the
    GPU's (a draw at a CDF boundary may flip between f32 and float64 logits); their
    probabilities are the oracle's.

    f32: preconditioned gradient and step within 1e-3 rel-L2 per K-FAC block
    (north_star).  bf16 forward (configs[4]'s "bf16 forward / fp32 K-FAC"): the
    tower rounds conv2 / conv3 inputs to 16 bits (range-relative error ~1e-3,
    test_bf16_forward_mode), which reaches the update -- the per-block errors are
    printed as the tracked end-to-end number (round 5: 2.8e-2 .. 5.1e-2 per block) and
    bounded at 1e-1."""
    from actorcritic import session as sess
    forward_mode(fwd)
    N, T, A, C3 = 32, 20, 4, 32
    env, model, agent, obj, gs, opt, op, params = _build(N, T, A, C3)
    gs.assign(40)
    with sess.Session() as s:
        data = agent.interact(s)
        feed = _feed(model, data)
        logits32 = model.engine.lookup_rollout(data[0]).flat_logits.cpu().numpy().copy()
        p_before = model.params.cpu().numpy().astype(np.float64)
        s.run(op, feed_dict=feed)
        torch.cuda.synchronize()
    obs, act, rew, term, nxt, _ = data
    M = N * T
    full = oracle.forward(p_before, obs.cpu().numpy().reshape(M, 84, 84, 4), A, C3)
    vb = oracle.forward(p_before, nxt.cpu().numpy(), A, C3)['value']
    tg = oracle.targets_f64(rew.cpu().numpy(), term.cpu().numpy(), vb, 0.99).reshape(-1)
    lg = oracle.a2c_loss_and_head_grads(full['logits'], full['value'], act.cpu().numpy().reshape(-1), tg)
    grads, _, afac = oracle.backward(p_before, full, lg['dlogits'], lg['dvalue'], A, C3, with_a_factors=True)
    _, g_v, y = oracle.sampled_head_grads(logits32, 0x4b464143, 0, 40)
    g_pi = np.exp(oracle.log_softmax(full['logits'])) - np.eye(A)[y]
    gfac = oracle.g_factors(p_before, full, g_pi, g_v, A, C3)
    inv = oracle.damped_inverses(afac, gfac, 0.01)
    new_p, _, precon, coeff = oracle.kfac_step(p_before, np.zeros_like(p_before), grads, inv,
                                               oracle.linear_decay(0.25, 0.025, 40, 1000), 0.9, 1e-4, A, C3)
    got_pre = opt.state['precon'].cpu().numpy().astype(np.float64)
    got_p = model.params.cpu().numpy().astype(np.float64)
    tol = 1e-3 if fwd == 'f32' else 1e-1
    for name, lo, hi in _blocks(A, C3):
        e_pre = np.linalg.norm(got_pre[lo:hi] - precon[lo:hi]) / np.linalg.norm(precon[lo:hi])
        e_step = np.linalg.norm(got_p[lo:hi] - new_p[lo:hi]) / np.linalg.norm(new_p[lo:hi] - p_before[lo:hi])
        print('%s forward, end to end: block %-11s precon rel-L2 %.2e  step rel-L2 %.2e' % (fwd, name, e_pre, e_step))
        assert e_pre < tol, (name, 'precon', e_pre)
        assert e_step < tol, (name, 'step', e_step)
    assert float(opt.state['coeff'][0]) == pytest.approx(coeff, rel=tol)


def test_cold_start_schedule(lib, cuda):
    from actorcritic import session as sess
    env, model, agent, obj, gs, opt, op, params = _build(2, 3)
    flags = []
    with sess.Session() as s:
        for _ in range(3):
            data = agent.interact(s)
            s.run(op, feed_dict=_feed(model, data))
            flags.append(opt.last_flags)
    assert flags == [(True, False, False)] * 3 and gs.value == 6
    assert torch.isfinite(model.params).all()


@pytest.mark.parametrize('N', [2, 32], ids=['toy', 'configs1-32x5'])
def test_a2c_update_matches_oracle(lib, cuda, N):
    """A2C: RMSProp + clip 0.5, one update vs the float64 oracle -- at a toy size and
    at BASELINE configs[1] (32 envs x 5 steps, C3 = 64, a2c_acktr.py:249-251)."""
    from actorcritic import session as sess
    env, model, agent, obj, gs, opt, op, params = _build(N, 5, C3=64)
    with sess.Session() as s:
        data = agent.interact(s)
        p0 = model.params.cpu().numpy().astype(np.float64)
        s.run(op, feed_dict=_feed(model, data))
    obs, act, rew, term, nxt, _ = data
    full = oracle.forward(p0, obs.cpu().numpy().reshape(-1, 84, 84, 4), 4, 64)
    vb = oracle.forward(p0, nxt.cpu().numpy(), 4, 64)['value']
    tg = oracle.targets_f64(rew.cpu().numpy(), term.cpu().numpy(), vb, 0.99).reshape(-1)
    lg = oracle.a2c_loss_and_head_grads(full['logits'], full['value'], act.cpu().numpy().reshape(-1), tg)
    grads, _ = oracle.backward(p0, full, lg['dlogits'], lg['dvalue'], 4, 64)
    rp, _, _ = oracle.rmsprop_apply(p0, np.ones_like(p0), np.zeros_like(p0), grads, 7e-4, 0.5)
    got = model.params.cpu().numpy().astype(np.float64)
    # per element: 1e-3 of the update plus the f32 rounding of the stored parameter
    bound = 1e-3 * np.abs(rp - p0) + 2 * np.finfo(np.float32).eps * np.abs(p0) + 1e-12
    assert np.all(np.abs(got - rp) <= bound)


def test_losses_and_fetches_through_session(lib, cuda):
    from actorcritic import session as sess
    N, T = 3, 4
    env, model, agent, obj, gs, opt, op, params = _build(N, T)
    with sess.Session() as s:
        data = agent.interact(s)
        feed = _feed(model, data)
        pl, bl, me, ent, lp = s.run([obj.policy_loss, obj.baseline_loss, obj.mean_entropy, model.policy.entropy,
                                     model.policy.log_prob], feed_dict=feed)
    obs, act, rew, term, nxt, _ = data
    full = oracle.forward(params, obs.cpu().numpy().reshape(-1, 84, 84, 4), 4, 32)
    vb = oracle.forward(params, nxt.cpu().numpy(), 4, 32)['value']
    tg = oracle.targets_f64(rew.cpu().numpy(), term.cpu().numpy(), vb, 0.99).reshape(-1)
    ref = oracle.a2c_loss_and_head_grads(full['logits'], full['value'], act.cpu().numpy().reshape(-1), tg)
    assert pl == pytest.approx(ref['policy_loss'], rel=1e-4, abs=1e-6)
    assert bl == pytest.approx(ref['baseline_loss'], rel=1e-4)
    assert me == pytest.approx(ref['mean_entropy'], rel=1e-5)
    assert ent.shape == (N, T) and lp.shape == (N, T)
    np.testing.assert_allclose(ent.reshape(-1), oracle.entropy(full['logits']), rtol=1e-5)


@pytest.mark.parametrize('acktr', [False, True])
def test_resumed_update_is_bit_identical(lib, cuda, tmp_path, acktr):
    """A checkpoint written between two updates and restored into a fresh graph gives
    the uninterrupted run's second update bit for bit: the RMSProp ms/mom slots (A2C)
    and the cold-start Momentum accumulator + K-FAC velocity (ACKTR, gs < 30) come
    back with the parameters and the global step (a2c_acktr.py:101-102)."""
    from actorcritic import checkpoint
    from actorcritic import session as sess
    C3 = 32 if acktr else 64
    env, model, agent, obj, gs, opt, op, params = _build(3, 4, C3=C3)
    with sess.Session() as s:
        s.run(op, feed_dict=_feed(model, agent.interact(s)))
        # a fresh copy of the second batch: both runs below take the same inputs
        # (and the same batched forward -- no rollout-cache hit on a copy)
        data = tuple(x.clone() if isinstance(x, torch.Tensor) else x for x in agent.interact(s))
        path = checkpoint.save(str(tmp_path / 'Atari'), gs.value, model, opt)
        s.run(op, feed_dict=_feed(model, data))
    torch.cuda.synchronize()
    uninterrupted, gs_after = model.params.clone(), gs.value

    env, model2, agent2, obj2, gs2, opt2, op2, _ = _build(3, 4, C3=C3)
    checkpoint.load(path, model2, opt2, gs2)
    with sess.Session() as s:
        s.run(op2, feed_dict=_feed(model2, data))
    torch.cuda.synchronize()
    assert gs2.value == gs_after
    assert not torch.equal(model2.params, torch.from_numpy(params).cuda())
    assert torch.equal(model2.params, uninterrupted)


def test_copy_batches_returns_fresh_tensors(lib, cuda):
    """copy_batches=True: a kept batch survives the next interact(); its update still
    re-uses the rollout activations (same result as the aliased buffers)."""
    from actorcritic import session as sess
    from actorcritic.agents import MultiEnvAgent
    env, model, agent, obj, gs, opt, op, params = _build(3, 4)
    agent = MultiEnvAgent(env, model, 4, copy_batches=True)
    with sess.Session() as s:
        first = agent.interact(s)
        assert model.engine.lookup_rollout(first[0]) is not None
        kept = [x.clone() for x in first[:5]]
        second = agent.interact(s)
        for a, b in zip(first[:5], kept):
            assert torch.equal(a, b)
        assert first[0].data_ptr() != second[0].data_ptr()
        assert model.engine.lookup_rollout(first[0]) is None  # superseded: recomputed if fed


def test_select_max_actions_and_single_env_agent(lib, cuda):
    """model.select_max_actions (model.py:153-169: session.run(policy.mode) on a
    [batch, 1] feed) is the argmax of the float64 oracle's logits, and
    SingleEnvAgent.interact (agents.py:50-131) steps one host env with
    sample_actions([[obs]]): [1, steps] outputs whose observations, rewards and
    terminals replay exactly through a second oracle env, and whose actions are the
    oracle's inverse-CDF draws from the counter RNG of each step."""
    from actorcritic import session as sess
    from actorcritic.agents import SingleEnvAgent
    env, model, agent, obj, gs, opt, op, params = _build(3, 4)
    rng = np.random.default_rng(17)
    B = 9
    obs = rng.integers(0, 256, size=(B, 1, 84, 84, 4), dtype=np.uint8)
    ref = oracle.forward(params, obs.reshape(B, 84, 84, 4), 4, 32)['logits']
    with sess.Session() as s:
        got = model.select_max_actions([list(o) for o in obs], s)
    assert isinstance(got, list) and len(got) == B
    top2 = np.sort(ref, axis=1)[:, -2:]
    clear = (top2[:, 1] - top2[:, 0]) > 1e-4 * np.abs(ref).max()
    assert clear.sum() >= B - 1
    np.testing.assert_array_equal(np.asarray(got)[clear], ref.argmax(1)[clear])

    T = 7
    host_env = oracle.SyntheticAtari(5, 0)
    single = SingleEnvAgent(host_env, model, T)
    eng = model.engine
    with sess.Session() as s:
        c0 = eng.sample_counter
        o, a, r, d, nxt, infos = single.interact(s)
        c1 = eng.sample_counter
        o2, a2, _, _, nxt2, _ = single.interact(s)
    assert [len(x) for x in (o, a, r, d, infos)] == [1] * 5 and len(o[0]) == T and len(nxt) == 1
    assert c1 - c0 == T
    np.testing.assert_array_equal(o2[0][0], nxt[0])  # carried into the next call
    replay = oracle.SyntheticAtari(5, 0)
    np.testing.assert_array_equal(o[0][0], replay.reset())
    logits = oracle.forward(params, np.stack(o[0]), 4, 32)['logits'].astype(np.float32)
    for t in range(T):
        u = oracle.sample_uniforms(3, 0, c0 + t, 1)
        draw = int(oracle.sample_f32(logits[t:t + 1], u)[0])
        # the GPU logits are f32 (1e-5 of the oracle's): a draw may differ only where
        # the uniform sits on a CDF boundary
        assert a[0][t] == draw, (t, a[0][t], draw)
        ob, rr, dd, _ = replay.step(a[0][t])
        assert rr == r[0][t] and dd == d[0][t]
        if t + 1 < T:
            np.testing.assert_array_equal(o[0][t + 1], ob)
    np.testing.assert_array_equal(nxt[0], ob)
