"""Generates tests/golden/* from the reference's own code (run in the build container,
where /root/reference exists; the GPU box only sees the committed fixtures).

What runs from /root/reference (read as text, executed without TensorFlow/gym):
  * objectives.py:180-196 `_discount.fn` and :209-211 `_discount_bootstrap.fn`
    (extracted with `ast`, executed with numpy exactly as tf.py_func would call them:
    terminals as a bool ndarray, discount_factor as a 0-d float32 ndarray);
  * agents.py (stdlib-only module: imported directly) — MultiEnvAgent.interact and
    transpose_list on a fake multi-env / fake model;
  * wrappers.py:224-235 FrameStackWrapper.step/reset, :282-323 EpisodeInfoWrapper and
    multi_env.py:127-137 _AutoResetWrapper.step/reset (the method bodies extracted with
    `ast` and bound to plain objects; no gym stand-in module is created) wrapped around
    the synthetic raw frame source of oracle.py.

tf.matmul (objectives.py:201) is not available: the fixture uses np.matmul in float32
as its stand-in and records the float64 product beside it.

Run:  PYTHONDONTWRITEBYTECODE=1 python -B oracle/make_golden.py
"""

import ast
import importlib.util
import json
import os
import sys
import textwrap
import types
import zlib

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = '/root/reference/actorcritic'
OUT = os.path.join(ROOT, 'tests', 'golden')
sys.path.insert(0, HERE)
import oracle  # noqa: E402


def _source(rel):
    with open(os.path.join(REF, rel)) as f:
        return f.read()


def _find(tree, name, cls=None):
    for node in ast.walk(tree):
        if cls is not None and isinstance(node, ast.ClassDef) and node.name == cls:
            for sub in node.body:
                if isinstance(sub, ast.FunctionDef) and sub.name == name:
                    return sub
        if cls is None and isinstance(node, ast.FunctionDef) and node.name == name:
            return node
    raise KeyError((cls, name))


def _compile(fn_node, src, env):
    code = textwrap.dedent(ast.get_source_segment(src, fn_node))
    # drop decorators (e.g. @staticmethod) from the extracted text
    lines = [ln for ln in code.splitlines() if not ln.lstrip().startswith('@')]
    ns = dict(env)
    exec(compile('\n'.join(lines), '<reference:{}>'.format(fn_node.name), 'exec'), ns)
    return ns[fn_node.name]


def reference_discount_closures():
    src = _source('objectives.py')
    tree = ast.parse(src)
    outer_d = _find(tree, '_discount')
    outer_b = _find(tree, '_discount_bootstrap')
    inner_d = [n for n in outer_d.body if isinstance(n, ast.FunctionDef) and n.name == 'fn'][0]
    inner_b = [n for n in outer_b.body if isinstance(n, ast.FunctionDef) and n.name == 'fn'][0]
    fn_d = _compile(inner_d, src, {'np': np})
    # the bootstrap closure reads `discount_factor` from the enclosing scope
    return fn_d, lambda disc: _compile(inner_b, src, {'np': np, 'discount_factor': disc})


def golden_returns():
    fn_d, make_b = reference_discount_closures()
    gamma = 0.99
    disc_t = np.array(gamma, dtype=np.float32)  # what tf.py_func passes for the float constant
    fn_b = make_b(gamma)  # Python float captured by the closure (objectives.py:205-211)
    rng = np.random.default_rng(123)
    cases = []
    shapes = [(1, 1), (1, 5), (3, 5), (3, 20), (32, 20), (32, 5), (4, 7)]
    patterns = ['none', 'first', 'last', 'multi', 'random', 'all']
    for N, T in shapes:
        for pat in patterns:
            term = np.zeros((N, T), bool)
            if pat == 'first':
                term[:, 0] = True
            elif pat == 'last':
                term[:, T - 1] = True
            elif pat == 'multi':
                term[:, ::3] = True
            elif pat == 'random':
                term = rng.random((N, T)) < 0.2
            elif pat == 'all':
                term[:] = True
            rewards = rng.choice(np.array([-1.0, 0.0, 1.0], np.float32), size=(N, T), p=[.2, .5, .3])
            rewards = (rewards + rng.standard_normal((N, T)).astype(np.float32) * 0.25).astype(np.float32)
            values = rng.standard_normal((N, T)).astype(np.float32)
            v_boot = rng.standard_normal(N).astype(np.float32)
            D = fn_d(term, disc_t)                       # [N, T, T] float32
            bf = fn_b(term)                              # [N, T] float32
            disc32 = np.matmul(rewards[:, None, :], D)[:, 0, :].astype(np.float32)
            disc64 = np.matmul(rewards[:, None, :].astype(np.float64), D.astype(np.float64))[:, 0, :]
            boot32 = (bf * v_boot[:, None]).astype(np.float32)
            tgt32 = (disc32 + boot32).astype(np.float32)
            tgt64 = disc64 + bf.astype(np.float64) * v_boot[:, None].astype(np.float64)
            cases.append(dict(N=N, T=T, pattern=pat, rewards=rewards, terminals=term, values=values,
                              v_boot=v_boot, D=D, boot_factors=bf, targets_f32=tgt32, targets_f64=tgt64,
                              adv_f32=(tgt32 - values).astype(np.float32)))
    arrays = {}
    for i, c in enumerate(cases):
        for k, v in c.items():
            if isinstance(v, np.ndarray):
                arrays['c{}_{}'.format(i, k)] = v
    meta = [dict(N=c['N'], T=c['T'], pattern=c['pattern']) for c in cases]
    np.savez_compressed(os.path.join(OUT, 'returns.npz'), meta=json.dumps(meta), gamma=np.float32(gamma),
                        **arrays)
    return len(cases)


def golden_agent_layout():
    spec = importlib.util.spec_from_file_location('ref_agents', os.path.join(REF, 'agents.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)

    class FakeMultiEnv:
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

    env, model = FakeMultiEnv(3), FakeModel()
    agent = mod.MultiEnvAgent(env, model, 4)
    first = agent.interact(None)
    second = agent.interact(None)

    # SingleEnvAgent (agents.py:50-131): one env, [[obs]]-shaped sample batches,
    # [1, steps] outputs, next observation kept between calls (no auto-reset)
    class FakeEnv:
        def __init__(self):
            self.t, self.resets = 0, 0

        def reset(self):
            self.resets += 1
            return 'obs(r{},t{})'.format(self.resets, self.t)

        def step(self, action):
            self.t += 1
            return 'obs(r{},t{})'.format(self.resets, self.t), 0.5 * action, action % 2 == 1, {'t': self.t}

    single_model = FakeModel()
    single = mod.SingleEnvAgent(FakeEnv(), single_model, 3)
    s_first = single.interact(None)
    s_second = single.interact(None)
    out = dict(
        transpose_list=mod.transpose_list([[1, 2, 3, 4], [5, 6, 7, 8], [9, 10, 11, 12]]),
        sample_batches=model.batches,
        first=[list(x) for x in first],
        second=[list(x) for x in second],
        single_sample_batches=single_model.batches,
        single_first=[list(x) for x in s_first],
        single_second=[list(x) for x in s_second],
    )
    with open(os.path.join(OUT, 'agent_layout.json'), 'w') as f:
        json.dump(out, f, indent=1)


class _Obj:
    pass


def _bind(obj, fns):
    for name, fn in fns.items():
        setattr(obj, name, types.MethodType(fn, obj))
    return obj


def golden_framestack(seed=7, envs=(0, 5), steps=700):
    """Reference wrappers around the synthetic raw frame source."""
    wsrc = _source('envs/atari/wrappers.py')
    wtree = ast.parse(wsrc)
    msrc = _source('multi_env.py')
    mtree = ast.parse(msrc)
    fs_step = _compile(_find(wtree, 'step', 'FrameStackWrapper'), wsrc, {'np': np})
    fs_reset = _compile(_find(wtree, 'reset', 'FrameStackWrapper'), wsrc, {'np': np})
    ei_step = _compile(_find(wtree, 'step', 'EpisodeInfoWrapper'), wsrc, {'np': np})
    ei_reset = _compile(_find(wtree, 'reset', 'EpisodeInfoWrapper'), wsrc, {'np': np})
    ei_batch = _compile(_find(wtree, 'get_episode_rewards_from_info_batch', 'EpisodeInfoWrapper'), wsrc,
                        {'np': np})
    ar_step = _compile(_find(mtree, 'step', '_AutoResetWrapper'), msrc, {})
    ar_reset = _compile(_find(mtree, 'reset', '_AutoResetWrapper'), msrc, {})

    class RawSynthetic:
        """The raw (unstacked) synthetic game: one [84,84,1] frame per step."""

        def __init__(self, seed, e):
            self.seed, self.e, self.k, self.t, self.started = seed, e, -1, 0, False

        def reset(self):
            self.k += 1
            self.t = 0
            self.L = oracle.episode_length(self.seed, self.e, self.k)
            return oracle.reset_frame(self.seed, self.e, self.k)[..., None]

        def step(self, a):
            self.t += 1
            base = int(oracle.key4(self.seed, self.e, self.k, self.t * 256 + (int(a) & 255)))
            rh = int(oracle.mix32(np.uint32(base) ^ oracle.REW_SALT)) >> 8
            r = -1.0 if rh < oracle.REW_LO else (1.0 if rh >= oracle.REW_HI else 0.0)
            return oracle._frame(base)[..., None], r, self.t >= self.L, {}

    rng = np.random.default_rng(99)
    record = {}
    infos_all = []
    for e in envs:
        raw = RawSynthetic(seed, e)
        ei = _bind(_Obj(), {'step': ei_step, 'reset': ei_reset})
        ei.env, ei.total_reward = raw, 0.0
        fs = _bind(_Obj(), {'step': fs_step, 'reset': fs_reset})
        fs.env, fs._num_stacked_frames = ei, 4
        fs._stacked_frames = np.zeros((84, 84, 4), np.uint8)
        ar = _bind(_Obj(), {'step': ar_step, 'reset': ar_reset})
        ar.env, ar._terminated = fs, False
        obs = ar.reset()
        crcs, rews, terms, acts, infos = [zlib.crc32(np.ascontiguousarray(obs).tobytes())], [], [], [], []
        keep = {}
        for t in range(steps):
            a = int(rng.integers(0, 4))
            obs, r, d, info = ar.step(a)
            crcs.append(zlib.crc32(np.ascontiguousarray(obs).tobytes()))
            rews.append(r)
            terms.append(bool(d))
            acts.append(a)
            infos.append(dict(info))
            if d or (t > 0 and terms[t - 1]):
                keep['obs_t{}'.format(t + 1)] = np.array(obs, np.uint8)
        infos_all.append(infos)
        record['env{}'.format(e)] = dict(crc=crcs, rewards=rews, terminals=terms, actions=acts)
        np.savez_compressed(os.path.join(OUT, 'framestack_env{}.npz'.format(e)), **keep)
    ep = ei_batch([inf[:steps] for inf in infos_all])
    record['episode_rewards'] = [[None if np.isnan(v) else float(v) for v in row] for row in ep]
    record['seed'] = seed
    record['envs'] = list(envs)
    with open(os.path.join(OUT, 'framestack_autoreset.json'), 'w') as f:
        json.dump(record, f)


def _atari_chain_reference(env, wsrc, wtree):
    """The make_atari_env chain (a2c_acktr.py:190-213) from the reference's method
    bodies, minus AtariPreprocessFrameWrapper (cv2 is absent: the frames stay raw RGB)
    and RenderWrapper.  gym.RewardWrapper.step (apply `reward` to the inner step's
    reward) is the one piece of glue written here."""
    def m(cls, name):
        return _compile(_find(wtree, name, cls), wsrc, {'np': np})

    noop = _bind(_Obj(), {'reset': m('AtariNoopResetWrapper', 'reset'), 'step': m('AtariNoopResetWrapper', 'step')})
    noop.env, noop.unwrapped, noop.noop_max = env, env, 30
    skip = _bind(_Obj(), {'step': m('AtariFrameskipWrapper', 'step'), 'reset': m('AtariFrameskipWrapper', 'reset')})
    skip.env, skip._frameskip = noop, 4
    info = _bind(_Obj(), {'step': m('EpisodeInfoWrapper', 'step'), 'reset': m('EpisodeInfoWrapper', 'reset')})
    info.env, info.total_reward = skip, 0.0
    life = _bind(_Obj(), {'step': m('AtariEpisodicLifeWrapper', 'step'),
                          'reset': m('AtariEpisodicLifeWrapper', 'reset')})
    life.env, life.lives, life.episode_terminal = info, 0, True
    fire = _bind(_Obj(), {'step': m('AtariFireResetWrapper', 'step'), 'reset': m('AtariFireResetWrapper', 'reset')})
    fire.env = life
    clip = _bind(_Obj(), {'reward': m('AtariClipRewardWrapper', 'reward')})

    def clip_step(self, action):
        o, r, d, i = self.env.step(action)
        return o, self.reward(r), d, i

    _bind(clip, {'step': clip_step, 'reset': lambda self, **kw: self.env.reset(**kw)})
    clip.env = fire
    clear = _bind(_Obj(), {'step': m('AtariInfoClearWrapper', 'step'), 'reset': m('AtariInfoClearWrapper', 'reset')})
    clear.env = clip
    return clear


def golden_atari_wrappers(seeds=(3, 11), steps=400):
    """Trace of the reference's Atari wrapper chain over oracle.FakeALE: per step the
    CRC32 of the (max-pooled raw) observation, clipped reward, terminal, episode
    total from info; plus every action the game itself received (noop/fire resets)."""
    wsrc = _source('envs/atari/wrappers.py')
    wtree = ast.parse(wsrc)
    rng = np.random.default_rng(5)
    record = {}
    for seed in seeds:
        game = oracle.FakeALE(seed)
        env = _atari_chain_reference(game, wsrc, wtree)
        obs = env.reset()
        crcs, rews, terms, eps, acts = [zlib.crc32(np.ascontiguousarray(obs).tobytes())], [], [], [], []
        for t in range(steps):
            a = int(rng.integers(0, 4))
            obs, r, d, info = env.step(a)
            crcs.append(zlib.crc32(np.ascontiguousarray(obs).tobytes()))
            rews.append(float(r))
            terms.append(bool(d))
            eps.append(info['episode']['total_reward'] if 'episode' in info else None)
            acts.append(a)
            if d:  # the training loop's auto-reset (multi_env.py:127-132)
                crcs.append(zlib.crc32(np.ascontiguousarray(env.reset()).tobytes()))
        record['seed{}'.format(seed)] = dict(crc=crcs, rewards=rews, terminals=terms, episode=eps, actions=acts,
                                            game_actions=game.actions)
    with open(os.path.join(OUT, 'atari_wrappers.json'), 'w') as f:
        json.dump(record, f)


def main():
    os.makedirs(OUT, exist_ok=True)
    n = golden_returns()
    golden_agent_layout()
    golden_framestack()
    golden_atari_wrappers()
    print('wrote {} returns cases, agent layout, frame-stack/auto-reset trace to {}'.format(n, OUT))


if __name__ == '__main__':
    main()
