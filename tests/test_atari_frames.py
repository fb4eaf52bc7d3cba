"""Real-frame Atari row: the reference's wrapper chain
(envs/atari/wrappers.py:16-260, make_atari_env a2c_acktr.py:175-213) and the device
frame preprocessing (acmi_atari_preprocess / acmi_atari_stack).

  * CPU: this engine's host wrapper chain replays tests/golden/atari_wrappers.json
    exactly (the reference's own method bodies run over oracle.FakeALE, made by
    oracle/make_golden.py); the oracle's cv2 restatement against cv2's published gray
    values and the float64 area integral.  cv2 itself is absent: the INTER_AREA
    restatement is "parity unpinned" against it.
  * GPU: the kernels are bit-exact with the oracle (byte work) on 210x160 and other
    shapes, single/paired frames, terminals, resets, in-place stacks.
"""
import json
import os
import sys
import zlib

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'oracle'))
import oracle  # noqa: E402


def _trace(env, steps, rng):
    obs = env.reset()
    crcs, rews, terms, eps, acts = [zlib.crc32(np.ascontiguousarray(obs).tobytes())], [], [], [], []
    for _ in range(steps):
        a = int(rng.integers(0, 4))
        obs, r, d, info = env.step(a)
        crcs.append(zlib.crc32(np.ascontiguousarray(obs).tobytes()))
        rews.append(float(r))
        terms.append(bool(d))
        eps.append(info['episode']['total_reward'] if 'episode' in info else None)
        acts.append(a)
        assert 'ale.lives' not in info  # AtariInfoClearWrapper
        if d:
            crcs.append(zlib.crc32(np.ascontiguousarray(env.reset()).tobytes()))
    return dict(crc=crcs, rewards=rews, terminals=terms, episode=eps, actions=acts)


def test_wrapper_chain_replays_reference_trace():
    from actorcritic.envs.atari import wrappers
    gold = json.load(open(os.path.join(HERE, 'golden', 'atari_wrappers.json')))
    rng = np.random.default_rng(5)  # the generator's action stream (make_golden.py)
    for key in sorted(gold, key=lambda k: int(k[4:])):
        g = gold[key]
        game = oracle.FakeALE(int(key[4:]))
        env = wrappers.wrap_atari_env(game, preprocess=False)
        got = _trace(env, len(g['actions']), rng)
        for field in ('actions', 'terminals', 'rewards', 'episode', 'crc'):
            assert got[field] == g[field], (key, field)
        assert game.actions == g['game_actions'], key


def test_frame_stack_wrapper_host_semantics():
    from actorcritic.envs.atari import wrappers
    from actorcritic import spaces

    class Gray:
        observation_space = spaces.Box(low=0, high=255, shape=(84, 84, 1), dtype=np.uint8)

        def __init__(self):
            self.t = 0

        def reset(self):
            self.t = 0
            return np.full((84, 84, 1), 9, np.uint8)

        def step(self, a):
            self.t += 1
            return np.full((84, 84, 1), self.t, np.uint8), 0.0, self.t == 3, {}

    env = wrappers.FrameStackWrapper(Gray(), 4)
    assert env.observation_space.shape == (84, 84, 4)
    s = env.reset()
    assert (s[0, 0] == [9, 9, 9, 9]).all()
    assert (env.step(0)[0][0, 0] == [9, 9, 9, 1]).all()
    assert (env.step(0)[0][0, 0] == [9, 9, 1, 2]).all()
    assert (env.step(0)[0][0, 0] == [0, 0, 0, 3]).all()  # terminal: zero-fill, then insert


def test_gray_restatement_matches_cv2_published_values():
    # cv2.cvtColor(COLOR_RGB2GRAY) of pure red / green / blue / white / black
    px = np.array([[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [0, 0, 0]], np.uint8)
    assert list(oracle.atari_gray(px)) == [76, 150, 29, 255, 0]


def test_area_tables_and_resize_restatement():
    for ssize in (210, 160, 250, 100):
        runs = oracle.area_tables(ssize)
        assert len(runs) == 84
        for first, alphas in runs:
            assert abs(sum(float(a) for a in alphas) - 1.0) < 1e-6
            assert 0 <= first and first + len(alphas) <= ssize
    # 210 -> 84 is a ratio of 2.5: weights .4 .4 .2 / .2 .4 .4
    r = oracle.area_tables(210)
    assert r[0][0] == 0 and np.allclose(r[0][1], [0.4, 0.4, 0.2])
    assert r[1][0] == 2 and np.allclose(r[1][1], [0.2, 0.4, 0.4])
    # constant images stay constant; random images agree with the float64 area integral
    # to within the float32 rounding of a half
    assert (oracle.area_resize(np.full((210, 160), 201, np.uint8)) == 201).all()
    rng = np.random.default_rng(0)
    g = rng.integers(0, 256, (210, 160), dtype=np.uint8)
    got = oracle.area_resize(g).astype(np.float64)
    ry, rx = oracle.area_tables(210), oracle.area_tables(160)
    ref = np.zeros((84, 84))
    for dy, (fy, by) in enumerate(ry):
        wy = np.zeros(210)
        wy[fy:fy + len(by)] = by
        for dx, (fx, ax) in enumerate(rx):
            wx = np.zeros(160)
            wx[fx:fx + len(ax)] = ax
            ref[dy, dx] = wy @ g.astype(np.float64) @ wx
    assert np.abs(got - ref).max() <= 0.5 + 1e-3


def test_frame_entry_points_reject_bad_shapes(lib):
    import ctypes
    buf = ctypes.create_string_buffer(168 * 168 * 3 + 16)
    out = ctypes.create_string_buffer(84 * 84)
    # integer ratios (cv2's fast path) and sizes below 84 are refused before any launch
    assert lib.acmi_atari_preprocess(buf, 168 * 168 * 3, 0, None, 1, 168, 168, out, 84 * 84, None) == -1
    assert lib.acmi_atari_preprocess(buf, 80 * 160 * 3, 0, None, 1, 80, 160, out, 84 * 84, None) == -1
    assert lib.acmi_atari_stack(buf, 210 * 160 * 3, 0, None, 1, 210, 160, None, 0, None, out, 4 * 84 * 84,
                                None) == -1  # step without a stack_in


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------
def _frames(rng, n, h=210, w=160):
    return rng.integers(0, 256, (n, h, w, 3), dtype=np.uint8)


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [(210, 160), (250, 160), (100, 92)])
def test_preprocess_kernel_bit_exact(shape, cuda):
    import torch
    from actorcritic.envs.atari import wrappers
    rng = np.random.default_rng(shape[0])
    n = 13
    last, prev = _frames(rng, n, *shape), _frames(rng, n, *shape)
    last[0] = 255  # saturated
    last[1] = 0
    got1 = wrappers.preprocess_frames(torch.from_numpy(last).cuda()).cpu().numpy()
    got2 = wrappers.preprocess_frames(torch.from_numpy(last).cuda(), torch.from_numpy(prev).cuda()).cpu().numpy()
    for i in range(n):
        assert np.array_equal(got1[i], oracle.atari_preprocess(last[i])), i
        assert np.array_equal(got2[i], oracle.atari_preprocess(last[i], prev[i])), i


@pytest.mark.gpu
def test_frame_pipeline_matches_wrapper_semantics(cuda):
    from actorcritic.envs.atari import wrappers
    rng = np.random.default_rng(1)
    n = 9
    pipe = wrappers.AtariFramePipeline(n)
    stacks = None
    for step in range(6):
        last, prev = _frames(rng, n), _frames(rng, n)
        single = rng.random(n) < 0.3
        pipe.load([(last[i], None if single[i] else prev[i]) for i in range(n)])
        terms = rng.random(n) < 0.3
        got = (pipe.reset() if step == 0 else pipe.step(terms)).cpu().numpy()
        f = [oracle.atari_preprocess(last[i], None if single[i] else prev[i]) for i in range(n)]
        if step == 0:
            stacks = [oracle.atari_stack(None, f[i], reset=True) for i in range(n)]
        else:
            stacks = [oracle.atari_stack(stacks[i], f[i], terminal=bool(terms[i])) for i in range(n)]
        for i in range(n):
            assert np.array_equal(got[i], stacks[i]), (step, i)


@pytest.mark.gpu
def test_preprocess_wrapper_in_the_full_chain(cuda):
    from actorcritic.envs.atari import wrappers
    seed = 3
    raw_env = wrappers.wrap_atari_env(oracle.FakeALE(seed), preprocess=False)
    dev_env = wrappers.wrap_atari_env(oracle.FakeALE(seed), preprocess=True)
    o_raw, o_dev = raw_env.reset(), dev_env.reset()
    assert o_dev.shape == (84, 84, 1) and o_dev.dtype == np.uint8
    assert np.array_equal(o_dev[..., 0], oracle.atari_preprocess(o_raw))
    rng = np.random.default_rng(2)
    for _ in range(40):
        a = int(rng.integers(0, 4))
        (o_raw, r1, d1, _), (o_dev, r2, d2, _) = raw_env.step(a), dev_env.step(a)
        assert (r1, d1) == (r2, d2)
        assert np.array_equal(o_dev[..., 0], oracle.atari_preprocess(o_raw))
        if d1:
            o_raw, o_dev = raw_env.reset(), dev_env.reset()
            assert np.array_equal(o_dev[..., 0], oracle.atari_preprocess(o_raw))
