"""CPU tests of the host side: the C-ABI library loads and exports every symbol
include/acmi.h declares (no compute calls), layouts, the ACKTR schedule, the
oracle's internal consistency, checkpoint format, API surface errors."""
import ctypes
import os
import re
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import oracle  # noqa: E402


def _declared():
    src = open(os.path.join(ROOT, 'include', 'acmi.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(acmi_[a-z0-9_]+)\s*\(', src)))


def test_library_exports_every_declared_symbol(lib):
    from actorcritic import _lib
    declared = _declared()
    assert len(declared) >= 25
    for name in declared:
        assert hasattr(lib, name), name
        assert name in _lib.EXPORTED, 'no ctypes signature for ' + name
    assert lib.acmi_abi_version() == 4


def test_ctypes_struct_mirrors_match_the_c_abi(lib):
    """The Python binding's ctypes mirrors have the C structs' sizes (a field added
    on one side only -- e.g. acmi_rollout_io_t's step-fusion fields -- would shift
    every later field the kernels read)."""
    from actorcritic import _lib
    sizes = (ctypes.c_int64 * 5)()
    assert lib.acmi_abi_struct_sizes(ctypes.cast(sizes, ctypes.c_void_p), 5) == 5
    mirrors = (_lib.Net, _lib.Acts, _lib.Bwd, _lib.EnvState, _lib.RolloutIO)
    assert [ctypes.sizeof(m) for m in mirrors] == list(sizes)


def test_gemm_launch_plans_cover_every_tile(lib):
    # host-only planner check inside libacmi: slab groups of the fused
    # wgrad/A-factor reduction (symred.hpp) and split-K chunking
    assert lib.acmi_selftest_plans(2048) == 0


def test_layout_counts_match_survey(lib):
    # 865,413 params ACKTR / 1,686,693 A2C; 3,655,382 factor floats
    assert lib.acmi_param_count(4, 32) == 865413
    assert lib.acmi_param_count(4, 64) == 1686693
    din = (ctypes.c_int64 * 6)()
    dout = (ctypes.c_int64 * 6)()
    so = (ctypes.c_int64 * 11)()
    tot = ctypes.c_int64()
    assert lib.acmi_kfac_layout(4, 32, din, dout, so, ctypes.byref(tot)) == 0
    assert tot.value == 3655382
    assert list(din) == [257, 513, 577, 1569, 513, 513]
    assert list(dout) == [32, 64, 32, 512, 4, 1]
    off = (ctypes.c_int64 * 12)()
    assert lib.acmi_param_offsets(4, 32, off) == 0
    o, _ = oracle.param_offsets(4, 32)
    assert list(off) == o


def test_bad_arguments_report_errors(lib):
    assert lib.acmi_param_count(0, 32) < 0
    assert lib.acmi_param_count(4, 48) < 0
    off = (ctypes.c_int64 * 12)()
    assert lib.acmi_param_offsets(4, 48, off) == -1
    assert b'bad' in lib.acmi_last_error()


def test_workspace_and_mode_checks_fail_before_any_launch(lib):
    """The ABI-4 argument checks run on the host before anything is enqueued (here
    without a GPU: fake device addresses are never touched): a workspace one float
    below acmi_backward_ws_floats is ACMI_ERR_WS for both update entry points, and
    an invalid per-net mode combination (bf16 forward in f32 gemm mode) is
    ACMI_ERR_ARG.  Reference: SURVEY 8(b), model.py:180-186 (errors raised early)."""
    from actorcritic import _lib
    A, C3, B = 4, 32, 24
    fake = lambda k: ctypes.c_void_p(0x100000 * k)
    net = _lib.Net(A, C3, fake(1).value, fake(2).value)
    acts = _lib.Acts(*[fake(3 + i).value for i in range(6)], A)
    bwd = _lib.Bwd(*[fake(10 + i).value for i in range(5)], 8)
    need = lib.acmi_backward_ws_floats(B, A, C3)
    assert need > 0
    rc = lib.acmi_backward(ctypes.byref(net), fake(20), 84 * 84 * 4, B, ctypes.byref(acts), ctypes.byref(bwd),
                           fake(21), fake(22), fake(23), need - 1, None)
    assert rc == -3 and b'workspace' in lib.acmi_last_error()
    rc = lib.acmi_kfac_output_stats(ctypes.byref(net), B, ctypes.byref(acts), ctypes.byref(bwd), 7, 0, 3,
                                    fake(22), fake(23), need - 1, None)
    assert rc == -3 and b'workspace' in lib.acmi_last_error()
    bad = _lib.Net(A, C3, fake(1).value, fake(2).value, _lib.GEMM_F32 + 1, _lib.FWD_BF16 + 1, 0)
    rc = lib.acmi_backward(ctypes.byref(bad), fake(20), 84 * 84 * 4, B, ctypes.byref(acts), ctypes.byref(bwd),
                           fake(21), fake(22), fake(23), need, None)
    assert rc == -1 and b'mode' in lib.acmi_last_error()
    assert lib.acmi_get_gemm_mode() == _lib.GEMM_X3  # the failed call changed no default


def test_schedule_matches_reference_semantics():
    from actorcritic.kfac_utils import schedule
    gs = 0
    seq = []
    for _ in range(40):
        cold, cov, inv, gs2 = schedule(gs, 30, 10)
        assert (cold, cov, inv, gs2) == oracle.schedule(gs, 30, 10)
        seq.append((gs, cold, cov, inv))
        gs = gs2
    cold_iters = [s for s in seq if s[1]]
    assert len(cold_iters) == 15 and all(s[0] % 2 == 0 for s in cold_iters)  # gs advances by 2
    first_inv = [s[0] for s in seq if s[3]]
    assert first_inv[0] == 40 and first_inv[1] == 50
    assert all(s[2] for s in seq if s[0] >= 30) and not any(s[2] for s in seq if s[0] < 30)


def test_linear_decay_matches_polynomial_decay():
    from actorcritic.nn import linear_decay
    from actorcritic.session import Session, Variable, _RunContext
    step = Variable(0, 'gs')
    lr = linear_decay(0.25, 0.025, step, 100)
    for s in (0, 10, 50, 100, 150):
        step.assign(s)
        v = _RunContext(None, {}).eval(lr)
        assert v == pytest.approx(oracle.linear_decay(0.25, 0.025, s, 100))


def test_space_placeholders_follow_reference():
    from actorcritic import spaces
    from actorcritic.model import _space_placeholder
    p = _space_placeholder(spaces.Discrete(4), [None, None], 'actions')
    assert p.dtype == np.uint8 and p.shape == (None, None)
    p = _space_placeholder(spaces.Box(0, 255, (84, 84, 4), np.uint8), [None], 'obs')
    assert np.dtype(p.dtype) == np.uint8 and p.shape == (None, 84, 84, 4)
    with pytest.raises(TypeError):
        _space_placeholder(object(), [None], 'x')


def test_oracle_backward_matches_finite_differences():
    rng = np.random.default_rng(0)
    A, C3 = 4, 32
    params = oracle.init_params(A, C3, 1).astype(np.float64)
    params += rng.standard_normal(params.shape) * 0.01
    obs = rng.integers(0, 256, (2, 84, 84, 4), dtype=np.uint8)
    acts = oracle.forward(params, obs, A, C3)
    dl = rng.standard_normal((2, A))
    dv = rng.standard_normal(2)
    g, _ = oracle.backward(params, acts, dl, dv, A, C3)

    def f(p):
        a = oracle.forward(p, obs, A, C3)
        return float((a['logits'] * dl).sum() + (a['value'] * dv).sum())

    off, _ = oracle.param_offsets(A, C3)
    for idx in [off[0] + 5, off[1] + 3, off[2] + 100, off[4] + 7, off[6] + 1234, off[7] + 9, off[8] + 2,
                off[10] + 5, off[11]]:
        e = np.zeros_like(params)
        e[idx] = 1e-5
        fd = (f(params + e) - f(params - e)) / 2e-5
        assert fd == pytest.approx(g[idx], rel=1e-4, abs=1e-6)


def test_oracle_loss_gradients_match_finite_differences():
    rng = np.random.default_rng(1)
    M, A = 6, 4
    z = rng.standard_normal((M, A))
    v = rng.standard_normal(M)
    a = rng.integers(0, A, M)
    tg = rng.standard_normal(M)
    out = oracle.a2c_loss_and_head_grads(z, v, a, tg)
    adv = tg - v  # stop-gradient advantage

    def loss(z_, v_):
        lp = oracle.log_softmax(z_)
        H = -(np.exp(lp) * lp).sum(-1)
        pl = -(np.mean(adv * lp[np.arange(M), a]) + 0.01 * np.mean(H))
        bl = np.mean((tg - v_) ** 2 / 2)
        return pl + 0.5 * bl

    e = 1e-6
    for i in range(M):
        for k in range(A):
            dz = np.zeros_like(z)
            dz[i, k] = e
            fd = (loss(z + dz, v) - loss(z - dz, v)) / (2 * e)
            assert fd == pytest.approx(out['dlogits'][i, k], rel=1e-5, abs=1e-9)
        dvv = np.zeros_like(v)
        dvv[i] = e
        fd = (loss(z, v + dvv) - loss(z, v - dvv)) / (2 * e)
        assert fd == pytest.approx(out['dvalue'][i], rel=1e-5, abs=1e-9)


def test_sharded_statistics_average_to_full_batch():
    """The data-parallel contract: the mean of per-shard factor
    statistics and mean-loss gradients equals the full-batch values."""
    rng = np.random.default_rng(2)
    A, C3 = 4, 32
    params = oracle.init_params(A, C3, 0)
    obs = rng.integers(0, 256, (4, 84, 84, 4), dtype=np.uint8)
    full = oracle.forward(params, obs, A, C3)
    af_full = oracle.a_factors(full)
    shards = [oracle.a_factors(oracle.forward(params, obs[i:i + 2], A, C3)) for i in (0, 2)]
    for f in range(5):
        np.testing.assert_allclose((shards[0][f] + shards[1][f]) / 2, af_full[f], rtol=1e-10, atol=1e-12)
    dl = rng.standard_normal((4, A)) / 4
    dv = rng.standard_normal(4) / 4
    g_full, _ = oracle.backward(params, full, dl, dv, A, C3)
    g_sh = [oracle.backward(params, oracle.forward(params, obs[i:i + 2], A, C3), dl[i:i + 2] * 2, dv[i:i + 2] * 2,
                            A, C3)[0] for i in (0, 2)]
    np.testing.assert_allclose((g_sh[0] + g_sh[1]) / 2, g_full, rtol=1e-9, atol=1e-12)


def test_atari57_game_table_and_names():
    """Mixed-game synthetic Atari-57 (BASELINE configs[4]): the oracle's game table keeps
    Breakout on the default dynamics, gives every other game its own salt, ranges inside
    the documented bounds, and the host name table matches the device action table."""
    sys.path.insert(0, os.path.join(ROOT, 'actor-critic_amd'))
    from actorcritic.envs.atari import wrappers
    assert len(wrappers.ATARI57) == 57 == len(wrappers.ATARI57_ACTIONS) == len(oracle.GAME_ACTIONS)
    assert tuple(wrappers.ATARI57_ACTIONS) == tuple(oracle.GAME_ACTIONS)
    assert wrappers.ATARI57[oracle.GAME_BREAKOUT] == 'Breakout'
    assert oracle.game_params(None) == (0, 50, 451, oracle.REW_LO, oracle.REW_HI, 256)
    assert oracle.game_params(oracle.GAME_BREAKOUT)[:5] == oracle.game_params(None)[:5]
    salts = set()
    for g in range(57):
        salt, lmin, lspan, lo, hi, nl = oracle.game_params(g)
        salts.add(salt)
        if g == oracle.GAME_BREAKOUT:
            continue
        assert 30 <= lmin <= 200 and 100 <= lspan <= 2000
        assert 0 <= lo < 0.05 * 2 ** 24 and 0.8 * 2 ** 24 <= hi < (1 - 0.005) * 2 ** 24 + 1
        assert nl == wrappers.ATARI57_ACTIONS[g]
    assert len(salts) == 57
    assert wrappers.game_index('PongNoFrameskip-v4') == wrappers.ATARI57.index('Pong')
    assert wrappers.game_index('BreakoutNoFrameskip-v4') == oracle.GAME_BREAKOUT
    assert wrappers.game_index('Asterix') != wrappers.game_index('Asteroids')
    with pytest.raises(ValueError):
        wrappers.game_index('NotAGame')
    # the default game is the same env as before the game table (golden traces)
    e = oracle.SyntheticAtari(5, 2)
    f = oracle.SyntheticAtari(5, 2, game=oracle.GAME_BREAKOUT)
    np.testing.assert_array_equal(e.reset(), f.reset())
    for t in range(80):
        a, b = e.step(t % 4), f.step(t % 4)
        np.testing.assert_array_equal(a[0], b[0])
        assert a[1:3] == b[1:3]
    # an illegal action of a 3-action game steps as NOOP
    g = wrappers.ATARI57.index('Freeway')
    x, y = oracle.SyntheticAtari(5, 0, game=g), oracle.SyntheticAtari(5, 0, game=g)
    x.reset(), y.reset()
    np.testing.assert_array_equal(x.step(17)[0], y.step(0)[0])
