"""SubprocessEnv / create_subprocess_envs / MultiEnv list path (reference:
actorcritic/multi_env.py:11-362): Pipe protocol, lazy auto-reset, ``None`` actions,
the child-restart path and the ValueError contract.  CPU only."""

import os

import pytest

from actorcritic import spaces
from actorcritic.multi_env import MultiEnv, SubprocessEnv, create_subprocess_envs


class CountingEnv(object):
    """Episode of `length` steps; observation = (episode, step); action 99 kills the
    process (to exercise the restart path)."""

    def __init__(self, length=3):
        self.length = length
        self.episode = -1
        self.t = 0
        self.action_space = spaces.Discrete(4)
        self.observation_space = spaces.Box(0, 255, (2,), 'uint8')

    def reset(self, start=0):
        self.episode += 1
        self.t = start
        return (self.episode, self.t)

    def step(self, action):
        if action == 99:
            os._exit(3)
        self.t += 1
        return (self.episode, self.t), float(action), self.t >= self.length, {'pid': os.getpid()}

    def render(self, mode='human'):
        return 'render:{}'.format(mode)


def make_env():
    return CountingEnv()


def test_protocol_and_errors():
    env = SubprocessEnv(make_env)
    with pytest.raises(ValueError):
        env.step(0)
    with pytest.raises(ValueError):
        env.initialize()
    env.start()
    with pytest.raises(ValueError):
        _ = env.action_space
    env.initialize()
    assert env.action_space.n == 4
    assert env.observation_space.shape == (2,)
    assert env.reset() == (0, 0)
    assert env.reset(start=5) == (1, 5)
    obs, r, term, info = env.step(2)
    assert obs == (1, 6) and r == 2.0 and term and info['pid'] != os.getpid()
    assert env.render() == 'render:human'
    assert env.render('rgb_array') == 'render:rgb_array'
    env.close()
    with pytest.raises(ValueError):
        env.close()
    with pytest.raises(ValueError):
        env.step(0)


def test_child_crash_restarts_transparently():
    env = SubprocessEnv(make_env)
    # children (restarts included) are fresh interpreters, never forks of a parent
    # that may have initialised HIP
    assert env._ctx.get_start_method() == 'spawn'
    env.start()
    env.initialize()
    env.reset()
    pid0 = env.step(1)[3]['pid']
    # the killed child is restarted, re-initialised and reset, then the action is
    # sent again -- to the new child, which dies again on 99: use a normal action
    env._parent_connection.send((SubprocessEnv._Command.STEP, 99))
    try:
        env._parent_connection.recv()
    except EOFError:
        pass
    obs, r, term, info = env.step(1)
    assert env.restarts == 1
    assert info['pid'] != pid0
    # new env: reset once by the restart path (episode 0), then one step
    assert obs == (0, 1) and r == 1.0 and not term
    env.close()


def test_multi_env_auto_reset_and_none_actions():
    envs = create_subprocess_envs([make_env, make_env])
    multi = MultiEnv(envs)
    assert multi.action_space.n == 4
    assert multi.reset() == [(0, 0), (0, 0)]
    for t in range(1, 4):
        obs, rew, term, infos = multi.step([1, None])
        assert obs[0] == (0, t) and obs[1] is None and rew[1] is None
        assert term[0] == (t == 3)
    # the reset after the terminal happens lazily inside the next step and its
    # observation is never emitted
    obs, rew, term, infos = multi.step([0, 0])
    assert obs == [(1, 1), (0, 1)]
    multi.close()


def test_unpicklable_env_fn_names_the_fix():
    """A lambda env_fn (fine under the reference's fork) fails at start() under the
    default spawn context with a ValueError that says what to pass instead."""
    env = SubprocessEnv(lambda: CountingEnv())
    with pytest.raises(ValueError, match="picklable env_fn.*functools.partial.*context='fork'"):
        env.start()
