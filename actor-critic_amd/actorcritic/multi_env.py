"""Multiple environments (reference: actorcritic/multi_env.py:11-137).

``MultiEnv(envs)`` accepts either
  * a batched device env (:class:`actorcritic.envs.atari.wrappers.SyntheticAtariEnvs`):
    the hot path — one kernel steps every env, observations never leave HBM; or
  * a list of gym-like envs: the reference's semantics (each wrapped in an
    auto-reset wrapper, stepped through a ThreadPoolExecutor, ``None`` actions skip an
    env), for CPU-hosted environments.
"""

import concurrent.futures


class _AutoResetWrapper(object):
    """Resets lazily at the step after a terminal (multi_env.py:121-137)."""

    def __init__(self, env):
        self.env = env
        self._terminated = False

    @property
    def observation_space(self):
        return self.env.observation_space

    @property
    def action_space(self):
        return self.env.action_space

    def step(self, action):
        if self._terminated:
            self.env.reset()
        observation, reward, terminal, info = self.env.step(action)
        self._terminated = terminal
        return observation, reward, terminal, info

    def reset(self, **kwargs):
        observation = self.env.reset(**kwargs)
        self._terminated = False
        return observation

    def close(self):
        if hasattr(self.env, 'close'):
            self.env.close()


class MultiEnv(object):
    def __init__(self, envs):
        if hasattr(envs, 'step_into'):
            self._batched = envs
            self._envs = None
            self._executor = None
        else:
            self._batched = None
            self._envs = [_AutoResetWrapper(env) for env in envs]
            self._executor = concurrent.futures.ThreadPoolExecutor(len(self._envs))

    @property
    def batched(self):
        """The batched device env, or None for a list of host envs."""
        return self._batched

    @property
    def envs(self):
        return self._envs if self._envs is not None else self._batched

    @property
    def num_envs(self):
        return self._batched.num_envs if self._batched is not None else len(self._envs)

    @property
    def observation_space(self):
        return self._batched.observation_space if self._batched is not None else self._envs[0].observation_space

    @property
    def action_space(self):
        return self._batched.action_space if self._batched is not None else self._envs[0].action_space

    def reset(self):
        if self._batched is not None:
            return self._batched.reset()
        return list(self._executor.map(lambda env: env.reset(), self._envs))

    def step(self, actions):
        if self._batched is not None:
            return self._batched.step(actions)

        def call_step(env_action):
            env, action = env_action
            if action is None:
                return None, None, None, None
            return env.step(action)

        observations, rewards, terminals, infos = zip(*list(self._executor.map(call_step, zip(self._envs, actions))))
        return list(observations), list(rewards), list(terminals), list(infos)

    def close(self):
        if self._batched is not None:
            self._batched.close()
            return
        for env in self._envs:
            self._executor.submit(env.close)
        self._executor.shutdown()
