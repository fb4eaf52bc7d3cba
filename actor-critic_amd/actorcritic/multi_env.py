"""Multiple environments (reference: actorcritic/multi_env.py:11-137).

``MultiEnv(envs)`` accepts either
  * a batched device env (:class:`actorcritic.envs.atari.wrappers.SyntheticAtariEnvs`):
    the hot path — one kernel steps every env, observations never leave HBM; or
  * a list of gym-like envs: the reference's semantics (each wrapped in an
    auto-reset wrapper, stepped through a ThreadPoolExecutor, ``None`` actions skip an
    env), for CPU-hosted environments, typically :class:`SubprocessEnv` instances from
    :func:`create_subprocess_envs` (multi_env.py:92-362).
"""

import concurrent.futures
import multiprocessing
import pickle


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


def create_subprocess_envs(env_fns, context='spawn'):
    """Creates one :class:`SubprocessEnv` per function, starts them all, then
    initialises them in parallel (multi_env.py:92-118)."""
    envs = []
    for env_fn in env_fns:
        env = SubprocessEnv(env_fn, context=context)
        env.start()
        envs.append(env)
    with concurrent.futures.ThreadPoolExecutor(max(1, len(envs))) as executor:
        for f in [executor.submit(env.initialize) for env in envs]:
            f.result()
    return envs


class SubprocessEnv(object):
    """A host environment in its own process behind a duplex Pipe (multi_env.py:140-362):
    for CPU-hosted (e.g. real gym/ALE) envs behind the list form of :class:`MultiEnv`;
    the hot path uses the batched device stepper instead.

    Protocol (parent sends ``(command, arg)``, child answers one response):
    INIT -> ``(action_space, observation_space)`` (the child calls ``env_fn`` here),
    STEP -> ``env.step(arg)``, RESET -> ``env.reset(**(arg or {}))``,
    RENDER -> ``env.render(arg or 'human')``, CLOSE -> no answer, child exits.
    A lost connection (child died) restarts the child transparently: re-INIT, then a
    RESET unless the failed command was one, then the command again
    (multi_env.py:217-239).  Errors: ValueError when used before start()/initialize()
    or after close() (multi_env.py:171-184).
    """

    class _Command:
        INIT, STEP, RESET, RENDER, CLOSE = range(5)

    def __init__(self, env_fn, context='spawn'):
        # 'spawn' by default: every child -- including one the restart path starts
        # mid-training, after this process has initialised HIP -- is a fresh
        # interpreter, never a fork of a GPU-initialised address space.  env_fn must
        # therefore be picklable (a module-level function or functools.partial);
        # context='fork' restores the reference's behaviour for CPU-only parents.
        self._env_fn = env_fn
        self._ctx = multiprocessing.get_context(context)
        self._parent_connection = self._child_connection = self._process = None
        self._started = False
        self._initialized = False
        self._action_space = None
        self._observation_space = None
        self.restarts = 0
        self._new_process()

    def _new_process(self):
        self._started = False
        self._initialized = False
        self._parent_connection, self._child_connection = self._ctx.Pipe(duplex=True)
        self._process = self._ctx.Process(target=_subprocess_env_worker,
                                          args=(self._child_connection, self._env_fn), name='SubprocessEnv')
        self._process.daemon = True

    def _check_closed(self):
        if self._process is None:
            raise ValueError('The subprocess was closed already.')

    def _check_initialized(self, method):
        self._check_closed()
        if not self._started:
            raise ValueError("The subprocess is not started yet. Call 'start()' and 'initialize()' before "
                             "calling '{}'.".format(method))
        if not self._initialized:
            raise ValueError("The subprocess is not initialized yet. Call 'initialize()' before calling "
                             "'{}'.".format(method))

    def start(self):
        """Starts the child process (does not block)."""
        self._check_closed()
        if not self._started:
            try:
                self._process.start()
            except (pickle.PicklingError, AttributeError, TypeError) as e:
                if self._ctx.get_start_method() == 'fork':
                    raise
                # the reference forks (multi_env.py:140-160), so a lambda or closure
                # env_fn worked there; under 'spawn' it has to cross a pickle
                raise ValueError(
                    "env_fn {!r} cannot be sent to a '{}' child process ({}: {}). Pass a picklable "
                    "env_fn -- a module-level function or a functools.partial of one -- or "
                    "SubprocessEnv(env_fn, context='fork') / create_subprocess_envs(env_fns, "
                    "context='fork') from a parent that has not initialised the GPU."
                    .format(self._env_fn, self._ctx.get_start_method(), type(e).__name__, e)) from e
            self._child_connection.close()
            self._started = True

    def initialize(self):
        """Creates the env in the child and fetches its spaces (blocks)."""
        self._check_closed()
        if not self._started:
            raise ValueError("The subprocess is not started yet. Call 'start()' before 'initialize()'.")
        if not self._initialized:
            self._action_space, self._observation_space = self._communicate(SubprocessEnv._Command.INIT)
            self._initialized = True

    def _send_recv(self, command, arg=None):
        self._parent_connection.send((command, arg))
        return self._parent_connection.recv()

    def _communicate(self, command, arg=None):
        try:
            return self._send_recv(command, arg)
        except (BrokenPipeError, ConnectionResetError, EOFError):
            self._parent_connection.close()
            self._process.terminate()
            self._process.join()
            self.restarts += 1
            self._new_process()
            self.start()
            self._action_space, self._observation_space = self._send_recv(SubprocessEnv._Command.INIT)
            self._initialized = True
            if command == SubprocessEnv._Command.INIT:
                return self._action_space, self._observation_space
            if command != SubprocessEnv._Command.RESET:
                self._send_recv(SubprocessEnv._Command.RESET)
            return self._send_recv(command, arg)

    @property
    def action_space(self):
        self._check_initialized('action_space')
        return self._action_space

    @property
    def observation_space(self):
        self._check_initialized('observation_space')
        return self._observation_space

    def step(self, action):
        self._check_initialized('step()')
        return self._communicate(SubprocessEnv._Command.STEP, action)

    def reset(self, **kwargs):
        self._check_initialized('reset()')
        return self._communicate(SubprocessEnv._Command.RESET, kwargs)

    def render(self, mode='human'):
        self._check_initialized('render()')
        return self._communicate(SubprocessEnv._Command.RENDER, None if mode == 'human' else mode)

    def close(self):
        """Stops the child (idempotence is the caller's: a second close raises ValueError)."""
        self._check_closed()
        if self._started:
            try:
                if self._process.is_alive():
                    self._parent_connection.send((SubprocessEnv._Command.CLOSE, None))
                self._parent_connection.close()
            except (BrokenPipeError, ConnectionResetError, EOFError):
                pass
            self._process.join()
        self._started = False
        self._initialized = False
        self._process = None


def _subprocess_env_worker(connection, env_fn):
    """Child loop of :class:`SubprocessEnv` (multi_env.py:331-362)."""
    env = None
    try:
        while True:
            command, arg = connection.recv()
            if command == SubprocessEnv._Command.CLOSE:
                break
            if command == SubprocessEnv._Command.INIT:
                env = env_fn()
                response = (env.action_space, env.observation_space)
            elif command == SubprocessEnv._Command.STEP:
                response = env.step(arg)
            elif command == SubprocessEnv._Command.RESET:
                response = env.reset(**(arg or {}))
            elif command == SubprocessEnv._Command.RENDER:
                response = env.render(arg if arg is not None else 'human')
            else:
                response = None
            connection.send(response)
    except (KeyboardInterrupt, EOFError):
        pass
    if env is not None and hasattr(env, 'close'):
        env.close()
    connection.close()
