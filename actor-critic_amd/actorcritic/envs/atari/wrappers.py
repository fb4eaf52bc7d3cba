"""Atari environments on the device (reference: actorcritic/envs/atari/wrappers.py).

:class:`SyntheticAtariEnvs` is the batched stepper that replaces the reference's
SubprocessEnv-per-env + FrameStackWrapper + EpisodeInfoWrapper stack for the hot path:
one HIP workgroup per env produces a synthetic 84x84 u8 frame from a counter hash of
(seed, env, episode, step, action), updates the 4-frame stack in place with the
reference semantics (np.roll then zero-fill on a terminal, wrappers.py:224-230), resets
lazily at the step after a terminal (multi_env.py:127-132: the reset observation is
never emitted), and tracks the EpisodeInfoWrapper total reward (wrappers.py:263-294).

Real ALE emulation and the frame preprocessing wrappers (wrappers.py:16-198) are out of
the hot-path scope.
"""

import ctypes

import numpy as np
import torch

from actorcritic import _lib, spaces
from actorcritic._engine import OBS_BYTES

# Breakout has 4 actions; the full Atari action set has 18
ATARI_NUM_ACTIONS = {'Breakout': 4, 'Pong': 6, 'SpaceInvaders': 6, 'Seaquest': 18, 'BeamRider': 9,
                     'Qbert': 6, 'Enduro': 9, 'MsPacman': 9, 'Asteroids': 14}


# Atari-57 (the usual benchmark list, alphabetical) with each game's minimal action-set
# size; the mixed-game synthetic stepper indexes games in this order (csrc/stepper.hpp
# kGameActions, oracle.GAME_ACTIONS).  Under the full 18-action set a game's actions
# past its minimal set step as NOOP.
ATARI57 = ('Alien', 'Amidar', 'Assault', 'Asterix', 'Asteroids', 'Atlantis', 'BankHeist', 'BattleZone',
           'BeamRider', 'Berzerk', 'Bowling', 'Boxing', 'Breakout', 'Centipede', 'ChopperCommand',
           'CrazyClimber', 'Defender', 'DemonAttack', 'DoubleDunk', 'Enduro', 'FishingDerby', 'Freeway',
           'Frostbite', 'Gopher', 'Gravitar', 'Hero', 'IceHockey', 'Jamesbond', 'Kangaroo', 'Krull',
           'KungFuMaster', 'MontezumaRevenge', 'MsPacman', 'NameThisGame', 'Phoenix', 'Pitfall', 'Pong',
           'PrivateEye', 'Qbert', 'Riverraid', 'RoadRunner', 'Robotank', 'Seaquest', 'Skiing', 'Solaris',
           'SpaceInvaders', 'StarGunner', 'Surround', 'Tennis', 'TimePilot', 'Tutankham', 'UpNDown', 'Venture',
           'VideoPinball', 'WizardOfWor', 'YarsRevenge', 'Zaxxon')
ATARI57_ACTIONS = (18, 10, 7, 9, 14, 4, 18, 18, 9, 18, 6, 18, 4, 18, 18, 9, 18, 6, 18, 9, 18, 3, 18, 8, 18, 18,
                   18, 18, 18, 18, 14, 18, 9, 6, 8, 18, 6, 18, 6, 18, 18, 18, 18, 3, 18, 6, 18, 5, 18, 10, 8,
                   6, 18, 9, 10, 18, 18)


def game_index(name):
    """Index of an Atari-57 game ('Pong', 'PongNoFrameskip-v4', or an int)."""
    if isinstance(name, (int, np.integer)):
        if not 0 <= int(name) < len(ATARI57):
            raise ValueError('game index {} out of range [0, {})'.format(name, len(ATARI57)))
        return int(name)
    hits = [i for i, g in enumerate(ATARI57) if name.startswith(g)]  # 'PongNoFrameskip-v4' -> Pong
    if hits:
        return max(hits, key=lambda i: len(ATARI57[i]))
    raise ValueError('unknown Atari-57 game {!r}'.format(name))


def num_actions_for(env_id):
    for k, v in ATARI_NUM_ACTIONS.items():
        if env_id.startswith(k):
            return v
    return 18


class EpisodeInfoBatch(object):
    """Batch-major [env, step] episode rewards (NaN where no episode ended): the device
    form of the infos the reference's EpisodeInfoWrapper writes."""

    def __init__(self, episode_rewards):
        self.episode_rewards = episode_rewards

    def __len__(self):
        return self.episode_rewards.shape[0]


class Wrapper(object):
    """gym.Wrapper's forwarding contract without gym (not a dependency here): step/reset/
    render/close go to the wrapped env, unknown public attributes are looked up on it."""

    def __init__(self, env):
        self.env = env
        self.observation_space = getattr(env, 'observation_space', None)
        self.action_space = getattr(env, 'action_space', None)

    def __getattr__(self, name):
        if name.startswith('_') or name == 'env':
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return getattr(self.env, 'unwrapped', self.env)

    def step(self, action):
        return self.env.step(action)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)

    def render(self, *args, **kwargs):
        return self.env.render(*args, **kwargs)

    def close(self):
        close = getattr(self.env, 'close', None)
        return close() if close is not None else None


class ObservationWrapper(Wrapper):
    def step(self, action):
        observation, reward, terminal, info = self.env.step(action)
        return self.observation(observation), reward, terminal, info

    def reset(self, **kwargs):
        return self.observation(self.env.reset(**kwargs))


class RewardWrapper(Wrapper):
    def step(self, action):
        observation, reward, terminal, info = self.env.step(action)
        return observation, self.reward(reward), terminal, info


class EpisodeInfoWrapper(Wrapper):
    """Stores {'total_reward': ...} under info['episode'] at the end of an episode
    (wrappers.py:263-294); the static helper also reads the device EpisodeInfoBatch."""

    def __init__(self, env):
        super().__init__(env)
        self.total_reward = 0.0

    def step(self, action):
        observation, reward, terminal, info = self.env.step(action)
        self.total_reward += reward
        if terminal:
            info['episode'] = {'total_reward': self.total_reward}
            self.total_reward = 0.0
        return observation, reward, terminal, info

    def reset(self, **kwargs):
        self.total_reward = 0.0
        return self.env.reset(**kwargs)

    @staticmethod
    def get_episode_rewards_from_info_batch(infos):
        """[env, step] float32 array of episode rewards, NaN elsewhere (wrappers.py:296-323)."""
        if isinstance(infos, EpisodeInfoBatch):
            return infos.episode_rewards.detach().cpu().numpy().astype(np.float32)
        rewards = np.full((len(infos), len(infos[0]) if len(infos) else 0), np.nan, np.float32)
        for e, row in enumerate(infos):
            for t, info in enumerate(row):
                if info and 'episode' in info:
                    rewards[e, t] = info['episode']['total_reward']
        return rewards


class SyntheticAtariEnvs(object):
    """A batch of synthetic Atari games with frame stacking, on one GPU.

    Args:
        num_envs: environments on this device.
        num_actions: size of the Discrete action space (Breakout 4).
        seed: game seed (frames, rewards, episode lengths are pure functions of it).
        env_offset: global id of the first env (data-parallel shards use rank*num_envs).
        games: None (every env the default game: Breakout's dynamics), 'atari57' (global
            env e plays ATARI57[e % 57]: a mixed-game batch, BASELINE configs[4]), or one
            game (name / index) per env.  Mixed batches need num_actions = 18 (the full
            action set every game accepts).
    """

    def __init__(self, num_envs, num_actions=4, seed=0, env_offset=0, device=None, games=None):
        _lib.require_gpu()
        self.num_envs = int(num_envs)
        self.seed = int(seed) & 0xFFFFFFFF
        self.env_offset = int(env_offset)
        self.device = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
        self.observation_space = spaces.Box(low=0, high=255, shape=(84, 84, 4), dtype=np.uint8)
        self.action_space = spaces.Discrete(num_actions)
        N = self.num_envs
        z = lambda dt: torch.zeros(N, dtype=dt, device=self.device)
        self._episode, self._step, self._length = z(torch.int32), z(torch.int32), z(torch.int32)
        self._total, self._done = z(torch.float32), z(torch.uint8)
        self.games = None
        if games is not None:
            if isinstance(games, str) and games == 'atari57':
                idx = [(self.env_offset + n) % len(ATARI57) for n in range(N)]
            else:
                idx = [game_index(g) for g in games]
                if len(idx) != N:
                    raise ValueError('games: {} entries for {} envs'.format(len(idx), N))
            if len(set(idx)) > 1 and num_actions != 18:
                raise ValueError('a mixed-game batch needs the full action set (num_actions=18)')
            if max(ATARI57_ACTIONS[i] for i in idx) > num_actions:
                raise ValueError('num_actions={} is smaller than a game\'s action set'.format(num_actions))
            self.games = torch.tensor(idx, dtype=torch.uint8, device=self.device)
        self.state = _lib.EnvState(self._episode.data_ptr(), self._step.data_ptr(), self._length.data_ptr(),
                                   self._total.data_ptr(), self._done.data_ptr(), self._game_ptr(0))
        self._obs = torch.zeros((N, 84, 84, 4), dtype=torch.uint8, device=self.device)

    def _stream(self):
        return _lib.stream_handle(self.device)

    def _game_ptr(self, n0):
        return None if self.games is None else self.games[n0:].data_ptr()

    def reset_into(self, obs_ptr, stride=OBS_BYTES):
        _lib.call('acmi_env_reset', ctypes.byref(self.state), self.num_envs, self.env_offset, self.seed,
                  ctypes.c_void_p(obs_ptr), stride, self._stream())

    def step_into(self, actions_ptr, obs_in_ptr, in_stride, obs_out_ptr, out_stride, rew_ptr, term_ptr, ep_ptr, ld):
        _lib.call('acmi_env_step', ctypes.byref(self.state), self.num_envs, self.env_offset, self.seed,
                  ctypes.c_void_p(actions_ptr), ctypes.c_void_p(obs_in_ptr), in_stride, ctypes.c_void_p(obs_out_ptr),
                  out_stride, ctypes.c_void_p(rew_ptr), ctypes.c_void_p(term_ptr), ctypes.c_void_p(ep_ptr), ld,
                  self._stream())

    def range_state(self, n0):
        """EnvState of envs n0.. (pointers at env n0)."""
        if n0 == 0:
            return self.state
        if not hasattr(self, '_range_states'):
            self._range_states = {}
        st = self._range_states.get(n0)
        if st is None:
            st = _lib.EnvState(self._episode[n0:].data_ptr(), self._step[n0:].data_ptr(),
                               self._length[n0:].data_ptr(), self._total[n0:].data_ptr(),
                               self._done[n0:].data_ptr(), self._game_ptr(n0))
            self._range_states[n0] = st
        return st

    def step_range_into(self, n0, n, actions_ptr, obs_in_ptr, in_stride, obs_out_ptr, out_stride, rew_ptr,
                        term_ptr, ep_ptr, ld):
        """step_into for envs n0 .. n0+n-1 only (every pointer already at env n0)."""
        st = self.range_state(n0)
        _lib.call('acmi_env_step', ctypes.byref(st), n, self.env_offset + n0, self.seed,
                  ctypes.c_void_p(actions_ptr), ctypes.c_void_p(obs_in_ptr), in_stride, ctypes.c_void_p(obs_out_ptr),
                  out_stride, ctypes.c_void_p(rew_ptr), ctypes.c_void_p(term_ptr), ctypes.c_void_p(ep_ptr), ld,
                  self._stream())

    # -- gym-like batched API --------------------------------------------------
    def reset(self):
        self.reset_into(self._obs.data_ptr())
        return self._obs.clone()

    def step(self, actions):
        """actions: [N] ints -> (obs [N,84,84,4] u8, rewards [N], terminals [N] bool, EpisodeInfoBatch)."""
        a = actions if isinstance(actions, torch.Tensor) else torch.as_tensor(np.asarray(actions))
        a = a.to(device=self.device, dtype=torch.int32).contiguous()
        N = self.num_envs
        rew = torch.empty(N, dtype=torch.float32, device=self.device)
        term = torch.empty(N, dtype=torch.uint8, device=self.device)
        ep = torch.empty(N, dtype=torch.float32, device=self.device)
        self.step_into(a.data_ptr(), self._obs.data_ptr(), OBS_BYTES, self._obs.data_ptr(), OBS_BYTES,
                       rew.data_ptr(), term.data_ptr(), ep.data_ptr(), 1)
        return self._obs.clone(), rew, term.view(torch.bool), EpisodeInfoBatch(ep[:, None])

    def close(self):
        pass


# ---------------------------------------------------------------------------
# Real (raw RGB) Atari frames: the reference's per-env wrapper chain
# (wrappers.py:16-260, assembled by make_atari_env, a2c_acktr.py:175-213).  The
# control-flow wrappers are host objects with the reference's semantics; the frame
# arithmetic (gray + INTER_AREA resize, frame stacking) runs on the device through
# acmi_atari_preprocess / acmi_atari_stack, batched in AtariFramePipeline.
# ---------------------------------------------------------------------------
RAW_HEIGHT, RAW_WIDTH = 210, 160


def _device_of(device):
    _lib.require_gpu()
    return torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())


def preprocess_frames(raw, prev=None, out=None):
    """Device preprocessing of a batch: raw [N,H,W,3] u8 (the last frames), optional prev
    [N,H,W,3] (max-pooled with them, wrappers.py:64-65) -> gray [N,84,84] u8
    (cv2 RGB2GRAY + INTER_AREA, wrappers.py:30-33)."""
    if raw.dim() != 4 or raw.shape[-1] != 3 or raw.dtype != torch.uint8 or not raw.is_cuda:
        raise ValueError('raw must be a [N, H, W, 3] uint8 cuda tensor')
    N, H, W, _ = raw.shape
    if prev is not None:
        frames = torch.stack([raw, prev.to(raw.device)], 1).contiguous()
        env_stride, frame_stride = frames.stride(0), frames.stride(1)
    else:
        frames = raw.contiguous()
        env_stride, frame_stride = frames.stride(0), 0
    if out is None:
        out = torch.empty((N, 84, 84), dtype=torch.uint8, device=raw.device)
    _lib.call('acmi_atari_preprocess', ctypes.c_void_p(frames.data_ptr()), env_stride, frame_stride, None, N, H,
              W, ctypes.c_void_p(out.data_ptr()), out.stride(0), _lib.stream_handle(raw.device))
    return out


class AtariFramePipeline(object):
    """Frameskip max + gray/resize + 4-frame stack for N envs in one launch per step.

    ``raw`` [N, 2, H, W, 3] u8 on the device holds each env's last frame in slot 0 and
    the frame before it in slot 1; ``nframes`` [N] says how many of them the frameskip
    produced (1 when the episode ended on the first skipped frame, wrappers.py:58-67).
    ``stacks`` [N, 84, 84, 4] u8 are the FrameStackWrapper observations.
    """

    def __init__(self, num_envs, height=RAW_HEIGHT, width=RAW_WIDTH, device=None):
        self.device = _device_of(device)
        self.num_envs, self.height, self.width = int(num_envs), int(height), int(width)
        N = self.num_envs
        self.raw = torch.zeros((N, 2, self.height, self.width, 3), dtype=torch.uint8, device=self.device)
        self.nframes = torch.full((N,), 2, dtype=torch.uint8, device=self.device)
        self.stacks = torch.zeros((N, 84, 84, 4), dtype=torch.uint8, device=self.device)
        self._host = None

    def load(self, frames):
        """Upload host frames: a list of N (last, prev_or_None) raw [H,W,3] u8 pairs (the
        two frames an AtariFrameskipWrapper would max-pool) in one pinned copy."""
        if self._host is None:
            self._host = torch.empty(self.raw.shape, dtype=torch.uint8).pin_memory()
            self._host_n = torch.empty((self.num_envs,), dtype=torch.uint8).pin_memory()
        torch.cuda.current_stream(self.device).synchronize()  # the previous upload has landed
        h, hn = self._host.numpy(), self._host_n.numpy()
        for n, (last, prev) in enumerate(frames):
            h[n, 0] = last
            if prev is not None:
                h[n, 1] = prev
            hn[n] = 1 if prev is None else 2
        self.raw.copy_(self._host, non_blocking=True)
        self.nframes.copy_(self._host_n, non_blocking=True)

    def _launch(self, terminals, reset):
        term = None
        if terminals is not None:
            t = terminals if isinstance(terminals, torch.Tensor) else torch.as_tensor(np.asarray(terminals))
            term = t.to(device=self.device, dtype=torch.uint8).contiguous()
        r = self.raw
        _lib.call('acmi_atari_stack', ctypes.c_void_p(r.data_ptr()), r.stride(0), r.stride(1),
                  ctypes.c_void_p(self.nframes.data_ptr()), self.num_envs, self.height, self.width,
                  None if term is None else ctypes.c_void_p(term.data_ptr()), int(reset),
                  ctypes.c_void_p(self.stacks.data_ptr()), ctypes.c_void_p(self.stacks.data_ptr()),
                  self.stacks.stride(0), _lib.stream_handle(self.device))
        return self.stacks

    def reset(self):
        """FrameStackWrapper.reset of every env from its current raw frame(s)."""
        return self._launch(None, True)

    def step(self, terminals=None):
        """FrameStackWrapper.step of every env: roll, zero where terminal, insert."""
        return self._launch(terminals, False)


class AtariPreprocessFrameWrapper(ObservationWrapper):
    """RGB -> gray, 210x160 -> 84x84 (wrappers.py:16-33) on the device."""

    def __init__(self, env, device=None):
        super().__init__(env)
        self.observation_space = spaces.Box(low=0, high=255, shape=(84, 84, 1), dtype=np.uint8)
        self._device = _device_of(device)

    def observation(self, frame):
        raw = torch.as_tensor(np.ascontiguousarray(frame)).to(self._device)[None]
        out = preprocess_frames(raw)
        return out[0].cpu().numpy()[..., None]


class AtariFrameskipWrapper(Wrapper):
    """Repeats the action `frameskip` times; the observation is the max of the last two
    frames (wrappers.py:36-70)."""

    def __init__(self, env, frameskip):
        super().__init__(env)
        self._frameskip = frameskip

    def step(self, action):
        frames = []
        total_reward = 0.0
        terminal = False
        info = None
        for _ in range(self._frameskip):
            next_frame, reward, terminal, info = self.env.step(action)
            frames.append(next_frame)
            total_reward += reward
            if terminal:
                break
        if len(frames) >= 2:
            return np.amax((frames[-2], frames[-1]), axis=0), total_reward, terminal, info
        return frames[0], total_reward, terminal, info


class AtariClipRewardWrapper(RewardWrapper):
    """Rewards clipped to [-1, 1] (wrappers.py:73-86)."""

    def reward(self, reward):
        return np.clip(reward, -1., 1.)


class AtariEpisodicLifeWrapper(Wrapper):
    """A lost life ends the (training) episode; the game resets only when it is really
    over (wrappers.py:89-117)."""

    def __init__(self, env):
        super().__init__(env)
        self.lives = 0
        self.episode_terminal = True

    def step(self, action):
        next_observation, reward, terminal, info = self.env.step(action)
        self.episode_terminal = terminal
        next_lives = info['ale.lives']
        if next_lives < self.lives:
            terminal = True
        self.lives = next_lives
        return next_observation, reward, terminal, info

    def reset(self, **kwargs):
        if self.episode_terminal:
            self.env.reset(**kwargs)
        observation, _, terminal, info = self.env.step(0)  # NOOP
        self.lives = info['ale.lives']
        return observation


class AtariFireResetWrapper(Wrapper):
    """FIRE after a reset (wrappers.py:120-141)."""

    def reset(self, **kwargs):
        self.env.reset(**kwargs)
        observation, _, terminal, _ = self.env.step(1)  # FIRE
        if terminal:
            print('WARNING')
            observation = self.env.reset(**kwargs)
        return observation


class AtariNoopResetWrapper(Wrapper):
    """1..noop_max NOOPs after a reset, drawn from the unwrapped env's np_random
    (wrappers.py:144-170)."""

    def __init__(self, env, noop_max):
        super().__init__(env)
        self.noop_max = noop_max

    def reset(self, **kwargs):
        observation = self.env.reset(**kwargs)
        num_noops = self.unwrapped.np_random.randint(1, self.noop_max + 1)
        for _ in range(num_noops):
            observation, _, terminal, _ = self.env.step(0)  # NOOP
            if terminal:
                observation = self.env.reset(**kwargs)
        return observation


class RenderWrapper(Wrapper):
    """render() every step, optionally throttled to `fps` (wrappers.py:173-198)."""

    def __init__(self, env, fps=None):
        super().__init__(env)
        self._spf = 1.0 / fps if fps is not None else None

    def step(self, action):
        import time
        self.env.render()
        if self._spf is not None:
            time.sleep(self._spf)
        return self.env.step(action)


class FrameStackWrapper(Wrapper):
    """Host form of the 4-frame stack (wrappers.py:201-235) for list-path envs; the
    batched device form is AtariFramePipeline / the synthetic stepper."""

    def __init__(self, env, num_stacked_frames):
        super().__init__(env)
        self._num_stacked_frames = num_stacked_frames
        low = np.repeat(env.observation_space.low, num_stacked_frames, axis=-1)
        # the reference builds `high` from `low` too (wrappers.py:219)
        self.observation_space = spaces.Box(low=low, high=low.copy(), dtype=env.observation_space.dtype)
        self._stacked_frames = np.zeros_like(low)

    def step(self, action):
        next_frame, reward, terminal, info = self.env.step(action)
        self._stacked_frames = np.roll(self._stacked_frames, shift=-1, axis=-1)
        if terminal:
            self._stacked_frames.fill(0)
        self._stacked_frames[..., -1:] = next_frame
        return self._stacked_frames, reward, terminal, info

    def reset(self, **kwargs):
        frame = self.env.reset(**kwargs)
        self._stacked_frames = np.repeat(frame, self._num_stacked_frames, axis=-1)
        return self._stacked_frames


class AtariInfoClearWrapper(Wrapper):
    """Drops info['ale.lives'] (wrappers.py:238-260)."""

    def step(self, action):
        observation, reward, terminal, info = self.env.step(action)
        del info['ale.lives']
        return observation, reward, terminal, info


def wrap_atari_env(env, render=False, preprocess=True, device=None):
    """The make_atari_env chain (a2c_acktr.py:190-213) around an ALE-like env (step ->
    (frame, reward, terminal, {'ale.lives': ...}), unwrapped.np_random).  With
    preprocess=False the frames stay raw RGB, for a batched AtariFramePipeline."""
    env = AtariNoopResetWrapper(env, noop_max=30)
    env = AtariFrameskipWrapper(env, frameskip=4)
    if preprocess:
        env = AtariPreprocessFrameWrapper(env, device=device)
    env = EpisodeInfoWrapper(env)
    env = AtariEpisodicLifeWrapper(env)
    env = AtariFireResetWrapper(env)
    env = AtariClipRewardWrapper(env)
    if render:
        env = RenderWrapper(env)
    return AtariInfoClearWrapper(env)


def make_atari_env(env_id, render=False, device=None):
    """a2c_acktr.py:175-213: gym.make(env_id) wrapped with the Atari chain."""
    try:
        import gym
    except ImportError as e:  # not in this image; ALE emulation is out of scope
        raise ImportError('make_atari_env needs gym with the Atari (ALE) environments') from e
    return wrap_atari_env(gym.make(env_id), render=render, device=device)
