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


class EpisodeInfoWrapper(object):
    """Only the static helper of the reference class is needed by a training loop."""

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
    """

    def __init__(self, num_envs, num_actions=4, seed=0, env_offset=0, device=None):
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
        self.state = _lib.EnvState(self._episode.data_ptr(), self._step.data_ptr(), self._length.data_ptr(),
                                   self._total.data_ptr(), self._done.data_ptr())
        self._obs = torch.zeros((N, 84, 84, 4), dtype=torch.uint8, device=self.device)

    def _stream(self):
        return _lib.stream_handle(self.device)

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
                               self._done[n0:].data_ptr())
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
