"""Agents (reference: actorcritic/agents.py:6-257).

``MultiEnvAgent.interact`` returns the reference's 6-tuple in batch-major [env, step]
layout.  With a batched device env and an :class:`AtariModel` it runs the whole
T-step rollout on the GPU: per step one strided tower forward that writes its
activations straight into the update's [N*T] buffers (row n*T + t), one sampling
kernel, one stepper kernel that writes the next stacked frame into the [N, T+1]
observation buffer — no host copies, no Python lists.  Anything else takes the
reference's list-based loop.
"""

from abc import ABCMeta, abstractmethod

import torch

from actorcritic import _lib
from actorcritic._engine import OBS_BYTES


class Agent(object, metaclass=ABCMeta):
    @abstractmethod
    def interact(self, session):
        pass


class SingleEnvAgent(Agent):
    """One env, multiple steps; list-based (agents.py:50-131)."""

    def __init__(self, env, model, num_steps):
        self._env = env
        self._model = model
        self._num_steps = num_steps
        self._observation = None

    def interact(self, session):
        observation_steps, action_steps, reward_steps, terminal_steps, info_steps = [], [], [], [], []
        next_observation = self._observation
        if next_observation is None:
            next_observation = self._env.reset()
        for _ in range(self._num_steps):
            observation_steps.append(next_observation)
            action = self._model.sample_actions([[next_observation]], session)[0]
            next_observation, reward, terminal, info = self._env.step(action)
            action_steps.append(action)
            reward_steps.append(reward)
            terminal_steps.append(terminal)
            info_steps.append(info)
        self._observation = next_observation
        return ([observation_steps], [action_steps], [reward_steps], [terminal_steps], [next_observation],
                [info_steps])


class _RolloutBuffers(object):
    def __init__(self, engine, N, T):
        dev = engine.device
        self.N, self.T = N, T
        self.obs = torch.zeros((N, T, 84, 84, 4), dtype=torch.uint8, device=dev)
        self.next_obs = torch.zeros((N, 84, 84, 4), dtype=torch.uint8, device=dev)
        self.actions_tn = torch.zeros((T, N), dtype=torch.int32, device=dev)
        self.actions = torch.zeros((N, T), dtype=torch.int32, device=dev)
        self.rewards = torch.zeros((N, T), dtype=torch.float32, device=dev)
        self.terminals = torch.zeros((N, T), dtype=torch.uint8, device=dev)
        self.episode_rewards = torch.zeros((N, T), dtype=torch.float32, device=dev)
        self.acts = engine.activations(N * T, 'rollout')
        self.bad_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self.bad_event = None


class MultiEnvAgent(Agent):
    """Multiple envs (MultiEnv), multiple steps (agents.py:134-228)."""

    def __init__(self, multi_env, model, num_steps):
        self._env = multi_env
        self._model = model
        self._num_steps = num_steps
        self._observations = None
        self._bufs = None

    def _fast(self):
        return getattr(self._env, 'batched', None) is not None and hasattr(self._model, 'engine')

    def interact(self, session):
        if self._fast():
            return self._interact_device()
        return self._interact_lists(session)

    # -- reference semantics (host lists) ---------------------------------------
    def _interact_lists(self, session):
        observation_steps, action_steps, reward_steps, terminal_steps, info_steps = [], [], [], [], []
        next_observations = self._observations
        if next_observations is None:
            next_observations = self._env.reset()
        for _ in range(self._num_steps):
            observation_steps.append(next_observations)
            batch_next_observations = transpose_list([next_observations])
            actions = self._model.sample_actions(batch_next_observations, session)
            next_observations, rewards, terminals, infos = self._env.step(actions)
            action_steps.append(actions)
            reward_steps.append(rewards)
            terminal_steps.append(terminals)
            info_steps.append(infos)
        self._observations = next_observations
        return (transpose_list(observation_steps), transpose_list(action_steps), transpose_list(reward_steps),
                transpose_list(terminal_steps), next_observations, transpose_list(info_steps))

    # -- device rollout ------------------------------------------------------------
    def _interact_device(self):
        from actorcritic.envs.atari.model import ForwardOut
        from actorcritic.envs.atari.wrappers import EpisodeInfoBatch
        eng = self._model.engine
        env = self._env.batched
        N, T = env.num_envs, self._num_steps
        if self._bufs is None or self._bufs.N != N or self._bufs.T != T:
            self._bufs = _RolloutBuffers(eng, N, T)
        rb = self._bufs
        if rb.bad_event is not None:  # deferred NaN-logit check of the previous rollout
            rb.bad_event.synchronize()
            if int(rb.bad_host[0]) > 0:
                eng.check_bad_rows()
        if self._observations is None:
            env.reset_into(rb.next_obs.data_ptr())
        rb.obs[:, 0].copy_(rb.next_obs)
        stream = eng.stream()
        A = eng.A
        obs0 = rb.obs.data_ptr()
        rew0, term0, ep0 = rb.rewards.data_ptr(), rb.terminals.data_ptr(), rb.episode_rewards.data_ptr()
        seed = (self._model._random_seed or 0) & 0xFFFFFFFF
        for t in range(T):
            src = obs0 + t * OBS_BYTES
            eng.forward(src, N, rb.acts.view(t, T), want_value=True, img_stride=T * OBS_BYTES, act_stride=T)
            act_t = rb.actions_tn[t]
            _lib.call('acmi_sample_actions', _lib.c_vp(rb.acts.logits.data_ptr() + 4 * t * A), T * A, N, A, seed,
                      eng.rank, eng.sample_counter, None, 0, _lib.c_vp(act_t.data_ptr()),
                      _lib.c_vp(eng._bad_rows.data_ptr()), stream)
            eng.sample_counter += 1
            if t + 1 < T:
                dst, dstride = obs0 + (t + 1) * OBS_BYTES, T * OBS_BYTES
            else:
                dst, dstride = rb.next_obs.data_ptr(), OBS_BYTES
            env.step_into(act_t.data_ptr(), src, T * OBS_BYTES, dst, dstride, rew0 + 4 * t, term0 + t, ep0 + 4 * t, T)
        rb.actions.copy_(rb.actions_tn.t())
        rb.bad_host.copy_(eng._bad_rows, non_blocking=True)
        rb.bad_event = torch.cuda.Event()
        rb.bad_event.record()
        fwd = ForwardOut(eng, rb.acts, N, T, rb.obs.view(N * T, 84, 84, 4))
        eng.register_rollout(rb.obs, fwd)
        self._observations = rb.next_obs
        return (rb.obs, rb.actions, rb.rewards, rb.terminals.view(torch.bool), rb.next_obs,
                EpisodeInfoBatch(rb.episode_rewards))


def transpose_list(values):
    """Transposes a list of lists (agents.py:231-257): [[1,2],[3,4]] -> [[1,3],[2,4]]."""
    return [list(row) for row in zip(*values)]
