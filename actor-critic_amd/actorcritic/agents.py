"""Agents (reference: actorcritic/agents.py:6-257).

``MultiEnvAgent.interact`` returns the reference's 6-tuple in batch-major [env, step]
layout.  With a batched device env and an :class:`AtariModel` it runs the whole
T-step rollout on the GPU: per step one strided tower forward that writes its
activations straight into the update's [N*T] buffers (row n*T + t), one sampling
kernel, one stepper kernel that writes the next stacked frame into the [N, T+1]
observation buffer — no host copies, no Python lists.  Anything else takes the
reference's list-based loop.

Two opt-in variants, bit-identical to the one-chain rollout (test_two_stream_rollout_
is_bit_identical, and across updates test_rollout_variants_give_identical_updates):
ACMI_ROLLOUT_SPLIT=1 runs the two env halves as two chains on two HIP streams (the
sampler keys its RNG by the global row, acmi_sample_actions_at, the stepper by the global
env id); ACMI_ROLLOUT_GRAPH=1 captures the rollout once as a hipGraph and replays it (the
RNG counter read from device memory, acmi_sample_actions_dev).  Neither is faster on one
MI355X (same lease, two rounds each: 512 x 20 2.68 vs 2.69-2.70 M env-steps/s split on /
off; 1024 x 20 bf16 2.72-2.75 M both): the per-step kernels are GPU-bound and the host
keeps up.  They are kept for hosts where launch overhead is not hidden.  (An earlier
+6 % for the split came from a race, since fixed: half 1 read the conv tower's prepared
weights while half 0's step 0 was re-making them after an update.)
"""

import ctypes
import os
import time

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
        # two-chain rollout: env halves on the current stream and a side stream,
        # each with its own forward workspace (fc4 split-K slabs)
        self.halves = (os.environ.get('ACMI_ROLLOUT_SPLIT', '0') == '1' and N >= 256 and N % 2 == 0)
        self.side = torch.cuda.Stream(device=dev) if self.halves else None
        need = int(_lib.load().acmi_forward_ws_floats(N // 2 if self.halves else N))
        self.ws = [torch.zeros(max(need, 1), dtype=torch.float32, device=dev) for _ in range(2)]
        self.use_graph = os.environ.get('ACMI_ROLLOUT_GRAPH', '0') == '1'
        self.fused = os.environ.get('ACMI_ROLLOUT_FUSED', '1') != '0'
        # step fusion: step t's tail also runs step t+1's conv tower (needs the
        # fused tower: x3 gemm mode, checked once per rollout, and prepared weights)
        self.fuse_steps = self.fused and os.environ.get('ACMI_ROLLOUT_FUSE_STEPS', '1') != '0'
        self.graph, self.graph_key, self.warm = None, None, False
        self.ctr_dev = torch.zeros(1, dtype=torch.int32, device=dev)


class MultiEnvAgent(Agent):
    """Multiple envs (MultiEnv), multiple steps (agents.py:134-228)."""

    def __init__(self, multi_env, model, num_steps, copy_batches=False):
        self._env = multi_env
        self._model = model
        self._num_steps = num_steps
        self._observations = None
        self._bufs = None
        self._copy = bool(copy_batches)

    def _fast(self):
        return getattr(self._env, 'batched', None) is not None and hasattr(self._model, 'engine')

    def interact(self, session):
        """One T-step rollout -> (observations [N,T,...], actions [N,T], rewards [N,T],
        terminals [N,T], next_observations [N,...], infos) (agents.py:157-228).

        Device rollout aliasing: the returned tensors are the agent's persistent
        rollout buffers and the NEXT interact() overwrites them in place (the
        reference returns fresh lists every call).  A caller that keeps a batch
        across calls (logging, replay, comparing rollouts) clones it, or constructs
        the agent with ``copy_batches=True`` to receive fresh tensors every call."""
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
    def _rollout_halves(self, eng, env, rb, N, T, A, seed, dev_ctr=False):
        """The T-step rollout as one chain (rb.halves False) or as the two env halves'
        chains on the current stream and rb.side."""
        main = torch.cuda.current_stream(eng.device)
        if not rb.fused:  # (the fused step 0 reads next_obs in place and files it into obs[:, 0])
            rb.obs[:, 0].copy_(rb.next_obs)
        # the tower's prepared weights are re-made on the first use after an update:
        # here, on this stream ahead of the fork (half 1 on rb.side would otherwise
        # read them before half 0's step 0 re-made them); always when capturing a
        # graph, so that every replay re-prepares from the updated parameters
        eng.net(force_prepare=dev_ctr)
        if rb.halves:
            rb.side.wait_stream(main)
        N2 = N // 2 if rb.halves else N
        # step fusion is decided once per rollout: a gemm mode switched mid-rollout must
        # not let step t skip a tower that step t-1's tail never ran
        fuse = bool(rb.fused and rb.fuse_steps and eng.lib.acmi_get_gemm_mode() == _lib.GEMM_X3)
        for t in range(T):
            _half_step(eng, env, rb, 0, N2, T, A, t, seed, dev_ctr, fuse)
            if rb.halves:
                with torch.cuda.stream(rb.side):
                    _half_step(eng, env, rb, 1, N2, T, A, t, seed, dev_ctr, fuse)
            if not dev_ctr:
                eng.sample_counter += 1
        if rb.halves:
            main.wait_stream(rb.side)
        if not rb.fused:  # (the fused tail writes actions [N, T] itself)
            rb.actions.copy_(rb.actions_tn.t())

    def _rollout_graph(self, eng, env, rb, N, T, A, seed):
        """The two-chain rollout as one hipGraph (torch.cuda.CUDAGraph over the
        libacmi launches): captured on the second rollout with these buffers, then
        replayed -- ~280 launches per rollout stop costing host time.  Everything
        that differs between rollouts lives in device memory (observations, env
        states, parameters updated in place); the RNG counter is refreshed in
        rb.ctr_dev before each replay."""
        # everything the captured launches bake in: buffers, env, seed, rank, and the
        # arithmetic modes / step fusion that chose the captured kernels
        lib = eng.lib
        key = (eng.params.data_ptr(), id(env), seed, eng.rank, int(lib.acmi_get_gemm_mode()),
               int(lib.acmi_get_forward_mode()), bool(rb.fuse_steps))
        if rb.graph is None or rb.graph_key != key:
            if not rb.warm:  # first rollout eager: loads the code objects, sizes workspaces
                rb.warm = True
                self._rollout_halves(eng, env, rb, N, T, A, seed)
                return
            rb.ctr_dev.fill_(eng.sample_counter & 0xFFFFFFFF)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._rollout_halves(eng, env, rb, N, T, A, seed, dev_ctr=True)
            rb.graph, rb.graph_key = g, key
        else:
            rb.ctr_dev.fill_(eng.sample_counter & 0xFFFFFFFF)
        rb.graph.replay()
        eng.sample_counter += T

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
            t_wait = time.perf_counter()
            rb.bad_event.synchronize()
            self.last_sync_wait = time.perf_counter() - t_wait  # (bench.py's host-time split)
            if int(rb.bad_host[0]) > 0:
                eng.check_bad_rows()
        if self._observations is None:
            env.reset_into(rb.next_obs.data_ptr())
        stream = eng.stream()
        A = eng.A
        obs0 = rb.obs.data_ptr()
        rew0, term0, ep0 = rb.rewards.data_ptr(), rb.terminals.data_ptr(), rb.episode_rewards.data_ptr()
        seed = (self._model._random_seed or 0) & 0xFFFFFFFF
        if rb.use_graph:
            self._rollout_graph(eng, env, rb, N, T, A, seed)
        elif rb.halves or rb.fused:
            self._rollout_halves(eng, env, rb, N, T, A, seed)
        else:
            rb.obs[:, 0].copy_(rb.next_obs)
            for t in range(T):
                src = obs0 + t * OBS_BYTES
                eng.forward(src, N, rb.acts.view(t, T), want_value=True, img_stride=T * OBS_BYTES, act_stride=T)
                act_t = rb.actions_tn[t]
                _lib.call('acmi_sample_actions_at', _lib.c_vp(rb.acts.logits.data_ptr() + 4 * t * A), T * A, N,
                          A, seed, 0, eng.sample_counter, eng.rank * N, None, 0, _lib.c_vp(act_t.data_ptr()),
                          _lib.c_vp(eng._bad_rows.data_ptr()), stream)
                eng.sample_counter += 1
                if t + 1 < T:
                    dst, dstride = obs0 + (t + 1) * OBS_BYTES, T * OBS_BYTES
                else:
                    dst, dstride = rb.next_obs.data_ptr(), OBS_BYTES
                env.step_into(act_t.data_ptr(), src, T * OBS_BYTES, dst, dstride, rew0 + 4 * t, term0 + t,
                              ep0 + 4 * t, T)
            rb.actions.copy_(rb.actions_tn.t())
        rb.bad_host.copy_(eng._bad_rows, non_blocking=True)
        rb.bad_event = torch.cuda.Event()
        rb.bad_event.record()
        self._observations = rb.next_obs
        out = (rb.obs, rb.actions, rb.rewards, rb.terminals.view(torch.bool), rb.next_obs, rb.episode_rewards)
        if self._copy:
            out = tuple(x.clone() for x in out)
        obs = out[0]
        # the update re-uses the rollout activations for exactly these observations
        fwd = ForwardOut(eng, rb.acts, N, T, obs.view(N * T, 84, 84, 4))
        eng.register_rollout(obs, fwd)
        return out[:5] + (EpisodeInfoBatch(out[5]),)


def _half_step(eng, env, rb, h, N2, T, A, t, seed, dev_ctr=False, fuse=False):
    """Rollout step t of env half h (envs h*N2 .. h*N2+N2-1) on the current stream.
    dev_ctr: the sampler's RNG counter is rb.ctr_dev + t (graph capture) instead of
    the host eng.sample_counter.  fuse: step fusion for the whole rollout (decided
    once by the caller, so tower_done at step t means step t-1 passed next_acts)."""
    n0 = h * N2
    row = n0 * T + t
    obs0 = rb.obs.data_ptr()
    src = obs0 + row * OBS_BYTES
    acts = rb.acts.view(row, T, ws_rows=N2)
    acts.ws = rb.ws[h].data_ptr()
    acts.ws_floats = rb.ws[h].numel()
    act_t = rb.actions_tn[t].data_ptr() + 4 * n0
    # the sampler's RNG is keyed by the global env row (stream 0): env shards over
    # ranks draw exactly what one process stepping all envs would
    row0 = eng.rank * rb.N + n0
    if dev_ctr:
        ctr_dev, ctr = _lib.c_vp(rb.ctr_dev.data_ptr()), t
    else:
        ctr_dev, ctr = None, eng.sample_counter & 0xFFFFFFFF
    if t + 1 < T:
        dst, dstride = src + OBS_BYTES, T * OBS_BYTES
    else:
        dst, dstride = rb.next_obs.data_ptr() + n0 * OBS_BYTES, OBS_BYTES
    rew, term, ep = rb.rewards.data_ptr() + 4 * row, rb.terminals.data_ptr() + row, \
        rb.episode_rewards.data_ptr() + 4 * row
    if rb.fused:  # tower + fused heads/sample/env-step tail (acmi_rollout_step)
        # step fusion: step t's tower ran in step t-1's tail; step t's tail runs
        # step t+1's tower (not the last step's: the bootstrap forward is the update's)
        nxt = rb.acts.view(row + 1, T, ws_rows=N2) if fuse and t + 1 < T else None
        # step 0 reads the previous rollout's final stacks (next_obs) in place and
        # copies them into obs[:, 0] (the batch's step-0 rows) as it goes
        src_t, sstride = (rb.next_obs.data_ptr() + n0 * OBS_BYTES, OBS_BYTES) if t == 0 else (src, T * OBS_BYTES)
        # actions straight into the [N, T] batch (element b at [b*T], like the rewards)
        act_nt = rb.actions.data_ptr() + 4 * row
        io = _lib.RolloutIO(seed, 0, ctr, ctr_dev, row0, act_nt, eng._bad_rows.data_ptr(), env.range_state(n0),
                            env.env_offset + n0, env.seed, dst, dstride, rew, term, ep, T,
                            1 if fuse and t > 0 else 0, ctypes.addressof(nxt) if nxt is not None else None, T,
                            src if t == 0 else None)
        _lib.call('acmi_rollout_step', ctypes.byref(eng.net()), ctypes.c_void_p(src_t), sstride, N2,
                  ctypes.byref(acts), T, ctypes.byref(io), eng.stream())
        return
    eng.forward(src, N2, acts, want_value=True, img_stride=T * OBS_BYTES, act_stride=T)
    _lib.call('acmi_sample_actions_dev', _lib.c_vp(rb.acts.logits.data_ptr() + 4 * row * A), T * A, N2, A,
              seed, 0, ctr_dev, ctr, row0, None, 0, _lib.c_vp(act_t),
              _lib.c_vp(eng._bad_rows.data_ptr()), eng.stream())
    env.step_range_into(n0, N2, act_t, src, T * OBS_BYTES, dst, dstride, rew, term, ep, T)


def transpose_list(values):
    """Transposes a list of lists (agents.py:231-257): [[1,2],[3,4]] -> [[1,3],[2,4]]."""
    return [list(row) for row in zip(*values)]
