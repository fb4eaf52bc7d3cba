"""Kernel paths that only engage at larger batches, and full-size properties.

The GEMM launches pick tiles, split-K chunkings and fused reductions by batch size
(net.hip: 128-row conv1 / 64x64 conv2 tiles and split-K fc4 below 2048 images,
256-row tiles above; plan_rounds chunk counts; the i8 conv1 A factor's chunks;
the heads kernel's NZ-way slab reduce; the narrow Gram kernel).  These tests run
each regime against float64 PyTorch references, and check at the BASELINE.json
workload size (512 envs x 20 steps) the size-independent properties the domain
offers: bit-identical replays (no atomics anywhere in the update) and symmetric A
factors with a non-negative diagonal and a homogeneous corner of 1.
"""
import ctypes

import numpy as np
import pytest
import torch

from actorcritic import _lib
from test_gpu_kernels import _layout, _net, alloc_acts, rand_params, torch_forward

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('B', [700, 2100, 4200])
def test_forward_batch_regimes_match_torch(lib, cuda, B):
    """700: split-K fc4 (nz slabs reduced by the heads kernel) + rollout tiles;
    2100: 256-row conv1 tiles with split fc4; 4200: no split (fc4 fills the chip)."""
    A, C3 = 4, 32
    params = rand_params(A, C3, cuda, seed=11)
    g = torch.Generator().manual_seed(12)
    obs = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.uint8)
    t, acts = alloc_acts(B, A, C3, cuda)
    ws = torch.zeros(max(1, lib.acmi_forward_ws_floats(B)), device=cuda)
    acts.ws = ws.data_ptr()
    acts.ws_floats = ws.numel()
    net = _net(params, A, C3)
    obs_d = obs.to(cuda)
    _lib.call('acmi_forward', ctypes.byref(net), _lib.ptr(obs_d), 84 * 84 * 4, B, ctypes.byref(acts), 1,
              _lib.stream_handle())
    torch.cuda.synchronize()
    ref = torch_forward(params, obs, A, C3)
    for name, r in zip(['a1', 'a2', 'a3', 'a4', 'logits', 'value'], ref):
        got = t[name].cpu().double().reshape(r.shape)
        rel = (got - r).abs().max().item() / max(1e-6, r.abs().max().item())
        assert rel < 1e-5, (B, name, rel)


@pytest.mark.parametrize('mode', [_lib.GEMM_X3, _lib.GEMM_F32])
def test_backward_multichunk_matches_torch(lib, cuda, mode):
    """B = 96 images: conv1 has 38400 rows (3 i8 A-factor chunks), every split-K
    reduction runs several chunks, the narrow Gram kernel several blocks.  Both
    arithmetic modes of the wgrad + A-factor reductions (bf16x3 split operands,
    f32 MFMA) hold the same float64 tolerance."""
    prev = lib.acmi_get_gemm_mode()
    _lib.call('acmi_set_gemm_mode', mode)
    try:
        _backward_multichunk(lib, cuda)
    finally:
        _lib.call('acmi_set_gemm_mode', prev)


def _backward_multichunk(lib, cuda):
    A, C3, B = 6, 32, 96
    params = rand_params(A, C3, cuda, seed=13)
    g = torch.Generator().manual_seed(14)
    obs = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.uint8)
    t, acts = alloc_acts(B, A, C3, cuda)
    net = _net(params, A, C3)
    obs_d = obs.to(cuda)
    _lib.call('acmi_forward', ctypes.byref(net), _lib.ptr(obs_d), 84 * 84 * 4, B, ctypes.byref(acts), 1,
              _lib.stream_handle())
    ldh = 8
    dhead = torch.zeros(B, ldh)
    dhead[:, :A + 1] = torch.randn(B, A + 1, generator=g)
    dhead_d = dhead.to(cuda)
    z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=cuda)
    d = dict(d1=z(B, 20, 20, 32), d2=z(B, 9, 9, 64), d3=z(B, 7, 7, C3), d4=z(B, 512))
    bwd = _lib.Bwd(d['d1'].data_ptr(), d['d2'].data_ptr(), d['d3'].data_ptr(), d['d4'].data_ptr(),
                   dhead_d.data_ptr(), ldh)
    off, n = _layout(A, C3)
    grads = z(n)
    din = (ctypes.c_int64 * 6)()
    dout = (ctypes.c_int64 * 6)()
    so = (ctypes.c_int64 * 11)()
    tot = ctypes.c_int64()
    _lib.call('acmi_kfac_layout', A, C3, din, dout, so, ctypes.byref(tot))
    astat = z(tot.value)
    ws = z(lib.acmi_backward_ws_floats(B, A, C3))
    _lib.call('acmi_backward', ctypes.byref(net), _lib.ptr(obs_d), 84 * 84 * 4, B, ctypes.byref(acts),
              ctypes.byref(bwd), _lib.ptr(grads), _lib.ptr(astat), _lib.ptr(ws), ws.numel(), _lib.stream_handle())
    # G statistics of a fixed output gradient through the same chain
    torch.cuda.synchronize()
    p64 = params.cpu().double().requires_grad_(True)
    a1, a2, a3f, a4, logits, value = torch_forward(p64, obs, A, C3)
    loss = (logits * dhead[:, :A].double()).sum() + (value * dhead[:, A].double()).sum()
    loss.backward()
    got = grads.cpu().double()
    ends = off[1:] + [n]
    for i, (o, e) in enumerate(zip(off, ends)):
        r = p64.grad[o:e]
        rel = (got[o:e] - r).abs().max().item() / max(1e-12, r.abs().max().item())
        assert rel < 2e-5, ('param block', i, rel)
    x = obs.double() / 255.0

    def patches(x, k, s):
        p = x.unfold(1, k, s).unfold(2, k, s)
        return p.permute(0, 1, 2, 4, 5, 3).reshape(-1, k * k * x.shape[-1])

    ins = [patches(x, 8, 4), patches(a1.detach(), 4, 2), patches(a2.detach(), 3, 1), a3f.detach(), a4.detach()]
    a_host = astat.cpu().double()
    for f, xin in enumerate(ins):
        xb = torch.cat([xin, torch.ones(xin.shape[0], 1, dtype=xin.dtype)], 1)
        r = xb.t() @ xb / xb.shape[0]
        got_f = a_host[so[f]:so[f] + din[f] * din[f]].reshape(din[f], din[f])
        rel = (got_f - r).abs().max().item() / r.abs().max().item()
        assert rel < 2e-5, ('A factor', f, rel)
    # pre-activation gradients of fc4 and conv3 (d4, d3: inputs of the G statistics);
    # d2 and d1 are exercised through the conv2 / conv1 weight gradients above
    p = params.cpu().double().requires_grad_(True)
    _, _, a3f, a4, logits, value = torch_forward(p, obs, A, C3)
    loss = (logits * dhead[:, :A].double()).sum() + (value * dhead[:, A].double()).sum()
    g4, g3 = torch.autograd.grad(loss, [a4, a3f])
    for name, gg, act in (('d4', g4, a4), ('d3', g3, a3f)):
        ref = (gg * (act > 0)).detach()
        got = d[name].cpu().double().reshape(ref.shape)
        rel = (got - ref).abs().max().item() / ref.abs().max().item()
        assert rel < 2e-5, (name, rel)


def _bench_like(N=512, T=20, seed=1234):
    from actorcritic import session as sess
    from actorcritic.agents import MultiEnvAgent
    from actorcritic.envs.atari.model import AtariModel
    from actorcritic.envs.atari.wrappers import SyntheticAtariEnvs
    from actorcritic.examples.atari.a2c_acktr import create_optimizer
    from actorcritic.multi_env import MultiEnv
    from actorcritic.nn import linear_decay
    from actorcritic.objectives import A2CObjective
    sess.reset_default_graph()
    env = MultiEnv(SyntheticAtariEnvs(N, num_actions=4, seed=seed, device=torch.device('cuda')))
    model = AtariModel(env.observation_space, env.action_space, 32, random_seed=7, device=torch.device('cuda'))
    agent = MultiEnvAgent(env, model, T)
    obj = A2CObjective(model, discount_factor=0.99, entropy_regularization_strength=0.01)
    gs = sess.get_or_create_global_step()
    opt = create_optimizer(True, model, linear_decay(0.25, 0.025, gs, 10000000 / (N * T)))
    op = obj.optimize_shared(opt, baseline_loss_weight=0.5, global_step=gs)
    gs.assign(39)  # the second update below runs the inverse (gs = 40)
    return env, model, agent, obj, gs, opt, op


def _run_two_updates(iters=2):
    from actorcritic import session as sess
    env, model, agent, obj, gs, opt, op = _bench_like()
    with sess.Session() as s:
        for _ in range(iters):
            obs, act, rew, term, nxt, _ = agent.interact(s)
            s.run(op, feed_dict={model.observations_placeholder: obs, model.bootstrap_observations_placeholder: nxt,
                                 model.actions_placeholder: act, model.rewards_placeholder: rew,
                                 model.terminals_placeholder: term}, host=False)
    torch.cuda.synchronize()
    return (model.params.clone(), opt.state['factors'].clone(), opt.state['inv'].clone(),
            opt.state['velocity'].clone(), model.engine.layout)


def test_rollout_variants_give_identical_updates(lib, cuda, monkeypatch):
    """Three rollout + ACKTR update iterations at 512 envs x 20 steps give bit-identical
    parameters, factors, inverses and velocities whichever rollout runs: one chain,
    the two env halves on two streams, and either replayed from a
    captured hipGraph.  The rollouts after an update read the conv tower's weights
    re-prepared from the updated parameters: prepared on the parent stream before the
    halves fork, and inside the captured graph so that every replay re-prepares."""
    outs = []
    for split, graph in (('0', '0'), ('1', '0'), ('1', '1'), ('0', '1')):
        monkeypatch.setenv('ACMI_ROLLOUT_SPLIT', split)
        monkeypatch.setenv('ACMI_ROLLOUT_GRAPH', graph)
        outs.append(_run_two_updates(iters=3)[:4])
    for k, other in enumerate(outs[1:], 1):
        for i, (a, b) in enumerate(zip(outs[0], other)):
            assert torch.equal(a, b), (k, i)


def test_full_size_updates_are_bit_identical_and_factors_well_formed(lib, cuda):
    """BASELINE.json workload (512 envs x 20 steps): two ACKTR updates (the second
    with an inverse) replayed from the same seeds give bit-identical parameters,
    factors, inverses and velocities; every A factor is symmetric with a
    non-negative diagonal and a homogeneous corner of 1 (to the EMA's f32 rounding)."""
    p1, f1, i1, v1, L = _run_two_updates()
    p2, f2, i2, v2, _ = _run_two_updates()
    assert torch.equal(p1, p2) and torch.equal(f1, f2) and torch.equal(i1, i2) and torch.equal(v1, v2)
    fac = f1.cpu().double()
    for f in range(5):
        d = L.din[f]
        m = fac[L.stat_off[f]:L.stat_off[f] + d * d].reshape(d, d)
        assert torch.equal(m, m.t()), f
        assert (torch.diagonal(m) >= 0).all(), f
        # every batch statistic has an exact 1 in the homogeneous corner; the
        # zero-debiased f32 EMA of two of them is 1 to within its rounding
        assert abs(m[d - 1, d - 1].item() - 1.0) < 1e-5, (f, m[d - 1, d - 1].item())
    assert torch.isfinite(p1).all()


def test_two_stream_rollout_is_bit_identical(lib, cuda, monkeypatch):
    """512 envs: the fused rollout step (acmi_rollout_step: tower + one
    heads/sample/env-step kernel), the rollout's two env halves on two HIP streams
    (agents.py _rollout_halves), eagerly and replayed from a captured hipGraph
    (_rollout_graph: rollout 1 eager, 2 captured + replayed, 3 replayed), give
    exactly the three-launch single-chain rollout: observations, actions, rewards, terminals,
    episode rewards, next observations and every activation row, three rollouts
    in a row (the later ones start mid-episode from auto-reset states)."""
    from actorcritic import session as sess
    outs = []
    # (split, graph, fused tail, step fusion: step t's tail runs step t+1's tower)
    for split, graph, fused, fsteps in (('0', '0', '0', '0'), ('0', '0', '1', '0'), ('0', '0', '1', '1'),
                                        ('1', '0', '0', '0'), ('1', '0', '1', '1'), ('1', '1', '1', '1'),
                                        ('0', '1', '1', '1')):
        monkeypatch.setenv('ACMI_ROLLOUT_SPLIT', split)
        monkeypatch.setenv('ACMI_ROLLOUT_GRAPH', graph)
        monkeypatch.setenv('ACMI_ROLLOUT_FUSED', fused)
        monkeypatch.setenv('ACMI_ROLLOUT_FUSE_STEPS', fsteps)
        env, model, agent, obj, gs, opt, op = _bench_like()
        got = []
        with sess.Session() as s:
            for _ in range(3):
                obs, act, rew, term, nxt, info = agent.interact(s)
                acts = agent._bufs.acts
                got += [x.clone() for x in (obs, act, rew, term, nxt, info.episode_rewards, acts.a1, acts.a2,
                                            acts.a3, acts.a4, acts.m1, acts.m2, acts.m3, acts.logits, acts.value)]
        torch.cuda.synchronize()
        assert agent._bufs.halves == (split == '1')
        assert (agent._bufs.graph is not None) == (graph == '1')
        assert agent._bufs.fuse_steps == (fused == '1' and fsteps == '1')  # (x3 gemm mode: the default)
        outs.append(got)
    for other in outs[1:]:
        for i, (a, b) in enumerate(zip(outs[0], other)):
            if a.is_floating_point():  # episode rewards are NaN where no episode ended
                assert torch.equal(torch.isnan(a), torch.isnan(b)), i
                a, b = torch.nan_to_num(a, nan=0.0), torch.nan_to_num(b, nan=0.0)
            assert torch.equal(a, b), i


def test_split_rollout_step_bit_identical_across_terminals(lib, cuda, monkeypatch):
    """32 envs (B <= 64: the split rollout step, each image's tower over 7
    workgroups, the post-step env states parked in the forward workspace and
    committed by the next step's fc4 launch): the fused steps, eagerly and
    replayed from a captured hipGraph, give exactly the three-launch chain over
    eight rollouts of 20 steps -- long enough that episodes end inside rollouts
    and across rollout boundaries (auto-reset of a terminal env, episode totals
    at terminals, the last unfused step's commit followed by the next rollout's
    step 0).  Reference: agents.py:202-216, multi_env.py auto-reset."""
    from actorcritic import session as sess
    outs = []
    for graph, fused, fsteps in (('0', '0', '0'), ('0', '1', '1'), ('1', '1', '1')):
        monkeypatch.setenv('ACMI_ROLLOUT_SPLIT', '0')
        monkeypatch.setenv('ACMI_ROLLOUT_GRAPH', graph)
        monkeypatch.setenv('ACMI_ROLLOUT_FUSED', fused)
        monkeypatch.setenv('ACMI_ROLLOUT_FUSE_STEPS', fsteps)
        env, model, agent, obj, gs, opt, op = _bench_like(N=32, T=20, seed=77)
        got, terms = [], []
        with sess.Session() as s:
            for _ in range(8):
                obs, act, rew, term, nxt, info = agent.interact(s)
                acts = agent._bufs.acts
                got += [x.clone() for x in (obs, act, rew, term, nxt, info.episode_rewards, acts.a1, acts.a2,
                                            acts.a3, acts.m1, acts.logits, acts.value)]
                terms.append(term.clone())
        torch.cuda.synchronize()
        assert agent._bufs.fuse_steps == (fused == '1' and fsteps == '1')
        assert (agent._bufs.graph is not None) == (graph == '1')
        term_all = torch.stack(terms).cpu()  # [rollout, env, step]
        assert term_all.any(), 'no episode ended: the terminal / auto-reset path went untested'
        # some env ends an episode on a rollout's last step (its reset is committed
        # by the unfused last step and read by the next rollout's step 0)
        assert term_all[:-1, :, -1].any() or term_all[1:, :, 0].any()
        outs.append(got)
    for other in outs[1:]:
        for i, (a, b) in enumerate(zip(outs[0], other)):
            if a.is_floating_point():  # episode rewards are NaN where no episode ended
                assert torch.equal(torch.isnan(a), torch.isnan(b)), i
                a, b = torch.nan_to_num(a, nan=0.0), torch.nan_to_num(b, nan=0.0)
            assert torch.equal(a, b), i


def test_concurrent_g_stats_bit_identical(lib, cuda, monkeypatch):
    """The sampled-loss backward (G statistics) on a side stream concurrently with the
    loss backward (NetEngine.backward_and_stats) gives bit-identical parameters,
    factors, inverses and velocities to running the two chains one after the other."""
    from actorcritic._engine import NetEngine
    monkeypatch.setattr(NetEngine, 'concurrent_stats', False)
    serial = _run_two_updates()
    # (one stream, the two chains' conv2 input gradients as one launch or two)
    monkeypatch.setattr(NetEngine, 'stacked_dx', not NetEngine.stacked_dx)
    other = _run_two_updates()
    monkeypatch.setattr(NetEngine, 'stacked_dx', not NetEngine.stacked_dx)
    for i, (a, b) in enumerate(zip(serial[:4], other[:4])):
        assert torch.equal(a, b), ('stacked', i)
    monkeypatch.setattr(NetEngine, 'concurrent_stats', True)
    # side chain started with the backward, and at its dX event (acmi_stream_wait_backward_dx)
    for after_dx in (False, True):
        monkeypatch.setattr(NetEngine, 'stats_after_dx', after_dx)
        conc = _run_two_updates()
        for i, (a, b) in enumerate(zip(serial[:4], conc[:4])):
            assert torch.equal(a, b), (after_dx, i)
