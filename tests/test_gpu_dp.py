"""Data-parallel ACKTR on the GPU (SURVEY.md §8e "Checks"): two ranks, each stepping
its shard of the envs through the full HIP path (rollout, update, K-FAC), against one
process stepping all envs.

The ranks rehearse the multi-GPU path on one card: ``torch.distributed`` with the
gloo backend over CUDA tensors (RCCL refuses two ranks on one device; the code path
above the collective -- the split [grads | losses | A stats] / [G stats] all-reduce,
the 1/world scales, the row-keyed RNG -- is the one RCCL runs at N > 1).

* rollout: bit-identical -- env ids are global (env_offset) and the sampler and the
  sampled-loss RNG are keyed by the global row, so a shard draws what the full batch
  draws;
* update (gs = 40: EMA + damped inverses + K-FAC step): factors, loss scalars and the
  parameter step agree with the full batch within fp32 reduction-order tolerance
  (the shards' sums are added by the collective instead of inside one kernel).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
N_TOTAL, T, WORLD = 8, 5, 2


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _iteration(n_envs, rank, gae=None, norm=False):
    """One bench-shaped ACKTR iteration at gs = 40 (steady state, inverse step);
    gae / norm: the objective options beyond the reference (GAE(lambda), globally
    normalised advantages)."""
    from actorcritic import session as sess
    from actorcritic.agents import MultiEnvAgent
    from actorcritic.envs.atari.model import AtariModel
    from actorcritic.envs.atari.wrappers import SyntheticAtariEnvs
    from actorcritic.examples.atari.a2c_acktr import create_optimizer
    from actorcritic.multi_env import MultiEnv
    from actorcritic.nn import linear_decay
    from actorcritic.objectives import A2CObjective
    dev = torch.device('cuda', torch.cuda.current_device())
    sess.reset_default_graph()
    env = MultiEnv(SyntheticAtariEnvs(n_envs, num_actions=4, seed=1234, env_offset=rank * n_envs, device=dev))
    model = AtariModel(env.observation_space, env.action_space, 32, random_seed=7, device=dev)
    agent = MultiEnvAgent(env, model, T)
    obj = A2CObjective(model, discount_factor=0.99, entropy_regularization_strength=0.01, gae_lambda=gae,
                       normalize_advantages=norm)
    gs = sess.get_or_create_global_step()
    opt = create_optimizer(True, model, linear_decay(0.25, 0.025, gs, 1e7 / (N_TOTAL * T)))
    op = obj.optimize_shared(opt, baseline_loss_weight=0.5, global_step=gs)
    gs.assign(40)
    before = model.params.clone()
    with sess.Session(dev) as s:
        obs, act, rew, term, nxt, _ = agent.interact(s)
        rollout = [x.clone() for x in (obs, act, rew, term, nxt)]
        out = s.run([obj.policy_loss, obj.baseline_loss, obj.mean_entropy, obj.advantage, op], feed_dict={
            model.observations_placeholder: obs, model.bootstrap_observations_placeholder: nxt,
            model.actions_placeholder: act, model.rewards_placeholder: rew, model.terminals_placeholder: term})
    torch.cuda.synchronize()
    assert opt.last_flags == (False, True, True)
    return dict(rollout=[x.cpu() for x in rollout], losses=torch.tensor(out[:3], dtype=torch.float64),
                adv=torch.as_tensor(np.asarray(out[3])).reshape(-1).cpu(),
                step=(model.params - before).cpu(), factors=opt.state['factors'].cpu(), inv=opt.state['inv'].cpu(),
                params=model.params.cpu())


def _worker(rank, port, out_dir, gae=None, norm=False):
    import sys
    sys.path.insert(0, os.path.join(ROOT, 'actor-critic_amd'))
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank), ACMI_DIST_BACKEND='gloo')
    from actorcritic import parallel
    world, r = parallel.init_from_env()
    assert (world, r) == (WORLD, rank)
    res = _iteration(N_TOTAL // WORLD, rank, gae, norm)
    torch.save(res, os.path.join(out_dir, 'rank{}.pt'.format(rank)))
    parallel.barrier()
    parallel.destroy()


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize('gae,norm', [(None, False), (0.95, True)])
def test_sharded_acktr_iteration_matches_full_batch(lib, cuda, tmp_path, gae, norm):
    """(None, False) is the reference objective; (0.95, True) adds GAE and the
    advantage normalisation, whose batch moments are summed over the ranks: each
    shard's advantages are its slice of the full batch's normalised advantages."""
    ctx = mp.get_context('spawn')
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, str(tmp_path), gae, norm)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
        assert p.exitcode == 0, 'rank failed with exit code {}'.format(p.exitcode)
    shards = [torch.load(str(tmp_path / 'rank{}.pt'.format(r)), weights_only=True) for r in range(WORLD)]
    full = _iteration(N_TOTAL, 0, gae, norm)

    # rollout: every shard is its slice of the full batch, bit for bit
    n = N_TOTAL // WORLD
    for r, sh in enumerate(shards):
        for i, (a, b) in enumerate(zip(sh['rollout'], full['rollout'])):
            assert torch.equal(a, b[r * n:(r + 1) * n]), ('rollout tensor', i, 'rank', r)
        # advantages (normalised with the global moments when norm)
        m = n * T
        np.testing.assert_allclose(sh['adv'].numpy(), full['adv'][r * m:(r + 1) * m].numpy(), rtol=0, atol=2e-5)
    # replicated state: bit-identical on every rank
    for key in ('params', 'factors', 'inv', 'step'):
        assert torch.equal(shards[0][key], shards[1][key]), key
    # the loss scalars fetched with the update are the global means
    np.testing.assert_allclose(shards[0]['losses'].numpy(), full['losses'].numpy(), rtol=2e-5, atol=1e-7)
    # factors (first EMA update = the reduced batch statistics) and damped inverses
    assert _rel(shards[0]['factors'], full['factors']) < 2e-5
    assert _rel(shards[0]['inv'], full['inv']) < 1e-3
    # the K-FAC parameter step (north_star tolerance for preconditioned updates)
    step_s, step_f = shards[0]['step'].double(), full['step'].double()
    assert step_f.norm() > 0
    assert ((step_s - step_f).norm() / step_f.norm()).item() < 1e-3


def test_bench_self_launches_ranks():
    """`python bench.py --gpus 2` without torchrun's environment spawns the two ranks
    itself (the parent stays off the GPU) and rank 0 prints one JSON line for the
    whole job (n_gpus 2, dp2, global envs = 2 shards).  gloo on one card here; the
    same launcher runs nccl (RCCL) ranks on a multi-GPU node."""
    import json
    import subprocess
    import sys
    env = dict(os.environ, ACMI_DIST_BACKEND='gloo')
    env.pop('WORLD_SIZE', None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--steps', '2', '--warmup', '1',
                        '--envs-per-gpu', '16', '--no-cpu-baseline'], env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out['n_gpus'] == 2 and out['config']['parallelism'] == 'dp2'
    assert out['config']['global_envs'] == 32 and out['config']['envs_per_gpu'] == 16
    assert out['value'] > 0 and out['cpu_baseline'] is None
    # the communication leg is separated from compute: the compute stream's stall on
    # the per-update all-reduce (ms, max over ranks) and the bytes summed per update
    # (grads + 4 loss scalars + packed A and G statistics, ACKTR C3 = 32: 10.8 MB)
    assert out['dist_backend'] == 'gloo'
    assert out['allreduce_updates_timed'] == 2
    assert out['allreduce_ms'] > 0 and out['allreduce_ms'] < out['ms_per_step']
    assert 10.0e6 < out['allreduce_bytes'] < 11.5e6, out['allreduce_bytes']
