"""The RCCL branch of the data-parallel update, executed on one GPU.

The 8-GPU scaling run is the driver's; on the one-GPU box the ``nccl`` backend
(= RCCL on ROCm) cannot host two ranks on one device, so the multi-rank tests use
gloo.  This test runs the engine's real exchange -- the packed
[grads | losses | A stats] prefix summed asynchronously on RCCL's stream while the
sampled-loss chain computes, the packed G tail, the unpack -- through an ``nccl``
process group of ONE rank (test-only switch ACMI_FORCE_COLLECTIVE=1), and checks
that a SUM over one rank leaves the update unchanged and that the bytes on the
wire are the 10.8 MB per update that DESIGN.md §7 states.
Reference: /root/reference/actorcritic/examples/atari/a2c_acktr.py:247 (the
reference itself is single-device).
"""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
N, T = 8, 5


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _iteration():
    """One ACKTR iteration at gs = 40 (EMA + damped inverses + K-FAC step)."""
    from actorcritic import session as sess
    from actorcritic.agents import MultiEnvAgent
    from actorcritic.envs.atari.model import AtariModel
    from actorcritic.envs.atari.wrappers import SyntheticAtariEnvs
    from actorcritic.examples.atari.a2c_acktr import create_optimizer
    from actorcritic.multi_env import MultiEnv
    from actorcritic.nn import linear_decay
    from actorcritic.objectives import A2CObjective
    dev = torch.device('cuda', 0)
    sess.reset_default_graph()
    env = MultiEnv(SyntheticAtariEnvs(N, num_actions=4, seed=99, device=dev))
    model = AtariModel(env.observation_space, env.action_space, 32, random_seed=11, device=dev)
    agent = MultiEnvAgent(env, model, T)
    obj = A2CObjective(model, discount_factor=0.99, entropy_regularization_strength=0.01)
    gs = sess.get_or_create_global_step()
    opt = create_optimizer(True, model, linear_decay(0.25, 0.025, gs, 1e6))
    op = obj.optimize_shared(opt, baseline_loss_weight=0.5, global_step=gs)
    gs.assign(40)
    eng = model.engine
    eng.comm_timing(True)
    before = model.params.clone()
    with sess.Session(dev) as s:
        obs, act, rew, term, nxt, _ = agent.interact(s)
        losses = s.run([obj.policy_loss, obj.baseline_loss, obj.mean_entropy, op], feed_dict={
            model.observations_placeholder: obs, model.bootstrap_observations_placeholder: nxt,
            model.actions_placeholder: act, model.rewards_placeholder: rew, model.terminals_placeholder: term})
    torch.cuda.synchronize()
    assert opt.last_flags == (False, True, True)
    ms, nbytes, nupd = eng.comm_collect()
    return dict(collective=eng.collective, losses=torch.tensor(losses[:3], dtype=torch.float64),
                step=(model.params - before).cpu(), factors=opt.state['factors'].cpu(), inv=opt.state['inv'].cpu(),
                params=model.params.cpu(), comm_bytes=nbytes, comm_updates=nupd)


def _worker(port, out_dir):
    sys.path.insert(0, os.path.join(ROOT, 'actor-critic_amd'))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    plain = _iteration()
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK='0', WORLD_SIZE='1',
                      LOCAL_RANK='0', ACMI_FORCE_COLLECTIVE='1')
    dist.init_process_group('nccl', init_method='env://', rank=0, world_size=1)
    assert dist.get_backend() == 'nccl'
    rccl = _iteration()
    dist.destroy_process_group()
    torch.save({'plain': plain, 'rccl': rccl}, os.path.join(out_dir, 'rccl.pt'))


def test_rccl_exchange_at_world_size_one_is_identity(lib, cuda, tmp_path):
    ctx = mp.get_context('spawn')
    p = ctx.Process(target=_worker, args=(_free_port(), str(tmp_path)))
    p.start()
    p.join(240)
    assert p.exitcode == 0, 'worker failed with exit code {}'.format(p.exitcode)
    r = torch.load(str(tmp_path / 'rccl.pt'), weights_only=True)
    plain, rccl = r['plain'], r['rccl']
    assert not plain['collective'] and rccl['collective']
    # the exchange ran once per update through RCCL with the packed buffer
    assert plain['comm_updates'] == 0
    assert rccl['comm_updates'] == 1
    assert 10.0e6 < rccl['comm_bytes'] < 11.5e6, rccl['comm_bytes']
    # a sum over one rank changes nothing: loss scalars, factors, inverses, the step
    for key in ('losses', 'factors', 'inv', 'step', 'params'):
        assert torch.equal(plain[key], rccl[key]), key
