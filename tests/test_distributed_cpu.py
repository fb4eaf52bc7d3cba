"""world_size-2 gloo tests of the data-parallel host logic (CPU, no GPU):
actorcritic.parallel's reduction of the [grads | losses | factor stats] buffer gives
every rank the full-batch mean of the oracle's shard statistics, bit-identical across
ranks, and rank-disjoint env shards step the same synthetic games."""
import os
import socket
import sys

import numpy as np
import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    sys.path.insert(0, os.path.join(ROOT, 'actor-critic_amd'))
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import oracle
    from actorcritic import parallel
    parallel.init_from_env(backend='gloo')
    assert parallel.world_size() == world and parallel.rank() == rank
    A, C3 = 4, 32
    params = oracle.init_params(A, C3, 0)
    rng = np.random.default_rng(5)
    obs = rng.integers(0, 256, (2 * world, 84, 84, 4), dtype=np.uint8)
    M = obs.shape[0]
    dl_full = rng.standard_normal((M, A)) / M
    dv_full = rng.standard_normal(M) / M
    mine = slice(2 * rank, 2 * rank + 2)
    acts = oracle.forward(params, obs[mine], A, C3)
    # per-rank: gradients of the local mean loss scaled by 1/world (the loss kernel's
    # grad_scale) and the local factor statistics
    g, _, af = oracle.backward(params, acts, dl_full[mine] * world / world, dv_full[mine] * world / world, A, C3,
                               with_a_factors=True)
    stats = np.concatenate([f.ravel() for f in af])
    # loss slots as acmi_a2c_loss writes them: this rank's means scaled by 1/world
    # (grad_scale), so the SUM all-reduce leaves the global means
    act_full = rng.integers(0, A, M)
    tg_full = rng.standard_normal(M)
    full_pre = oracle.forward(params, obs, A, C3)
    mine_l = oracle.a2c_loss_and_head_grads(full_pre['logits'][mine], full_pre['value'][mine], act_full[mine],
                                            tg_full[mine])
    full_l = oracle.a2c_loss_and_head_grads(full_pre['logits'], full_pre['value'], act_full, tg_full)
    names = ('policy_loss', 'baseline_loss', 'mean_entropy')
    loss_slots = [mine_l[k] / world for k in names] + [0.0]
    red = torch.from_numpy(np.concatenate([g, loss_slots, stats]))
    # the split path of a K-FAC update (engine.allreduce_begin/_end): the prefix
    # [grads | losses | A stats] asynchronously, the G tail synchronously, then wait
    red2 = red.clone()
    split = g.size + 4 + stats.size // 2
    pending = parallel.allreduce_sum_async(red2[:split])
    parallel.allreduce_sum_(red2[split:])
    pending.wait()
    parallel.allreduce_sum_(red)
    assert torch.equal(red, red2)
    n = g.size
    grads = red[:n].numpy()
    stats_mean = red[n + 4:].numpy() / world
    # full-batch references
    full = oracle.forward(params, obs, A, C3)
    g_full, _, af_full = oracle.backward(params, full, dl_full, dv_full, A, C3, with_a_factors=True)
    np.testing.assert_allclose(grads, g_full, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(stats_mean, np.concatenate([f.ravel() for f in af_full]), rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(red[n:n + 3].numpy(), [full_l[k] for k in names], rtol=1e-12)
    # every rank holds bit-identical reduced buffers
    digest = torch.tensor([float(np.frombuffer(red.numpy().tobytes(), np.uint8).astype(np.int64).sum())],
                          dtype=torch.float64)
    ref = digest.clone()
    parallel.broadcast_(ref, 0)
    assert ref.item() == digest.item()
    assert parallel.max_over_ranks(rank) == world - 1
    # env shards: rank r owns global env ids r*N .. r*N+N-1
    envs = [oracle.SyntheticAtari(11, rank * 2 + i) for i in range(2)]
    frames = np.stack([e.reset() for e in envs])
    np.save(os.path.join(out_dir, 'frames{}.npy'.format(rank)), frames)
    parallel.barrier()
    parallel.destroy()


def test_dp_reduction_gloo_world2(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle
    f0 = np.load(tmp_path / 'frames0.npy')
    f1 = np.load(tmp_path / 'frames1.npy')
    single = np.stack([oracle.SyntheticAtari(11, e).reset() for e in range(4)])
    np.testing.assert_array_equal(np.concatenate([f0, f1]), single)
