"""CPU baseline for bench.py -- test/measurement infrastructure, never the product path.

The reference (TensorFlow 1.x + kfac + gym, a2c_acktr.py) cannot run here or on the
GPU box, so the baseline is a restatement with the reference's process structure and
arithmetic placement (kind "port"):

* environments: one synthetic Atari game per env producing 84x84x1 u8 frames (the
  same counter-hash frames, rewards and episode lengths as the device stepper and
  oracle.SyntheticAtari) inside ``EpisodeInfoWrapper`` semantics; with ``ipc`` each
  game runs in its own child process behind the reference's ``SubprocessEnv`` Pipe
  protocol (actorcritic.multi_env, the restatement of multi_env.py:140-362), the
  4-frame stack is kept in the parent (FrameStackWrapper, a2c_acktr.py:170-171) and
  ``MultiEnv`` fans the steps out over a ThreadPoolExecutor(N) with the lazy
  auto-reset (multi_env.py:18-89); without ``ipc`` (large N: one process per env is
  not practical at 512 envs) the same wrapped games step in-process on the pool;
* rollout: T serial batch-N forwards + categorical draws (agents.py:202-216,
  model.py:149-151);
* update (a2c_acktr.py:117-126): forward over the N*T batch and the bootstrap
  observations, the n-step targets of objectives.py:178-214, the A2C losses
  (objectives.py:123-154), the backward; ACKTR: the K-FAC A factors (patch Grams),
  the sampled-loss backward for the G factors, the EMA, the damped inverses every 10
  updates (timed once, amortised 1/10), the preconditioned trust-region momentum
  step (DESIGN.md section 4 conventions); A2C: global-norm clip 0.5 + RMSProp;
* arithmetic: torch on the CPU in float32 (oneDNN convolutions, BLAS GEMMs) on every
  core this process may use (torch.set_num_threads).
"""

import functools
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import oracle  # noqa: E402

_ROOT = os.path.dirname(HERE)
_PKG = os.path.join(_ROOT, 'actor-critic_amd')
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)


def cpu_threads():
    """Cores this process may use (the GPU box's CPU share), capped by OMP_NUM_THREADS."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    if os.environ.get('OMP_NUM_THREADS', '').isdigit():
        n = min(n, int(os.environ['OMP_NUM_THREADS']))
    return max(1, n)


class _Discrete(object):
    def __init__(self, n):
        self.n = n


class _Box(object):
    def __init__(self, shape):
        self.low = np.zeros(shape, np.uint8)
        self.high = np.full(shape, 255, np.uint8)
        self.shape = shape
        self.dtype = np.dtype(np.uint8)


class SyntheticRawAtari(object):
    """One synthetic game, raw 84x84x1 frames, with EpisodeInfoWrapper's episode total
    in info (wrappers.py:263-294).  Frames/rewards/lengths: oracle.SyntheticAtari's."""

    def __init__(self, seed, env_id, num_actions, game=None):
        self.seed, self.e, self.game = seed, env_id, game
        self.salt, _, _, self.rew_lo, self.rew_hi, self.n_legal = oracle.game_params(game)
        self.k, self.t, self.total = -1, 0, 0.0
        self.L = 0
        self.action_space = _Discrete(num_actions)
        self.observation_space = _Box((84, 84, 1))

    def reset(self):
        self.k += 1
        self.t, self.total = 0, 0.0
        self.L = oracle.episode_length(self.seed, self.e, self.k, self.game)
        return oracle.reset_frame(self.seed, self.e, self.k, self.game)[..., None]

    def step(self, action):
        self.t += 1
        a = int(action) & 255
        a = a if a < self.n_legal else 0
        base = int(oracle.key4(self.seed ^ self.salt, self.e, self.k, self.t * 256 + a))
        rh = int(oracle.mix32(np.uint32(base) ^ oracle.REW_SALT)) >> 8
        r = -1.0 if rh < self.rew_lo else (1.0 if rh >= self.rew_hi else 0.0)
        term = self.t >= self.L
        self.total += r
        info = {}
        if term:
            info['episode'] = {'total_reward': self.total}
            self.total = 0.0
        return oracle._frame(base)[..., None], r, term, info

    def close(self):
        pass


def make_raw_env(seed, env_id, num_actions, game=None):
    return SyntheticRawAtari(seed, env_id, num_actions, game)


def make_envs(n_envs, num_actions, seed, ipc, games=None):
    from actorcritic.envs.atari.wrappers import FrameStackWrapper
    from actorcritic.multi_env import MultiEnv, create_subprocess_envs
    game = (lambda e: e % 57) if games == 'atari57' else (lambda e: None)
    fns = [functools.partial(make_raw_env, seed, e, num_actions, game(e)) for e in range(n_envs)]
    raw = create_subprocess_envs(fns) if ipc else [fn() for fn in fns]
    return MultiEnv([FrameStackWrapper(env, 4) for env in raw])


class TorchNet(object):
    """The Nature CNN of envs/atari/model.py:173-217 in torch fp32 on the CPU, on the
    flat parameter layout of the GPU engine (HWIO convs, [in, out] FCs)."""

    def __init__(self, params, A, C3):
        import torch
        self.torch = torch
        self.A, self.C3 = A, C3
        off, n = oracle.param_offsets(A, C3)
        shapes = [s for pair in oracle.layer_shapes(A, C3) for s in pair]
        ends = list(off[1:]) + [n]
        flat = torch.from_numpy(np.asarray(params, np.float32).copy())
        self.blocks = [flat[o:e].reshape(s).clone().requires_grad_(True) for o, e, s in zip(off, ends, shapes)]

    def forward(self, obs, grad):
        torch = self.torch
        F = torch.nn.functional
        w1, b1, w2, b2, w3, b3, w4, b4, wp, bp, wv, bv = self.blocks
        with torch.set_grad_enabled(grad):
            x = torch.from_numpy(np.ascontiguousarray(obs)).permute(0, 3, 1, 2).float() / 255.0
            z1 = F.conv2d(x, w1.permute(3, 2, 0, 1), b1, stride=4)
            a1 = torch.relu(z1)
            z2 = F.conv2d(a1, w2.permute(3, 2, 0, 1), b2, stride=2)
            a2 = torch.relu(z2)
            z3 = F.conv2d(a2, w3.permute(3, 2, 0, 1), b3, stride=1)
            a3 = torch.relu(z3)
            a3f = a3.permute(0, 2, 3, 1).reshape(a3.shape[0], -1)  # NHWC flatten (model.py:197-206)
            z4 = a3f @ w4 + b4
            a4 = torch.relu(z4)
            logits = a4 @ wp + bp
            value = (a4 @ wv + bv)[:, 0]
        return dict(x=x, z1=z1, a1=a1, z2=z2, a2=a2, z3=z3, a3=a3, a3f=a3f, z4=z4, a4=a4, logits=logits,
                    value=value)

    def a_factors(self, fw):
        """[x;1]^T[x;1] / rows per layer; conv rows = every location, columns (kh, kw, c)."""
        torch = self.torch
        nhwc = lambda t: t.permute(0, 2, 3, 1)

        def patches(x, k, s):
            p = x.unfold(1, k, s).unfold(2, k, s)
            return p.permute(0, 1, 2, 4, 5, 3).reshape(-1, k * k * x.shape[-1])

        ins = [patches(nhwc(fw['x']), 8, 4), patches(nhwc(fw['a1']), 4, 2), patches(nhwc(fw['a2']), 3, 1),
               fw['a3f'], fw['a4']]
        out = []
        for xin in ins:
            xin = xin.detach()
            xb = torch.cat([xin, torch.ones(xin.shape[0], 1)], 1)
            out.append(xb.t() @ xb / xb.shape[0])
        return out


def _sample(torch, logits, gen):
    p = torch.softmax(logits, -1)
    return torch.multinomial(p, 1, generator=gen)[:, 0]


def run(n_envs=32, n_steps=20, iters=3, A=4, C3=32, algo='acktr', seed=0, time_budget_s=20.0, ipc=None,
        threads=None, games=None, min_iters=3):
    """Times warm-up + up to `iters` iterations; after `min_iters` timed iterations it
    stops once ~time_budget_s have passed.  Returns env-steps/s, the update / rollout
    split and every timed iteration's seconds (the spread of the sample)."""
    import torch
    threads = threads or cpu_threads()
    torch.set_num_threads(threads)
    if ipc is None:
        ipc = n_envs <= 64
    acktr = algo == 'acktr'
    gen = torch.Generator().manual_seed(seed)
    net = TorchNet(oracle.init_params(A, C3, seed), A, C3)
    W = net.blocks
    din, dout = oracle.kfac_dims(A, C3)
    fac_A = [torch.zeros(d, d) for d in din[:5]]
    fac_G = [torch.zeros(d, d) for d in dout]
    inverses = [(torch.eye(din[l]), torch.eye(dout[l])) for l in range(6)]
    vel = [torch.zeros_like(w) for w in W]
    ms = [torch.ones_like(w) for w in W]
    gamma, beta, lr_acktr, lr_a2c = 0.99, 0.01, 0.25, 7e-4
    env = make_envs(n_envs, A, seed, ipc, games)
    obs = np.stack(env.reset())
    stats = dict(rollout=0.0, update=0.0, n=0, iter_s=[], env=0.0)
    inv_s = 0.0
    t_start = time.perf_counter()
    try:
        for it in range(iters + 1):  # iteration 0: warm-up (oneDNN primitives, pools)
            t0 = time.perf_counter()
            ob_steps = np.zeros((n_envs, n_steps, 84, 84, 4), np.uint8)
            actions = np.zeros((n_envs, n_steps), np.int64)
            rewards = np.zeros((n_envs, n_steps), np.float32)
            terms = np.zeros((n_envs, n_steps), bool)
            for t in range(n_steps):
                ob_steps[:, t] = obs
                a = _sample(torch, net.forward(obs, False)['logits'], gen).numpy()
                te = time.perf_counter()
                nxt, r, d, _ = env.step(a.tolist())
                obs = np.stack(nxt)
                if it > 0:
                    stats['env'] += time.perf_counter() - te
                actions[:, t], rewards[:, t], terms[:, t] = a, r, d
            t1 = time.perf_counter()
            M = n_envs * n_steps
            fw = net.forward(ob_steps.reshape(M, 84, 84, 4), True)
            vb = net.forward(obs, False)['value'].numpy()
            tg = torch.from_numpy(oracle.targets_f64(rewards, terms, vb, gamma).astype(np.float32).reshape(-1))
            logits, value = fw['logits'], fw['value']
            logp_all = torch.log_softmax(logits, -1)
            logp = logp_all.gather(1, torch.from_numpy(actions.reshape(-1, 1)))[:, 0]
            ent = -(logp_all.exp() * logp_all).sum(-1)
            adv = tg - value.detach()
            l_pi = -((adv * logp).mean() + beta * ent.mean())
            l_v = ((tg - value) ** 2 / 2).mean()
            grads = torch.autograd.grad(l_pi + 0.5 * l_v, W, retain_graph=acktr)
            with torch.no_grad():
                if acktr:
                    # K-FAC statistics: A from the layer inputs, G from the sampled losses
                    ys = _sample(torch, logits.detach(), gen)
                    yv = value.detach() + torch.randn(M, generator=gen)
                    with torch.enable_grad():
                        ls = -torch.log_softmax(logits, -1).gather(1, ys[:, None]).sum() + \
                            ((yv - value) ** 2 / 2).sum()
                        gz = torch.autograd.grad(ls, [fw['z1'], fw['z2'], fw['z3'], fw['z4'], logits, value])
                    gs = [g.permute(0, 2, 3, 1).reshape(-1, g.shape[1]) for g in gz[:3]] + [gz[3], gz[4],
                                                                                             gz[5][:, None]]
                    stat_A = net.a_factors(fw)
                    stat_G = [g.t() @ g / g.shape[0] for g in gs]
                    fac_A = [0.99 * F_ + 0.01 * S for F_, S in zip(fac_A, stat_A)]
                    fac_G = [0.99 * F_ + 0.01 * S for F_, S in zip(fac_G, stat_G)]
                    pre = []
                    for l in range(6):
                        gb = torch.cat([grads[2 * l].reshape(din[l] - 1, dout[l]), grads[2 * l + 1].reshape(1, -1)])
                        Ai, Gi = inverses[l]
                        pre.append(Ai @ gb @ Gi)
                    sq = sum(float((torch.cat([grads[2 * l].reshape(din[l] - 1, dout[l]),
                                               grads[2 * l + 1].reshape(1, -1)]) * pre[l]).sum()) for l in range(6))
                    coeff = min(1.0, (1e-4 / (sq * lr_acktr * lr_acktr)) ** 0.5) if sq > 0 else 1.0
                    for l in range(6):
                        for j, part in ((2 * l, pre[l][:-1].reshape(W[2 * l].shape)),
                                        (2 * l + 1, pre[l][-1].reshape(W[2 * l + 1].shape))):
                            vel[j].mul_(0.9).add_(part, alpha=coeff)
                            W[j].sub_(lr_acktr * vel[j])
                else:
                    norm = float(torch.sqrt(sum((g * g).sum() for g in grads)))
                    scale = 0.5 / max(norm, 0.5)
                    for w, g, m in zip(W, grads, ms):
                        g = g * scale
                        m.mul_(0.9).addcmul_(g, g, value=0.1)
                        w.sub_(lr_a2c * g / torch.sqrt(m + 1e-10))
            t2 = time.perf_counter()
            if it > 0:
                stats['rollout'] += t1 - t0
                stats['update'] += t2 - t1
                stats['n'] += 1
                stats['iter_s'].append(t2 - t0)
                if stats['n'] >= min_iters and time.perf_counter() - t_start > time_budget_s:
                    break
        if acktr:  # the damped inverses (every 10 updates), timed once, amortised
            t3 = time.perf_counter()
            with torch.no_grad():
                for l in range(6):
                    A_, G_ = fac_A[min(l, 4)], fac_G[l]
                    pi = float(torch.sqrt((torch.trace(A_) / A_.shape[0]) / (torch.trace(G_) / G_.shape[0]).clamp_min(
                        1e-30)))
                    inverses[l] = (torch.linalg.inv(A_ + pi * 0.1 * torch.eye(A_.shape[0])),
                                   torch.linalg.inv(G_ + 0.1 / pi * torch.eye(G_.shape[0])))
            inv_s = time.perf_counter() - t3
    finally:
        env.close()
    n = max(1, stats['n'])
    per_iter = (stats['rollout'] + stats['update']) / n + inv_s / 10.0
    return dict(env_steps_per_s=n_envs * n_steps / per_iter, update_ms=1e3 * (stats['update'] / n + inv_s / 10.0),
                rollout_ms=1e3 * stats['rollout'] / n, inverse_ms=1e3 * inv_s, iters=stats['n'], threads=threads,
                n_envs=n_envs, n_steps=n_steps, ipc=ipc, algo=algo, iter_s=stats['iter_s'],
                structure=('{} SubprocessEnv children (Pipe protocol) + ThreadPoolExecutor({})'.format(n_envs, n_envs)
                           if ipc else '{} in-process envs on a ThreadPoolExecutor({}) (one SubprocessEnv child per env '
                           'is used up to 64 envs; {} children plus the {}-thread pool would approach the GPU box\'s '
                           'limit on processes per call; in-process env stepping was {:.1f}% of the timed '
                           'iterations, so the Pipe round trips the reference pays are NOT in this number)'.format(
                               n_envs, n_envs, n_envs, n_envs, 100.0 * stats['env'] / max(1e-9, sum(stats['iter_s'])))),
                env_step_frac=stats['env'] / max(1e-9, sum(stats['iter_s'])))


if __name__ == '__main__':
    import json
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    algo = sys.argv[2] if len(sys.argv) > 2 else 'acktr'
    print(json.dumps(run(n_envs=n, n_steps=20 if algo == 'acktr' else 5, C3=32 if algo == 'acktr' else 64,
                         algo=algo, iters=3)))
