"""CPU baseline for bench.py — test/measurement infrastructure, never the product path.

A float32 numpy run of the oracle's restatement of the reference's ACKTR iteration with
the reference's structure (a2c_acktr.py:104-137): a T-step rollout that per step runs
the tower on the N current observations (model.py:149-151), samples, and steps N
synthetic Atari envs with the reference wrapper semantics; then one update: forward on
the N*T batch, n-step targets, A2C losses and head gradients, backward fused with the
K-FAC A factors, the sampled-loss backward for the G factors, EMA, natural-gradient
step; the damped inverses (every 10 updates in the reference schedule) are timed once
and amortised at 1/10 per update.  Threads: whatever OpenBLAS uses (reported).

The reference itself (TensorFlow 1.x + kfac + gym) cannot run here or on the GPU box,
so this port is the baseline (kind "port").
"""

import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import oracle  # noqa: E402


def blas_threads():
    try:
        from threadpoolctl import threadpool_info
        n = [i.get('num_threads') for i in threadpool_info() if i.get('user_api') == 'blas']
        if n:
            return int(n[0])
    except Exception:
        pass
    for var in ('OPENBLAS_NUM_THREADS', 'OMP_NUM_THREADS'):
        if os.environ.get(var):
            return int(os.environ[var])
    return os.cpu_count() or 1


def run(n_envs=32, n_steps=20, iters=3, A=4, C3=32, seed=0, time_budget_s=30.0):
    f32 = np.float32
    params = oracle.init_params(A, C3, seed).astype(f32)
    din, dout = oracle.kfac_dims(A, C3)
    envs = [oracle.SyntheticAtari(seed, e) for e in range(n_envs)]
    obs = np.stack([e.reset() for e in envs])
    factors_A = [np.zeros((d, d), f32) for d in din[:5]]
    factors_G = [np.zeros((d, d), f32) for d in dout]
    inverses = [(np.eye(din[l], dtype=f32), np.eye(dout[l], dtype=f32)) for l in range(6)]
    velocity = np.zeros_like(params)
    gp_gamma = 0.99
    rollout_s = update_s = 0.0
    done_iters = 0
    t_start = time.perf_counter()
    for it in range(iters):
        t0 = time.perf_counter()
        ob_steps = np.zeros((n_envs, n_steps, 84, 84, 4), np.uint8)
        actions = np.zeros((n_envs, n_steps), np.int64)
        rewards = np.zeros((n_envs, n_steps), f32)
        terms = np.zeros((n_envs, n_steps), bool)
        for t in range(n_steps):
            ob_steps[:, t] = obs
            fw = oracle.forward(params, obs, A, C3, dtype=f32)
            u = oracle.sample_uniforms(seed, 0, it * n_steps + t, n_envs)
            a = oracle.sample_f32(fw['logits'], u)
            actions[:, t] = a
            nxt = []
            for n, env in enumerate(envs):
                o, r, d, _ = env.step(a[n])
                nxt.append(o)
                rewards[n, t], terms[n, t] = r, d
            obs = np.stack(nxt)
        t1 = time.perf_counter()
        M = n_envs * n_steps
        fw = oracle.forward(params, ob_steps.reshape(M, 84, 84, 4), A, C3, dtype=f32)
        vb = oracle.forward(params, obs, A, C3, dtype=f32)['value']
        tg = oracle.targets_f64(rewards, terms, vb, gp_gamma).astype(f32).reshape(-1)
        lg = oracle.a2c_loss_and_head_grads(fw['logits'], fw['value'], actions.reshape(-1), tg)
        grads, _, afac = oracle.backward(params, fw, lg['dlogits'].astype(f32), lg['dvalue'].astype(f32), A, C3,
                                         dtype=f32, with_a_factors=True)
        g_pi, g_v, _ = oracle.sampled_head_grads(fw['logits'], 0x4b464143, 0, it)
        gfac = oracle.g_factors(params, fw, g_pi.astype(f32), g_v.astype(f32), A, C3, dtype=f32)
        decay = f32(0.99)
        factors_A = [decay * F + (1 - decay) * S.astype(f32) for F, S in zip(factors_A, afac)]
        factors_G = [decay * F + (1 - decay) * S.astype(f32) for F, S in zip(factors_G, gfac)]
        params, velocity, _, _ = oracle.kfac_step(params, velocity, grads, inverses, 0.25, 0.9, 1e-4, A, C3)
        params, velocity = params.astype(f32), velocity.astype(f32)
        t2 = time.perf_counter()
        rollout_s += t1 - t0
        update_s += t2 - t1
        done_iters += 1
        if time.perf_counter() - t_start > time_budget_s:
            break
    # damped inverses, timed once, amortised over invert_every = 10 updates
    t3 = time.perf_counter()
    inverses = [(Ai.astype(f32), Gi.astype(f32)) for Ai, Gi in
                oracle.damped_inverses([F.astype(np.float64) for F in factors_A],
                                       [F.astype(np.float64) for F in factors_G], 0.01)]
    inv_s = time.perf_counter() - t3
    per_iter = (rollout_s + update_s) / done_iters + inv_s / 10.0
    steps = n_envs * n_steps
    return dict(env_steps_per_s=steps / per_iter, update_ms=1e3 * (update_s / done_iters + inv_s / 10.0),
                rollout_ms=1e3 * rollout_s / done_iters, inverse_ms=1e3 * inv_s, iters=done_iters,
                threads=blas_threads(), n_envs=n_envs, n_steps=n_steps)


if __name__ == '__main__':
    print(run(iters=int(sys.argv[1]) if len(sys.argv) > 1 else 2))
