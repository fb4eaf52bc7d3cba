"""ACKTR (or A2C) env-steps/s on synthetic Breakout 84x84x4 — the BASELINE.json metric.

One step = one full training iteration of the reference loop (a2c_acktr.py:104-137):
``agent.interact`` (T-step device rollout: tower forward, sampling, batched stepper)
+ ``session.run(optimize_op)`` (targets, losses, backward fused with the K-FAC
A statistics, sampled-loss backward for the G statistics, RCCL all-reduce when
N > 1, EMA, the damped inverses every 10th update, the preconditioned trust-region
momentum step).  The global step starts after the 30-update cold start (the timed
iterations are steady-state K-FAC iterations, inverse included at its natural 1/10
rate).  Weak scaling: every GPU runs --envs-per-gpu envs (default 512 = the 8x512
shard of BASELINE.json configs[3]).

  python bench.py --gpus N --steps K --warmup W
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Without torchrun's environment, ``--gpus N > 1`` launches the N ranks itself: the
parent never touches the GPU, it spawns N fresh interpreters (one per GPU, RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_* set as torchrun would), each pins its device and
joins the process group (nccl = RCCL; ACMI_DIST_BACKEND=gloo rehearses N ranks on one
GPU), and rank 0 prints the one JSON line.
"""

import argparse
import ctypes
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, 'actor-critic_amd'), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense f32-input MFMA peak
BF16_MFMA_PEAK_TFLOPS = 2516.6  # dense bf16 MFMA: 256 CUs x 4 SIMDs x 1024 FLOP/clk x 2.4 GHz
# bf16x3 split operands: six bf16 MFMAs per f32-accurate product tile, so the
# f32-equivalent ceiling of that arithmetic is the bf16 peak / 6
X3_F32EQ_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 6
# f16x2 split operands (f16x2.hpp): three f16 MFMAs (f16 dense peak = bf16's)
F16X2_F32EQ_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 3
HBM_PEAK_GBS = 8000.0
PMC_PACKAGE = 'r06_final'  # profiles/<this>/: the current measurement package


def measured_traffic(kernel, workload):
    """HBM bytes per launch of the roofline kernel from the committed PMC summary
    of the current measurement package (PMC_PACKAGE; else any other
    profiles/*/pmc_traffic.json: rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, separate
    passes) when it was measured on this kernel and workload; else None."""
    import glob
    first = os.path.join(ROOT, 'profiles', PMC_PACKAGE, 'pmc_traffic.json')
    rest = sorted(glob.glob(os.path.join(ROOT, 'profiles', '*', 'pmc_traffic.json')), reverse=True)
    for path in [first] + [p for p in rest if p != first]:
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get('kernel') == kernel and d.get('workload') == workload:
            return d.get('hbm_bytes_per_launch')
    return None


INT8_MFMA_PEAK_TOPS = 2 * BF16_MFMA_PEAK_TFLOPS  # v_mfma_i32_32x32x32_i8: twice the bf16 rate
U8F16X2_F32EQ_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 2  # u8 pixels exact: two f16 MFMAs per product
FP64_MFMA_PEAK_TFLOPS = 78.6  # v_mfma_f64_16x16x4f64, dense


def iteration_ceiling(N, T, A, C3, acktr, band_tiles=None, forward='f32'):
    """The build's algorithmic work per training iteration (DESIGN.md section 3,
    per-kernel accounting), each kernel's work priced at the ceiling of the
    arithmetic it runs: the time the iteration would take if every kernel ran at
    its roofline.  band_tiles: (conv2, conv3) needed 64x64 sub-tiles of the band
    reductions (acmi_band_info); forward 'bf16': the conv tower on one 16-bit MFMA per
    product.  Returns {component: (work, unit, ceiling, ms)}."""
    M = N * T
    K3 = 49 * C3
    imgs = M + N  # the rollout's towers (T steps) and the bootstrap forward
    f2, x3 = F16X2_F32EQ_PEAK_TFLOPS, X3_F32EQ_PEAK_TFLOPS
    c = {}

    def add(name, work, ceil, unit='GFLOP'):
        # work in G-units; ceil in T-units per second -> ms
        c[name] = (work, unit, ceil, work / ceil)

    # rollout: conv tower (conv1 u8 x f16x2 on two MFMAs; conv2 / conv3 f16x2), fc4 + heads
    tw1, tw23 = ((BF16_MFMA_PEAK_TFLOPS, BF16_MFMA_PEAK_TFLOPS) if forward == 'bf16'
                 else (U8F16X2_F32EQ_PEAK_TFLOPS, f2))
    add('tower conv1', 2 * 400 * 256 * 32 * imgs / 1e9, tw1)
    add('tower conv2 + conv3', (2 * 81 * 512 * 64 + 2 * 49 * 576 * C3) * imgs / 1e9, tw23)
    add('rollout fc4 + heads', (2 * K3 * 512 + 2 * 512 * (A + 1)) * imgs / 1e9, f2)
    # env stepping: the 4-frame stack read and written per env-step (HBM)
    add('stepper', 2 * 84 * 84 * 4 * M / 1e9, HBM_PEAK_GBS / 1e3, 'GB')
    chains = 2 if acktr else 1  # the loss backward, and the sampled-loss (G statistics) chain
    add('dX fc4 / conv3 / conv2', chains * (2 * K3 * 512 + 2 * 49 * 576 * C3 + 2 * 81 * 512 * 64) * M / 1e9, f2)
    if acktr:
        t2, t3 = band_tiles
        add('band conv2 (wgrad + A)', 2 * 64 * 64 * t2 * M / 1e9, f2)
        add('band conv3 (wgrad + A)', 2 * 64 * 64 * t3 * M / 1e9, f2)
        add('fc4 wgrad + A', 2 * ((K3 + 1) * (K3 + 2) / 2 + (K3 + 1) * 512) * M / 1e9, f2)
        add('heads wgrad + A', 2 * (513 * 514 / 2 + 513 * (A + 1)) * M / 1e9, x3)
        add('conv1 A factor (i8, unique)', 2 * 400 * 256 * 257 / 2 * M / 1e9, INT8_MFMA_PEAK_TOPS, 'Gop')
        add('conv1 wgrad', 2 * 400 * 257 * 32 * M / 1e9, U8F16X2_F32EQ_PEAK_TFLOPS)
        add('G factors (unique)', (512 * 513 + 81 * 64 * 65 + 49 * C3 * (C3 + 1) + 400 * 32 * 33) * M / 1e9, f2)
        # the damped inverses (fp64 block sweep, ~2 n^3 per matrix) every 10th update
        dims = [257, 513, 577, K3 + 1, 513, 513, 32, 64, C3, 512, A, 1]
        add('K-FAC inverse (1/10)', sum(2.0 * n ** 3 for n in dims) / 10 / 1e9, FP64_MFMA_PEAK_TFLOPS)
        # the preconditioned step: Ainv G Ginv per layer (f32 MFMA)
        blocks = [(257, 32), (513, 64), (577, C3), (K3 + 1, 512), (513, A), (513, 1)]
        add('K-FAC step', sum(2.0 * a * b * (a + b) for a, b in blocks) / 1e9, FP32_MFMA_PEAK_TFLOPS)
    else:
        add('wgrad conv1..heads', 2 * (400 * 257 * 32 + 81 * 513 * 64 + 49 * 577 * C3 + (K3 + 1) * 512
                                       + 513 * (A + 1)) * M / 1e9, f2)
    return c


def workload_name(algo, N, T, A, forward, world, games=None):
    """The BASELINE.json config a line measures (configs[1]-[4]; others: as given)."""
    if games == 'atari57':
        return ('Mixed Atari-57 {} {} envs/GPU x {} steps, {} actions, {} forward / fp32 K-FAC{}'.format(
            algo.upper(), N, T, A, forward, ' (BASELINE configs[4] shard)' if forward == 'bf16' and A == 18 else ''))
    if forward == 'bf16':
        return ('Atari {} {} envs/GPU x {} steps, {} actions, bf16 forward / fp32 K-FAC (BASELINE configs[4] '
                'shard)'.format(algo.upper(), N, T, A))
    name = 'Breakout {} {} envs/GPU x {} steps'.format(algo.upper(), N, T)
    if algo == 'a2c' and N * world == 32 and T == 5:
        return name + ' (BASELINE configs[1])'
    if algo == 'acktr' and N * world == 32 and T == 20:
        return name + ' (BASELINE configs[2])'
    if algo == 'acktr' and N == 512 and T == 20:
        return name + ' (BASELINE configs[3] shard)'
    return name


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--warmup', type=int, default=5)
    p.add_argument('--algo', choices=['acktr', 'a2c'], default='acktr')
    p.add_argument('--envs-per-gpu', type=int, default=512)
    p.add_argument('--nsteps', type=int, default=None, help='rollout length T (ACKTR 20, A2C 5)')
    p.add_argument('--num-actions', type=int, default=4, help='Breakout: 4; full Atari action set: 18')
    p.add_argument('--forward', choices=['f32', 'bf16'], default=None,
                   help='conv tower precision (default: ACMI_FORWARD or f32; bf16: BASELINE configs[4] '
                        '"bf16 forward / fp32 KFAC factors")')
    p.add_argument('--games', choices=['atari57'], default=None,
                   help='atari57: env e plays Atari-57 game e %% 57 (mixed-game batch, BASELINE configs[4]; '
                        'needs --num-actions 18); default: every env synthetic Breakout')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--cpu-iters', type=int, default=3, help='timed CPU-baseline iterations (at most ~20 s)')
    p.add_argument('--no-configs2', action='store_true',
                   help='skip the nested BASELINE configs[2] line (ACKTR 32 envs x 20 steps) timed after the headline')
    p.add_argument('--configs2-steps', type=int, default=60)
    p.add_argument('--quiet', action='store_true')
    return p.parse_args()


def _free_port():
    import socket
    sk = socket.socket()
    sk.bind(('127.0.0.1', 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def _rank_main(rank, world, port, argv):
    """One self-launched rank: torchrun's environment, then the ordinary run."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    sys.argv = [sys.argv[0]] + list(argv)
    run(parse())


def launch(args):
    """--gpus N without WORLD_SIZE: N spawned ranks (the parent stays off the GPU);
    a failed rank takes the others down and its exit code is returned."""
    import multiprocessing as mp
    ctx = mp.get_context('spawn')
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, args.gpus, port, sys.argv[1:]), name='bench-rank{}'.format(r))
             for r in range(args.gpus)]
    for p in procs:
        p.start()
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            p.join(0.2)
            if p.exitcode is None:
                continue
            alive.remove(p)
            if p.exitcode != 0 and rc == 0:
                rc = p.exitcode if p.exitcode > 0 else 128 - p.exitcode
                print('bench: {} exited with {}; stopping the other ranks'.format(p.name, p.exitcode),
                      file=sys.stderr)
                for q in alive:
                    q.terminate()
    return rc


def main():
    args = parse()
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(launch(args))
    run(args)


def _measure(args, N, T, A, algo, games, steps, warmup, prof_site=None, forward_mode=None):
    """Build the reference training graph for one workload and time `steps`
    iterations after `warmup` (barrier + synchronize on both sides; wall time is
    the max over ranks).  prof_site: the libacmi HIP-event profiling site of the
    roofline kernel (timed only for the headline workload)."""
    from actorcritic import _lib, parallel
    from actorcritic import session as sess
    from actorcritic.agents import MultiEnvAgent
    from actorcritic.envs.atari.model import AtariModel
    from actorcritic.envs.atari.wrappers import SyntheticAtariEnvs
    from actorcritic.examples.atari.a2c_acktr import create_optimizer
    from actorcritic.multi_env import MultiEnv
    from actorcritic.nn import linear_decay
    from actorcritic.objectives import A2CObjective

    world, rank = parallel.world_size(), parallel.rank()
    dev = torch.device('cuda', torch.cuda.current_device())
    acktr = algo == 'acktr'
    C3 = 32 if acktr else 64

    sess.reset_default_graph()
    env = MultiEnv(SyntheticAtariEnvs(N, num_actions=A, seed=1234, env_offset=rank * N, device=dev,
                                      games=games))
    # (forward_mode: this model's conv-tower precision, the acmi_net_t mode field)
    model = AtariModel(env.observation_space, env.action_space, C3, random_seed=7, device=dev,
                       forward_mode=forward_mode)
    agent = MultiEnvAgent(env, model, T)
    objective = A2CObjective(model, discount_factor=0.99, entropy_regularization_strength=0.01)
    gs = sess.get_or_create_global_step()
    max_step = 10000000 / (N * T * world)
    lr = linear_decay(0.25, 0.025, gs, max_step) if acktr else linear_decay(7e-4, 7e-5, gs, max_step)
    optimizer = create_optimizer(acktr, model, lr)
    op = objective.optimize_shared(optimizer, baseline_loss_weight=0.5, global_step=gs)
    if acktr:
        gs.assign(30)  # steady state: past the cold start (kfac_utils.py:42-44)

    def iteration(s, marks=None):
        if marks is not None:
            marks[0].record()
        obs, act, rew, term, nxt, infos = agent.interact(s)
        if marks is not None:
            marks[1].record()
        s.run(op, feed_dict={model.observations_placeholder: obs, model.bootstrap_observations_placeholder: nxt,
                             model.actions_placeholder: act, model.rewards_placeholder: rew,
                             model.terminals_placeholder: term}, host=False)
        if marks is not None:
            marks[2].record()

    tot_ms, cnt = ctypes.c_double(), ctypes.c_int()
    with sess.Session(dev) as s:
        for _ in range(warmup):
            iteration(s)
        torch.cuda.synchronize()
        parallel.barrier()
        torch.cuda.synchronize()
        if prof_site is not None:
            _lib.call('acmi_prof_enable', prof_site, max(1, steps))
        model.engine.comm_timing(True)
        marks = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
        inv_flags = []
        # Python's cyclic GC off inside the timed region, as timeit does: a
        # collection over the previous workload's objects (the nested configs[2]
        # run follows the headline one in this process) landed in some timed
        # regions of the host-launch-bound small config (rollout 0.52 -> 0.56-0.61 ms)
        gc.collect()
        gc.disable()
        try:
            t0 = time.perf_counter()
            host = []  # host time per iteration minus its wait on the previous rollout's event
            for k in range(steps):
                th = time.perf_counter()
                agent.last_sync_wait = 0.0
                iteration(s, marks[k])
                host.append(time.perf_counter() - th - getattr(agent, 'last_sync_wait', 0.0))
                inv_flags.append(bool(getattr(optimizer, 'last_flags', (0, 0, 0))[2]) if acktr else False)
            torch.cuda.synchronize()
            parallel.barrier()
            torch.cuda.synchronize()
            elapsed = time.perf_counter() - t0
        finally:
            gc.enable()
        if prof_site is not None:
            _lib.call('acmi_prof_collect', ctypes.byref(tot_ms), ctypes.byref(cnt))
            _lib.call('acmi_prof_enable', 0, 0)
        comm_ms, comm_bytes, comm_n = model.engine.comm_collect()
        model.engine.comm_timing(False)
    elapsed = parallel.max_over_ranks(elapsed, dev)
    comm_ms_max = parallel.max_over_ranks(comm_ms, dev)
    roll_ms = [m[0].elapsed_time(m[1]) for m in marks]
    upd_ms = [m[1].elapsed_time(m[2]) for m in marks]
    mean = lambda xs: (sum(xs) / len(xs)) if xs else None
    return dict(value=N * T * steps * world / elapsed, ms_per_step=1e3 * elapsed / steps, elapsed=elapsed,
                update_ms=mean(upd_ms), update_ms_inverse_iters=mean([u for u, f in zip(upd_ms, inv_flags) if f]),
                update_ms_plain_iters=mean([u for u, f in zip(upd_ms, inv_flags) if not f]),
                rollout_ms=mean(roll_ms), host_ms=1e3 * mean(host[1:] or host), comm_ms=comm_ms_max,
                comm_bytes=comm_bytes, comm_n=comm_n,
                prof_ms=tot_ms.value, prof_n=cnt.value)


def _cpu_leg(N, T, A, C3, algo, games, iters):
    """The CPU baseline (oracle/cpu_baseline.py: measurement infrastructure, run
    after the timed GPU region) on the same workload."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import cpu_baseline
    r = cpu_baseline.run(n_envs=N, n_steps=T, iters=iters, A=A, C3=C3, algo=algo, games=games)
    return {'value': r['env_steps_per_s'], 'unit': 'env-steps/s', 'cores': r['threads'], 'kind': 'port',
            'sample': '{} timed iterations (after one warm-up; per iteration min {:.2f} s, max {:.2f} s) of '
                      'the same {} workload ({} envs x {} steps): torch-CPU fp32 restatement, {}{}'.format(
                          r['iters'], min(r['iter_s']), max(r['iter_s']), algo.upper(), r['n_envs'],
                          r['n_steps'], r['structure'],
                          ', K-FAC inverse timed once and amortised 1/10' if algo == 'acktr' else ''),
            'iter_s': r['iter_s'], 'update_ms': r['update_ms'], 'rollout_ms': r['rollout_ms']}


def run(args):
    from actorcritic import _lib, parallel

    world, rank = parallel.init_from_env()
    # the headline model's forward precision: --forward, else the process default
    # (ACMI_FORWARD); carried by its net, not set process-wide
    fwd = {'bf16': _lib.FWD_BF16, 'f32': _lib.FWD_F32}.get(args.forward, _lib.load().acmi_get_forward_mode())
    args.forward = 'bf16' if fwd == _lib.FWD_BF16 else 'f32'
    if world != args.gpus:
        raise SystemExit('bench: --gpus {} but the process group has {} ranks (WORLD_SIZE={})'.format(
            args.gpus, world, os.environ.get('WORLD_SIZE')))
    acktr = args.algo == 'acktr'
    N = args.envs_per_gpu
    T = args.nsteps or (20 if acktr else 5)
    C3 = 32 if acktr else 64
    A = args.num_actions
    r = _measure(args, N, T, A, args.algo, args.games, args.steps, args.warmup, prof_site=_lib.PROF_CONV2_WGRAD,
                 forward_mode=fwd)
    value, ms_per_step = r['value'], r['ms_per_step']
    tot_ms = ctypes.c_double(r['prof_ms'])
    cnt = ctypes.c_int(r['prof_n'])

    # BASELINE configs[2] (the reference's own ACKTR config, a2c_acktr.py:306-310:
    # 32 envs x 20 steps, Breakout, f32) -- the config north_star's ">=10x the
    # reference CPU at 1 GPU" target is stated on -- timed by the same clock in the
    # same run, with its SubprocessEnv CPU leg (32 Pipe children)
    c2 = None
    if (world == 1 and not args.no_configs2
            and not (acktr and N == 32 and T == 20 and A == 4 and args.forward == 'f32' and not args.games)):
        c2r = _measure(args, 32, 20, 4, 'acktr', None, args.configs2_steps, max(5, args.warmup),
                       forward_mode=_lib.FWD_F32)
        c2 = {'workload': workload_name('acktr', 32, 20, 4, 'f32', 1), 'envs': 32, 'num_steps': 20,
              'num_actions': 4, 'forward': 'f32', 'steps': args.configs2_steps, 'warmup': max(5, args.warmup),
              'value': c2r['value'], 'unit': 'env-steps/s', 'ms_per_step': c2r['ms_per_step'],
              'update_ms': c2r['update_ms'], 'update_ms_inverse_iters': c2r['update_ms_inverse_iters'],
              'update_ms_plain_iters': c2r['update_ms_plain_iters'], 'rollout_ms': c2r['rollout_ms'],
              'host_ms_per_step': c2r['host_ms']}

    # dominant kernel: conv2 weight gradient fused with the K-FAC A factor,
    # [P;1]^T [P | dY] over the M*81 conv2 output pixels, P = 4x4x32 patches.
    # Algorithmic FLOP per pixel = 2 * (unique outputs): the symmetric 513x513
    # A factor counted once (513*514/2) plus the 513x64 [dW;db] block
    # (DESIGN.md "Roofline").  The slab-grouped kernel (symred.hpp) executes 44
    # 64x64 sub-tiles per pixel (2*44*64*64 FLOP), reported as executed_tflops.
    M = N * T
    rows = 81 * M
    lib = _lib.load()
    x3 = lib.acmi_get_gemm_mode() == _lib.GEMM_X3
    band = acktr and x3 and lib.acmi_get_conv_stats_mode() == _lib.CONV_STATS_BAND
    patch_flops = 2.0 * (513 * 514 / 2 + 513 * 64) * rows  # the patch-row sums it replaces
    if band:
        # pixel-pair band reduction (band.hpp): the needed 64x64 sub-tiles of
        # [X | dY]^T [X | dY] over the M images' dense rows, 2*64*64 FLOP per
        # sub-tile and image; every executed sub-tile is needed
        info = (ctypes.c_int64 * 5)()
        _lib.call('acmi_band_info', 1, C3, M, info)
        kern_flops = exec_flops = 2.0 * 64 * 64 * info[0] * M
        kern_name = ('conv2 band reduction: wgrad + K-FAC A factor over pixel-pair sub-tiles '
                     '(f16x2 split-operand MFMA, f32-accurate)')
    elif acktr:
        kern_flops = patch_flops
        exec_flops = 2.0 * 44 * 64 * 64 * rows
        kern_name = ('conv2 wgrad + K-FAC A-factor reduction GEMM (bf16x3 split-operand MFMA, f32-accurate)'
                     if x3 else 'conv2 wgrad + K-FAC A-factor reduction GEMM (f32 MFMA)')
    else:
        kern_flops = 2.0 * 513 * 64 * rows
        exec_flops = 2.0 * 8 * 128 * 32 * rows
        kern_name = ('conv2 wgrad reduction GEMM (bf16x3 split-operand MFMA, f32-accurate)' if x3
                     else 'conv2 wgrad reduction GEMM (f32 MFMA)')
    # MFMAs per f32-accurate product: 3 (f16x2, band), 6 (bf16x3), 1 (f32 MFMA)
    nmf = 3 if band else 6 if x3 else 1
    peak = F16X2_F32EQ_PEAK_TFLOPS if band else X3_F32EQ_PEAK_TFLOPS if x3 else FP32_MFMA_PEAK_TFLOPS
    kern_ms = tot_ms.value / max(1, cnt.value)
    achieved = kern_flops / (kern_ms * 1e-3) / 1e12 if cnt.value else None
    executed = exec_flops / (kern_ms * 1e-3) / 1e12 if cnt.value else None
    traffic = measured_traffic(kern_name, 'Breakout {} {} envs/GPU x {} steps'.format(args.algo.upper(), N, T))
    roofline = {'bound': 'mfma', 'kernel': kern_name,
                'achieved': achieved, 'peak': peak, 'unit': 'TFLOP/s',
                'frac': (achieved / peak) if achieved else None, 'traffic': traffic,
                'launches': cnt.value, 'avg_ms': kern_ms, 'flops_per_launch': kern_flops,
                'executed_tflops': executed}
    if band and achieved:
        roofline['sub_tiles'] = int(info[0])
        roofline['groups'] = int(info[1])
        roofline['chunks'] = int(info[2])
        # the patch-row formulation's unique FLOPs over the same time: the rate
        # the replaced kernel would have needed to match
        roofline['patch_equivalent_tflops'] = patch_flops / (kern_ms * 1e-3) / 1e12
    if x3:
        # the whole iteration against its roofline: every kernel's algorithmic work
        # at the ceiling of its arithmetic, summed, over the measured ms_per_step
        bt = None
        if acktr:
            i2, i3 = (ctypes.c_int64 * 5)(), (ctypes.c_int64 * 5)()
            _lib.call('acmi_band_info', 1, C3, M, i2)
            _lib.call('acmi_band_info', 2, C3, M, i3)
            bt = (int(i2[0]), int(i3[0]))
        ceil = iteration_ceiling(N, T, A, C3, acktr, bt, args.forward)
        ceil_ms = sum(v[3] for v in ceil.values())
        roofline['iteration_frac'] = ceil_ms / ms_per_step
        roofline['iteration_ceiling_ms'] = ceil_ms
        roofline['iteration_ceiling'] = {k: {'work': round(v[0], 4), 'unit': v[1], 'ceiling_per_s': round(v[2], 1),
                                             'ms': round(v[3], 5)} for k, v in ceil.items()}
    if x3 and achieved:
        # peak = 16-bit dense peak / nmf (f32-equivalent); the same rate against
        # the f32-input MFMA peak and the bf16x3 ceiling, and the 16-bit MFMA work
        # actually issued
        roofline['mfma_per_product'] = nmf
        roofline['frac_of_f32_mfma_peak'] = achieved / FP32_MFMA_PEAK_TFLOPS
        roofline['frac_of_bf16x3_ceiling'] = achieved / X3_F32EQ_PEAK_TFLOPS
        roofline['executed_16bit_tflops'] = nmf * executed
        roofline['executed_frac_of_16bit_peak'] = nmf * executed / BF16_MFMA_PEAK_TFLOPS

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the same workload as the GPU line (envs, steps, algorithm, actions, C3)
        cpu = _cpu_leg(N, T, A, C3, args.algo, args.games, args.cpu_iters)
        if c2 is not None:
            # configs[2]'s CPU leg: 32 SubprocessEnv children behind the Pipe protocol
            c2['cpu_baseline'] = _cpu_leg(32, 20, 4, 32, 'acktr', None, args.cpu_iters)
            c2['speedup_vs_cpu'] = c2['value'] / c2['cpu_baseline']['value']

    if rank == 0:
        out = {
            'metric': 'env-steps/sec (whole node) + ACKTR update ms, Breakout 84x84x4',
            'value': value, 'unit': 'env-steps/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': ms_per_step, 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
            'dtype': 'fp32' if args.forward == 'f32' else 'bf16 forward / fp32 update', 'data': 'synthetic (hashed 84x84 u8 frames, random-init orthogonal weights)',
            'config': {'workload': workload_name(args.algo, N, T, A, args.forward, world, args.games),
                       'algo': args.algo, 'games': args.games or 'Breakout',
                       'envs_per_gpu': N, 'num_steps': T,
                'global_envs': N * world, 'num_actions': A, 'conv3_filters': C3, 'forward': args.forward,
                'parallelism': 'dp{}'.format(world)},
            'update_ms': r['update_ms'], 'update_ms_inverse_iters': r['update_ms_inverse_iters'],
            'update_ms_plain_iters': r['update_ms_plain_iters'], 'rollout_ms': r['rollout_ms'],
            # host time per iteration of the Python loop (ctypes launches, graph
            # evaluation): below ms_per_step the GPU, not the host, sets the pace
            'host_ms_per_step': r['host_ms'],
            # communication: compute-stream stall on the per-update all-reduce
            # (NetEngine.comm_timing; max over ranks), bytes summed per update
            'allreduce_ms': r['comm_ms'] if world > 1 else 0.0, 'allreduce_bytes': r['comm_bytes'],
            'allreduce_updates_timed': r['comm_n'], 'dist_backend': parallel.backend_name(),
            'roofline': roofline, 'cpu_baseline': cpu,
            # BASELINE configs[2] on the same clock (null at N > 1 or with --no-configs2)
            'configs2': c2,
        }
        if cpu:
            out['speedup_vs_cpu'] = value / cpu['value']
        print(json.dumps(out))
    parallel.destroy()


if __name__ == '__main__':
    main()
