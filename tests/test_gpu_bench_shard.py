"""The update statistics at the bench shard's own size against float64.

BASELINE configs[3] runs 512 envs x 20 steps per GPU: acmi_backward and
acmi_kfac_output_stats see M = 10240 image rows, the size at which the production
plans engage -- the band reduction's 4-chunk, 243-group conv2 plan (band.hpp,
bandplan.hpp), conv2's input gradient on pre-split weights (convt2.hpp) with the
conv1 G factor fused into the sampled chain, the role-split conv1 A-factor kernel over
many i8 chunks, the six-slab fc4 plan.  Every parameter-gradient block, all five A
factors and all six G factors of one backward + sampled-loss backward are compared
with a float64 computation of the same formulas on the GPU (torch.float64 GEMMs,
chunked over images): the reference's conv layers as patch products
(envs/atari/model.py:173-217, nn.py:88-126), kfac's factors as the DESIGN.md section 4
conventions (rows = every conv location of every image, homogeneous coordinate last,
G from the sampled head gradients of oracle.sampled_head_grads).

Tolerances (max-abs error over max-abs value, per block): gradients and A factors
2e-5, G factors 5e-5 -- the section 5 bounds of the small-size tests.
"""
import ctypes
import os
import sys

import numpy as np
import pytest
import torch

from actorcritic import _lib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'oracle'))
import oracle  # noqa: E402

pytestmark = pytest.mark.gpu


def _patches(x, k, s):
    """[B,H,W,C] -> rows (img, oh, ow), columns (kh, kw, c) (extract_image_patches order)."""
    p = x.unfold(1, k, s).unfold(2, k, s)  # B, OH, OW, C, KH, KW
    return p.permute(0, 1, 2, 4, 5, 3).reshape(-1, k * k * x.shape[-1])


def _conv_input_grad(dy, w, s, in_shape):
    k, _, cin, co = w.shape
    B, OH, OW, _ = dy.shape
    dp = (dy.reshape(-1, co) @ w.reshape(-1, co).t()).reshape(B, OH, OW, k, k, cin)
    dx = torch.zeros(in_shape, dtype=dy.dtype, device=dy.device)
    for kh in range(k):
        for kw in range(k):
            dx[:, kh:kh + s * (OH - 1) + 1:s, kw:kw + s * (OW - 1) + 1:s, :] += dp[:, :, :, kh, kw, :]
    return dx


class _Ref(object):
    """Sums of grads, A factors and G factors over image chunks in `dtype`
    (float64: the reference; float32: what plain f32 arithmetic gets -- the bar of
    the "f32-class" claim)."""

    def __init__(self, blocks, A, C3, dev, dtype=torch.float64):
        self.dt = dtype
        self.w = [b.to(dtype) for b in blocks]
        self.A, self.C3, self.dev = A, C3, dev
        self.grad = None
        self.afac = [0.0] * 5
        self.gfac = [0.0] * 6
        self.rows = [0] * 6

    def _forward(self, obs):
        w1, b1, w2, b2, w3, b3, w4, b4, wp, bp, wv, bv = self.w
        x = obs.to(self.dt) / 255.0
        p1 = _patches(x, 8, 4)
        a1 = torch.relu(p1 @ w1.reshape(-1, 32) + b1).reshape(-1, 20, 20, 32)
        p2 = _patches(a1, 4, 2)
        a2 = torch.relu(p2 @ w2.reshape(-1, 64) + b2).reshape(-1, 9, 9, 64)
        p3 = _patches(a2, 3, 1)
        a3 = torch.relu(p3 @ w3.reshape(-1, self.C3) + b3).reshape(-1, 7, 7, self.C3)
        a3f = a3.reshape(a3.shape[0], -1)
        a4 = torch.relu(a3f @ w4 + b4)
        return [p1, p2, p3, a3f, a4], (a1, a2, a3, a4)

    def _chain(self, masks, dlogits, dvalue):
        w1, b1, w2, b2, w3, b3, w4, b4, wp, bp, wv, bv = self.w
        m1, m2, m3, m4 = masks
        d4 = (dlogits @ wp.t() + dvalue[:, None] * wv[:, 0][None, :]) * m4
        d3 = (d4 @ w4.t()).reshape(m3.shape) * m3
        d2 = _conv_input_grad(d3, w3, 1, m2.shape) * m2
        d1 = _conv_input_grad(d2, w2, 2, m1.shape) * m1
        return [d1.reshape(-1, 32), d2.reshape(-1, 64), d3.reshape(-1, self.C3), d4, dlogits, dvalue[:, None]]

    def _inputs(self, obs, gpu_acts):
        """The layer inputs from the GPU's own forward (a1..a4 in float64): what the
        update is fed (a2c_acktr.py:243-247) when the forward is not float64-exact
        (the bf16 tower of BASELINE configs[4])."""
        a1, a2, a3, a4 = [a.to(self.dt) for a in gpu_acts]
        x = obs.to(self.dt) / 255.0
        return [_patches(x, 8, 4), _patches(a1, 4, 2), _patches(a2, 3, 1), a3.reshape(a3.shape[0], -1), a4]

    def add(self, obs, gpu_acts, dlogits, dvalue, g_pi, g_v, gpu_inputs=False):
        """gpu_acts: the kernel forward's f32 a1..a4 of these images, whose ReLU
        masks the chains use: a pre-activation within f32 rounding of 0 may have
        the other sign in float64, and at 10240 rows such flips (one whole term of
        a cancelling sum each) would dominate the comparison of the backward's
        arithmetic.  The forward itself is compared with float64 elsewhere.
        gpu_inputs: take the layer inputs from gpu_acts too (else the float64
        forward's)."""
        ins = self._inputs(obs, gpu_acts) if gpu_inputs else self._forward(obs)[0]
        ins = ins + [ins[4]]
        masks = [(a > 0).to(self.dt) for a in gpu_acts]
        douts = self._chain(masks, dlogits, dvalue)
        gouts = self._chain(masks, g_pi, g_v)
        blocks = []
        for l in range(6):
            xin = torch.cat([ins[l], torch.ones(ins[l].shape[0], 1, dtype=self.dt, device=self.dev)], 1)
            blocks.append((xin.t() @ douts[l]).reshape(-1))
            if l < 5:
                self.afac[l] = self.afac[l] + xin.t() @ xin
            self.gfac[l] = self.gfac[l] + gouts[l].t() @ gouts[l]
            self.rows[l] += xin.shape[0]
        g = torch.cat(blocks)
        self.grad = g if self.grad is None else self.grad + g

    def result(self):
        return (self.grad, [a / r for a, r in zip(self.afac, self.rows)],
                [g / r for g, r in zip(self.gfac, self.rows)])


def _rel(got, ref):
    return ((got.double() - ref).abs().max() / ref.abs().max()).item()


def _stats_vs_float64(lib, cuda, B, params, seed=2024):
    """One acmi_forward + acmi_backward (loss gradients + A factors) + one
    acmi_kfac_output_stats (G factors of the sampled losses) over B images, each
    block against float64 (and against plain float32 arithmetic of the same
    formulas): {(kind, block): (kernel rel err, plain-f32 rel err)}."""
    from actorcritic._engine import Layout
    A, C3 = 4, 32
    L = Layout(A, C3)
    gen = torch.Generator(device=cuda).manual_seed(seed)
    obs = torch.randint(0, 256, (B, 84, 84, 4), generator=gen, device=cuda, dtype=torch.uint8)
    z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=cuda)
    t = dict(a1=z(B, 20, 20, 32), a2=z(B, 9, 9, 64), a3=z(B, 7, 7, C3), a4=z(B, 512), logits=z(B, A), value=z(B))
    acts = _lib.Acts(*[t[k].data_ptr() for k in ('a1', 'a2', 'a3', 'a4', 'logits', 'value')], A)
    zi = lambda *s: torch.zeros(*s, dtype=torch.int32, device=cuda)  # the production path's ReLU' masks
    t.update(m1=zi(B, 400), m2=zi(B, 162), m3=zi(B, 49 * C3 // 32))
    acts.m1, acts.m2, acts.m3 = t['m1'].data_ptr(), t['m2'].data_ptr(), t['m3'].data_ptr()
    prep = torch.empty(int(lib.acmi_conv_prep_bytes(C3)), dtype=torch.uint8, device=cuda)
    net = _lib.Net(A, C3, params.data_ptr(), prep.data_ptr())
    st = _lib.stream_handle()
    _lib.call('acmi_conv_prepare', ctypes.byref(net), _lib.ptr(prep), st)
    _lib.call('acmi_forward', ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts), 1, st)
    # head gradients shaped like the A2C loss's (a2c_loss: mean over M rows)
    ldh = 8
    dhead = z(B, ldh)
    dhead[:, :A + 1] = torch.randn(B, A + 1, generator=gen, device=cuda) / B
    din = (ctypes.c_int64 * 6)()
    so = (ctypes.c_int64 * 11)()
    tot = ctypes.c_int64()
    _lib.call('acmi_kfac_layout', A, C3, din, None, so, ctypes.byref(tot))
    ws = z(int(lib.acmi_backward_ws_floats(B, A, C3)))
    d = [z(B, 20, 20, 32), z(B, 9, 9, 64), z(B, 7, 7, C3), z(B, 512)]
    bwd = _lib.Bwd(*[x.data_ptr() for x in d], dhead.data_ptr(), ldh)
    grads, astat, gstat = z(params.numel()), z(tot.value), z(tot.value)
    _lib.call('acmi_backward', ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts),
              ctypes.byref(bwd), _lib.ptr(grads), _lib.ptr(astat), _lib.ptr(ws), ws.numel(), st)
    ds = [z(B, 20, 20, 32), z(B, 9, 9, 64), z(B, 7, 7, C3), z(B, 512)]
    dhead_s = z(B, ldh)  # the sampled chain writes its own head gradients here
    bwd_s = _lib.Bwd(*[x.data_ptr() for x in ds], dhead_s.data_ptr(), ldh)
    seed_s, counter = 0x4b464143, 41
    _lib.call('acmi_kfac_output_stats', ctypes.byref(net), B, ctypes.byref(acts), ctypes.byref(bwd_s), seed_s, 0,
              counter, _lib.ptr(gstat), _lib.ptr(ws), ws.numel(), st)
    torch.cuda.synchronize()
    assert torch.isfinite(grads).all() and torch.isfinite(astat).all() and torch.isfinite(gstat).all()

    # the sampled head gradients from the kernel's own f32 logits and counters
    g_pi, g_v, _ = oracle.sampled_head_grads(t['logits'].cpu().numpy(), seed_s, 0, counter)
    g_pi = torch.from_numpy(np.asarray(g_pi, np.float64)).to(cuda)
    g_v = torch.from_numpy(np.asarray(g_v, np.float64)).to(cuda)
    ref = _Ref(L.split(params), A, C3, cuda)
    ref32 = _Ref(L.split(params), A, C3, cuda, torch.float32)
    dh64 = dhead.double()
    chunk = 1024
    for i in range(0, B, chunk):
        j = min(B, i + chunk)
        for r in (ref, ref32):
            r.add(obs[i:j], [t[k][i:j] for k in ('a1', 'a2', 'a3', 'a4')], dh64[i:j, :A].to(r.dt),
                  dh64[i:j, A].to(r.dt), g_pi[i:j].to(r.dt), g_v[i:j].to(r.dt))
    g_ref, a_ref, gf_ref = ref.result()
    g_32, a_32, gf_32 = ref32.result()

    errs = {}
    ends = L.offsets[1:] + [L.nparams]
    for blk, (o, e) in enumerate(zip(L.offsets, ends)):
        errs[('grad', blk)] = (_rel(grads[o:e], g_ref[o:e]), _rel(g_32[o:e], g_ref[o:e]))
    for f in range(5):
        n = din[f]
        errs[('A', f)] = (_rel(astat[so[f]:so[f] + n * n].reshape(n, n), a_ref[f]), _rel(a_32[f], a_ref[f]))
    for l in range(6):
        n = gf_ref[l].shape[0]
        errs[('G', l)] = (_rel(gstat[so[5 + l]:so[5 + l] + n * n].reshape(n, n), gf_ref[l]), _rel(gf_32[l], gf_ref[l]))
    for k, (v, v32) in errs.items():
        print(k, 'kernel %.2e  plain f32 %.2e' % (v, v32))
    return errs


def test_update_statistics_at_bench_shard_match_float64(lib, cuda):
    """One acmi_backward (loss gradients + A factors) and one acmi_kfac_output_stats
    (G factors of the sampled losses) over M = 512 x 20 = 10240 images -- the
    BASELINE configs[3] per-GPU shard, default arithmetic (f16x2 / bf16x3, band
    reductions, pre-split weights) -- against float64 on the GPU."""
    from actorcritic._engine import Layout
    B = 512 * 20
    info = (ctypes.c_int64 * 5)()
    _lib.call('acmi_band_info', 1, 32, B, info)
    assert info[2] >= 2, list(info)  # the production plan of the bench shard: several image chunks
    params = torch.from_numpy(Layout(4, 32).init_params(seed=7)).to(cuda)
    errs = _stats_vs_float64(lib, cuda, B, params)
    # f32-class: within the section 5 bound (gradients / A factors 2e-5, G 5e-5)
    # or within 4x of what plain float32 arithmetic of the same formulas gets --
    # at 10240 images the weight-gradient sums cancel (random-sign head
    # gradients), which magnifies every implementation's rounding alike
    for k, (v, v32) in errs.items():
        tol = 5e-5 if k[0] == 'G' else 2e-5
        assert v < max(tol, 4 * v32), (k, v, v32)


def test_update_statistics_with_tiny_output_gradients(lib, cuda):
    """Head weights scaled to ~1e-17: every output gradient d1..d4 (and so the G
    factors' Grams of one tensor with itself) sits near 1e-17 ~ 2^-56.  f16x2 scales
    each operand by a power of two putting its bound below 2^14 (f16x2.hpp
    f16x2_scale); uncapped, that scale would be 2^70 and the Gram's unscale
    1/(s s) = 1/2^140 = 1/inf would zero the factor.  The cap (2^60) keeps it
    finite: the G factors (~1e-34), the gradients and the A factors stay within the
    bench-shard test's f32-class bounds of float64."""
    from actorcritic._engine import Layout
    L = Layout(4, 32)
    p = L.init_params(seed=7)
    for blk in (8, 9, 10, 11):  # fc_policy W, b; fc_baseline W, b
        o, e = L.offsets[blk], (L.offsets[blk + 1] if blk < 11 else L.nparams)
        p[o:e] *= np.float32(1e-15)
    params = torch.from_numpy(p).to(cuda)
    errs = _stats_vs_float64(lib, cuda, 256, params, seed=5)
    for k, (v, v32) in errs.items():
        tol = 5e-5 if k[0] == 'G' else 2e-5
        assert v < max(tol, 4 * v32), (k, v, v32)


_SHARD_CASES = [
    # (N, T, A, games, forward): the per-GPU shards of BASELINE configs[3] and configs[4]
    (512, 20, 4, None, 'f32'),
    (1024, 20, 18, 'atari57', 'bf16'),
]


@pytest.mark.parametrize('N,T,A,games,fwd', _SHARD_CASES, ids=['configs3-shard-512x20', 'configs4-shard-1024x20-a18-bf16'])
def test_acktr_update_at_shard_size_matches_float64(lib, cuda, N, T, A, games, fwd):
    """One steady-state ACKTR update at gs = 40 -- covariance EMA (first step, zero-
    debiased: the batch statistics), the damped inverses (acmi_kfac_inverse), the
    preconditioned trust-region momentum step (acmi_kfac_step) -- through the
    reference's graph (objectives.optimize_shared, kfac_utils.py:38-53) at the
    per-GPU shard sizes of BASELINE configs[3] (512 envs x 20 steps, M = 10240) and
    configs[4] (1024 x 20 = 20480 rows, A = 18, mixed Atari-57 games, bf16 forward /
    fp32 K-FAC): the production band plans, the 19-column heads and
    kfac_narrow_kernel at their own sizes.

    The float64 side (torch.float64 on the GPU for the 20480-row sums, numpy for the
    inverses and the step: oracle.damped_inverses / kfac_step) is fed the GPU's own
    forward -- activations, logits, values, targets (a2c_acktr.py:243-247) -- so it
    checks the update's arithmetic on identical inputs.  Per K-FAC block: gradients
    and A factors within 2e-5 (or 4x plain-f32 arithmetic of the same sums), G
    factors 5e-5 (or 4x f32), damped inverses rel 1e-3, preconditioned gradient and
    step rel-L2 1e-3 (north_star), the trust-region coefficient rel 1e-3.
    References: kfac_utils.py:38-53, a2c_acktr.py:243-247, policies.py:146-158,
    baselines.py:55-69."""
    from actorcritic import session as sess
    from actorcritic.agents import MultiEnvAgent
    from actorcritic.envs.atari.model import AtariModel
    from actorcritic.envs.atari.wrappers import SyntheticAtariEnvs
    from actorcritic.examples.atari.a2c_acktr import create_optimizer
    from actorcritic.multi_env import MultiEnv
    from actorcritic.nn import linear_decay
    from actorcritic.objectives import A2CObjective
    C3 = 32
    prev_mode = lib.acmi_get_forward_mode()
    _lib.call('acmi_set_forward_mode', _lib.FWD_BF16 if fwd == 'bf16' else _lib.FWD_F32)
    try:
        sess.reset_default_graph()
        kw = {} if games is None else dict(games=games)
        env = MultiEnv(SyntheticAtariEnvs(N, num_actions=A, seed=11, device=cuda, **kw))
        params = oracle.init_params(A, C3, seed=1)
        model = AtariModel(env.observation_space, env.action_space, C3, params=params, random_seed=3, device=cuda)
        agent = MultiEnvAgent(env, model, T)
        obj = A2CObjective(model)
        gs = sess.get_or_create_global_step()
        opt = create_optimizer(True, model, linear_decay(0.25, 0.025, gs, 1000))
        op = obj.optimize_shared(opt, 0.5, global_step=gs)
        gs.assign(40)
        M = N * T
        with sess.Session() as s:
            data = agent.interact(s)
            feed = {model.observations_placeholder: data[0], model.bootstrap_observations_placeholder: data[4],
                    model.actions_placeholder: data[1], model.rewards_placeholder: data[2],
                    model.terminals_placeholder: data[3]}
            fwd_out = model.engine.lookup_rollout(data[0])
            acts = fwd_out.acts
            gpu_acts = [acts.a1[:M].clone(), acts.a2[:M].clone(), acts.a3[:M].clone(), acts.a4[:M].clone()]
            logits32 = fwd_out.flat_logits.cpu().numpy().copy()
            value64 = fwd_out.flat_value.cpu().double().numpy()
            p_before = model.params.cpu().numpy().astype(np.float64)
            tg = np.asarray(s.run(obj.target_values, feed_dict=feed), np.float64).reshape(-1)
            s.run(op, feed_dict=feed)
            torch.cuda.synchronize()
        assert opt.last_flags == (False, True, True), opt.last_flags  # K-FAC step + covariance + inverse
        grads_gpu = model.engine.update_state(M).grads.cpu().numpy().astype(np.float64)
        st = opt.state
        fac = st['factors'].cpu().numpy().astype(np.float64)
        got_pre = st['precon'].cpu().numpy().astype(np.float64)
        got_p = model.params.cpu().numpy().astype(np.float64)
        coeff_gpu = float(st['coeff'][0])
        inv_got = st['inv']
        obs = data[0].reshape(M, 84, 84, 4)
        act = data[1].cpu().numpy().reshape(-1)
        if games is not None:
            assert act.max() >= 4  # the draws reach actions beyond Breakout's four
    finally:
        _lib.call('acmi_set_forward_mode', prev_mode)

    # float64: head gradients of the loss and the sampled losses from the GPU's logits
    lg = oracle.a2c_loss_and_head_grads(logits32.astype(np.float64), value64, act, tg)
    g_pi, g_v, _ = oracle.sampled_head_grads(logits32, 0x4b464143, 0, 40)
    blocks = [torch.from_numpy(b).to(cuda) for b in oracle.unpack(p_before, A, C3)]
    ref = _Ref(blocks, A, C3, cuda)
    ref32 = _Ref(blocks, A, C3, cuda, torch.float32)
    dl = torch.from_numpy(np.asarray(lg['dlogits'])).to(cuda)
    dv = torch.from_numpy(np.asarray(lg['dvalue'])).to(cuda)
    gp = torch.from_numpy(np.asarray(g_pi, np.float64)).to(cuda)
    gv = torch.from_numpy(np.asarray(g_v, np.float64)).to(cuda)
    chunk = 1024
    for i in range(0, M, chunk):
        j = min(M, i + chunk)
        for r in (ref, ref32):
            r.add(obs[i:j], [a[i:j] for a in gpu_acts], dl[i:j].to(r.dt), dv[i:j].to(r.dt), gp[i:j].to(r.dt),
                  gv[i:j].to(r.dt), gpu_inputs=True)
    g_ref, a_ref, gf_ref = ref.result()
    g_32, a_32, gf_32 = ref32.result()
    L = model.engine.layout
    names = ['conv1', 'conv2', 'conv3', 'fc4', 'fc_policy', 'fc_baseline']
    off, nparams = oracle.param_offsets(A, C3)
    spans = [(names[l], off[2 * l], off[2 * l + 2] if l < 5 else nparams) for l in range(6)]
    g_ref_np = g_ref.cpu().numpy()
    for name, lo, hi in spans:
        v = np.abs(grads_gpu[lo:hi] - g_ref_np[lo:hi]).max() / np.abs(g_ref_np[lo:hi]).max()
        v32 = _rel(g_32[lo:hi], g_ref[lo:hi])
        print('grad %-11s kernel %.2e  plain f32 %.2e' % (name, v, v32))
        assert v < max(2e-5, 4 * v32), ('grad', name, v, v32)
    afac, gfac = [a.cpu().numpy() for a in a_ref], [g.cpu().numpy() for g in gf_ref]
    for f in range(5):
        d = L.din[f]
        got = fac[L.stat_off[f]:L.stat_off[f] + d * d].reshape(d, d)
        v, v32 = np.abs(got - afac[f]).max() / np.abs(afac[f]).max(), _rel(a_32[f], a_ref[f])
        print('A %d kernel %.2e  plain f32 %.2e' % (f, v, v32))
        assert v < max(2e-5, 4 * v32), ('A', f, v, v32)
    for l in range(6):
        d = L.dout[l]
        got = fac[L.stat_off[5 + l]:L.stat_off[5 + l] + d * d].reshape(d, d)
        v, v32 = np.abs(got - gfac[l]).max() / np.abs(gfac[l]).max(), _rel(gf_32[l], gf_ref[l])
        print('G %d kernel %.2e  plain f32 %.2e' % (l, v, v32))
        assert v < max(5e-5, 4 * v32), ('G', l, v, v32)
    inv = oracle.damped_inverses(afac, gfac, 0.01)
    for l in range(6):
        for m, r in ((2 * l, inv[l][0]), (2 * l + 1, inv[l][1])):
            got = L.inverse_block(inv_got, m).cpu().numpy().astype(np.float64)
            rel = np.abs(got - r).max() / np.abs(r).max()
            print('inverse %-11s %s rel %.2e' % (names[l], 'AG'[m % 2], rel))
            assert rel < 1e-3, ('inverse', l, m % 2, rel)
    new_p, _, precon, coeff = oracle.kfac_step(p_before, np.zeros_like(p_before), g_ref_np, inv,
                                               oracle.linear_decay(0.25, 0.025, 40, 1000), 0.9, 1e-4, A, C3)
    for name, lo, hi in spans:
        e_pre = np.linalg.norm(got_pre[lo:hi] - precon[lo:hi]) / np.linalg.norm(precon[lo:hi])
        e_step = np.linalg.norm(got_p[lo:hi] - new_p[lo:hi]) / np.linalg.norm(new_p[lo:hi] - p_before[lo:hi])
        print('block %-11s precon rel-L2 %.2e  step rel-L2 %.2e' % (name, e_pre, e_step))
        assert e_pre < 1e-3, (name, 'precon', e_pre)
        assert e_step < 1e-3, (name, 'step', e_step)
    print('coeff gpu %.6e float64 %.6e' % (coeff_gpu, coeff))
    assert coeff_gpu == pytest.approx(coeff, rel=1e-3)
    assert np.linalg.norm(got_pre - precon) / np.linalg.norm(precon) < 1e-3
