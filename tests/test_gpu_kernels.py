"""Kernel-level parity of libacmi against plain PyTorch float64 references on the CPU.

These are the early numerics checks for the f32 MFMA GEMM engine (forward, input
gradients, fused weight-gradient/A-factor reductions), the fp64 damped inverse, the
trust-region step and the optimizers.  Tolerances are written per check.
"""
import ctypes

import numpy as np
import pytest
import torch

from actorcritic import _lib

pytestmark = pytest.mark.gpu


def _net(params, A, C3):
    return _lib.Net(A, C3, params.data_ptr())


def _layout(A, C3):
    off = (ctypes.c_int64 * 12)()
    _lib.call('acmi_param_offsets', A, C3, off)
    return list(off), _lib.load().acmi_param_count(A, C3)


def _split(params, A, C3):
    off, n = _layout(A, C3)
    shapes = [(8, 8, 4, 32), (32,), (4, 4, 32, 64), (64,), (3, 3, 64, C3), (C3,), (49 * C3, 512), (512,),
              (512, A), (A,), (512, 1), (1,)]
    ends = off[1:] + [n]
    return [params[o:e].reshape(s) for o, e, s in zip(off, ends, shapes)]


def torch_forward(params, obs_u8, A, C3):
    """float64 CPU reference of envs/atari/model.py:92-217 (NHWC, VALID)."""
    w1, b1, w2, b2, w3, b3, w4, b4, wp, bp, wv, bv = [t.double().cpu() for t in _split(params, A, C3)]
    x = obs_u8.cpu().double() / 255.0
    x = x.permute(0, 3, 1, 2)

    def conv(x, w, b, s):
        return torch.relu(torch.nn.functional.conv2d(x, w.permute(3, 2, 0, 1), b, stride=s))

    a1 = conv(x, w1, b1, 4)
    a2 = conv(a1, w2, b2, 2)
    a3 = conv(a2, w3, b3, 1)
    a3f = a3.permute(0, 2, 3, 1).reshape(x.shape[0], -1)
    a4 = torch.relu(a3f @ w4 + b4)
    logits = a4 @ wp + bp
    value = (a4 @ wv + bv)[:, 0]
    nhwc = lambda t: t.permute(0, 2, 3, 1).contiguous()
    return nhwc(a1), nhwc(a2), a3f, a4, logits, value


def rand_params(A, C3, device, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    n = _lib.load().acmi_param_count(A, C3)
    p = torch.empty(n, dtype=torch.float32)
    off, _ = _layout(A, C3)
    fans = [256, 1, 512, 1, 576, 1, 49 * C3, 1, 512, 1, 512, 1]
    ends = off[1:] + [n]
    for o, e, f in zip(off, ends, fans):
        p[o:e] = torch.randn(e - o, generator=g) * (scale * (2.0 / f) ** 0.5 if f > 1 else 0.1)
    return p.to(device)


def alloc_acts(B, A, C3, device, masks=False):
    z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=device)
    t = dict(a1=z(B, 20, 20, 32), a2=z(B, 9, 9, 64), a3=z(B, 7, 7, C3), a4=z(B, 512), logits=z(B, A),
             value=z(B))
    acts = _lib.Acts(*[t[k].data_ptr() for k in ('a1', 'a2', 'a3', 'a4', 'logits', 'value')], A)
    if masks:  # ReLU' bit masks (acmi_acts_t m1..m3)
        zi = lambda *s: torch.zeros(*s, dtype=torch.int32, device=device)
        t.update(m1=zi(B, 400), m2=zi(B, 162), m3=zi(B, 49 * C3 // 32))
        acts.m1, acts.m2, acts.m3 = t['m1'].data_ptr(), t['m2'].data_ptr(), t['m3'].data_ptr()
    return t, acts


def _relu_bits(a, words):
    """uint32 words of (a > 0), bit e of word e // 32, as int32 [B, words]."""
    b = (a.reshape(a.shape[0], words, 32) > 0).long()
    v = (b << torch.arange(32, device=a.device)).sum(-1)
    return torch.where(v >= 2 ** 31, v - 2 ** 32, v).int()


@pytest.mark.parametrize('use_prep,B', [(True, 300), (True, 5), (False, 300)],
                         ids=['tower', 'split-tower', 'per-layer'])
def test_relu_masks_written_and_bit_identical(lib, cuda, use_prep, B):
    """The ReLU' bit masks (acmi_acts_t m1..m3) written by the forward -- the fused
    tower's ballots (B = 300), the split tower's (B = 5 <= kSplitMaxB: each image
    over 7 workgroups, every mask word written by the part that owns its row) or
    the per-layer path's act_mask_kernel -- equal (a > 0) bit for bit, and the
    backward and output statistics that mask their input gradients from them
    instead of re-reading a1..a3 are bit-identical to the mask-free run."""
    A, C3 = 4, 32
    params = rand_params(A, C3, cuda, seed=41)
    g = torch.Generator().manual_seed(42)
    obs = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.uint8).to(cuda)
    prep = torch.empty(int(lib.acmi_conv_prep_bytes(C3)), dtype=torch.uint8, device=cuda)
    net = _lib.Net(A, C3, params.data_ptr(), prep.data_ptr() if use_prep else None)
    if use_prep:
        _lib.call('acmi_conv_prepare', ctypes.byref(net), _lib.ptr(prep), _lib.stream_handle())
    ldh = 8
    dhead = torch.zeros(B, ldh)
    dhead[:, :A + 1] = torch.randn(B, A + 1, generator=g) / B
    dhead = dhead.to(cuda)
    z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=cuda)
    so = (ctypes.c_int64 * 11)()
    tot = ctypes.c_int64()
    _lib.call('acmi_kfac_layout', A, C3, None, None, so, ctypes.byref(tot))
    ws = z(lib.acmi_backward_ws_floats(B, A, C3))
    out = {}
    for masks in (False, True):
        t, acts = alloc_acts(B, A, C3, cuda, masks=masks)
        _lib.call('acmi_forward', ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts), 1,
                  _lib.stream_handle())
        d = [z(B, 20, 20, 32), z(B, 9, 9, 64), z(B, 7, 7, C3), z(B, 512)]
        bwd = _lib.Bwd(*[x.data_ptr() for x in d], dhead.data_ptr(), ldh)
        grads, astat, gstat = z(params.numel()), z(tot.value), z(tot.value)
        _lib.call('acmi_backward', ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts),
                  ctypes.byref(bwd), _lib.ptr(grads), _lib.ptr(astat), _lib.ptr(ws), ws.numel(), _lib.stream_handle())
        d1 = d[0].clone()
        _lib.call('acmi_kfac_output_stats', ctypes.byref(net), B, ctypes.byref(acts), ctypes.byref(bwd),
                  7, 0, 3, _lib.ptr(gstat), _lib.ptr(ws), ws.numel(), _lib.stream_handle())
        torch.cuda.synchronize()
        if masks:
            for k, words in (('1', 400), ('2', 162), ('3', 49 * C3 // 32)):
                assert torch.equal(t['m' + k], _relu_bits(t['a' + k], words)), k
        out[masks] = (grads.cpu(), astat.cpu(), gstat.cpu(), d1.cpu())
    for a, b in zip(out[False], out[True]):
        assert torch.equal(a, b)


@pytest.mark.parametrize('C3,B', [(32, 24), (64, 640)])
def test_backward_workspace_contract(lib, cuda, C3, B):
    """ws_floats in the ABI (v4): an undersized workspace fails with ACMI_ERR_WS
    before anything is enqueued -- the workspace with a guard region past the
    nominal end, the gradients, the factors and d1..d4 (all NaN-filled) stay
    untouched -- and every legal size gives bit-identical results.  At C3 = 64,
    B = 640 with K-FAC statistics the minimum workspace cannot hold the heads'
    (5.3 M floats) and fc4's (22.9 M) split-K partials side by side (the minimum
    partial region is the largest single plan, 26.6 M), so the backward
    finalizes its deferred set early (acmi_debug_ws_flushes > 0); five times the
    minimum never does.
    Reference: SURVEY 8(b) "workspaces passed in"; the error mapping of
    actorcritic/model.py:180-186."""
    A = 4
    g = torch.Generator().manual_seed(31)
    obs = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.uint8).to(cuda)
    params = rand_params(A, C3, cuda, seed=5)
    prep = torch.empty(int(lib.acmi_conv_prep_bytes(C3)), dtype=torch.uint8, device=cuda)
    net = _lib.Net(A, C3, params.data_ptr(), prep.data_ptr())
    _lib.call('acmi_conv_prepare', ctypes.byref(net), _lib.ptr(prep), _lib.stream_handle())
    ldh = 8
    dhead = torch.zeros(B, ldh)
    dhead[:, :A + 1] = torch.randn(B, A + 1, generator=g) / B
    dhead = dhead.to(cuda)
    so = (ctypes.c_int64 * 11)()
    tot = ctypes.c_int64()
    _lib.call('acmi_kfac_layout', A, C3, None, None, so, ctypes.byref(tot))
    t, acts = alloc_acts(B, A, C3, cuda, masks=True)
    _lib.call('acmi_forward', ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts), 1,
              _lib.stream_handle())
    need = int(lib.acmi_backward_ws_floats(B, A, C3))
    nan = float('nan')
    guard = 4096

    def run(ws_floats, alloc):
        ws = torch.full((alloc,), nan, dtype=torch.float32, device=cuda)
        d = [torch.full(sh, nan, device=cuda) for sh in ((B, 20, 20, 32), (B, 9, 9, 64), (B, 7, 7, C3), (B, 512))]
        bwd = _lib.Bwd(*[x.data_ptr() for x in d], dhead.data_ptr(), ldh)
        grads = torch.full((params.numel(),), nan, device=cuda)
        astat = torch.full((tot.value,), nan, device=cuda)
        gstat = torch.full((tot.value,), nan, device=cuda)
        torch.cuda.synchronize()
        lib.acmi_debug_ws_flushes()
        rc_b = lib.acmi_backward(ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts),
                                 ctypes.byref(bwd), _lib.ptr(grads), _lib.ptr(astat), _lib.ptr(ws), ws_floats,
                                 _lib.stream_handle())
        rc_s = lib.acmi_kfac_output_stats(ctypes.byref(net), B, ctypes.byref(acts), ctypes.byref(bwd), 7, 0, 3,
                                          _lib.ptr(gstat), _lib.ptr(ws), ws_floats, _lib.stream_handle())
        torch.cuda.synchronize()
        return rc_b, rc_s, lib.acmi_debug_ws_flushes(), ws, [grads, astat, gstat] + d

    # undersized by one float: both entry points refuse, nothing is written
    rc_b, rc_s, fl, ws, outs = run(need - 1, need + guard)
    assert rc_b == -3 and rc_s == -3, (rc_b, rc_s)
    assert b'workspace' in lib.acmi_last_error()
    assert fl == 0
    assert torch.isnan(ws).all(), 'an undersized call wrote into its workspace or the guard region'
    for x in outs:
        assert torch.isnan(x).all(), 'an undersized call wrote an output'
    # the minimum and a large workspace: identical bits; nothing past ws_floats
    rc_b, rc_s, fl_min, ws_min, out_min = run(need, need + guard)
    assert rc_b == 0 and rc_s == 0
    assert torch.isnan(ws_min[need:]).all(), 'the backward wrote past ws_floats'
    rc_b, rc_s, fl_big, _, out_big = run(5 * need, 5 * need)
    assert rc_b == 0 and rc_s == 0
    assert fl_big == 0
    if C3 == 64:
        assert fl_min > 0, 'the minimum workspace was expected to finalize the deferred set early'
    # written: grads, the A part of a_stats, the G part of g_stats, d1..d4
    ga = so[5]
    written = [out_min[0], out_min[1][:ga], out_min[2][ga:]] + out_min[3:]
    for a in written:
        assert not torch.isnan(a).any()
    for a, b in zip(out_min, out_big):
        assert torch.equal(torch.isnan(a), torch.isnan(b))
        assert torch.equal(torch.nan_to_num(a), torch.nan_to_num(b))


@pytest.mark.parametrize('B,use_prep,masks', [(700, True, True), (700, True, False), (24, True, True),
                                               (24, False, True)], ids=['700-stacked', '700-stacked-nomask',
                                                                        '24-stacked', '24-no-prep'])
def test_backward_stacked_bit_identical_to_two_calls(lib, cuda, B, use_prep, masks):
    """acmi_backward_stacked + acmi_kfac_output_stats_finish (conv2's input gradient
    of the loss and the sampled-loss chain as ONE launch, convt2_kernel MIX) equal
    acmi_backward + acmi_kfac_output_stats bit for bit: gradients, A and G
    factors, the loss chain's d1..d4 and the sampled chain's d2..d4.  Without
    prepared weights the stacked call runs the two conv2 launches itself.
    Reference: objectives.py:78-79, policies.py:157-158 (the two graphs)."""
    A, C3 = 4, 32
    g = torch.Generator().manual_seed(41)
    obs = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.uint8).to(cuda)
    params = rand_params(A, C3, cuda, seed=6)
    prep = torch.empty(int(lib.acmi_conv_prep_bytes(C3)), dtype=torch.uint8, device=cuda)
    net = _lib.Net(A, C3, params.data_ptr(), prep.data_ptr() if use_prep else None)
    if use_prep:
        _lib.call('acmi_conv_prepare', ctypes.byref(net), _lib.ptr(prep), _lib.stream_handle())
    ldh = 8
    dhead = torch.zeros(B, ldh)
    dhead[:, :A + 1] = torch.randn(B, A + 1, generator=g) / B
    dhead = dhead.to(cuda)
    so = (ctypes.c_int64 * 11)()
    tot = ctypes.c_int64()
    _lib.call('acmi_kfac_layout', A, C3, None, None, so, ctypes.byref(tot))
    t, acts = alloc_acts(B, A, C3, cuda, masks=masks)
    _lib.call('acmi_forward', ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts), 1,
              _lib.stream_handle())
    need = int(lib.acmi_backward_ws_floats(B, A, C3))
    z = lambda *sh: torch.zeros(*sh, dtype=torch.float32, device=cuda)

    def dbufs():
        d = [z(B, 20, 20, 32), z(B, 9, 9, 64), z(B, 7, 7, C3), z(B, 512)]
        return d, _lib.Bwd(*[x.data_ptr() for x in d], dhead.data_ptr(), ldh)

    out = {}
    for stacked in (False, True):
        d, bwd = dbufs()
        ds, bwd_s = dbufs()
        ws, ws_s = z(need), z(need)
        grads, stats = z(params.numel()), z(tot.value)
        if stacked:
            _lib.call('acmi_backward_stacked', ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts),
                      ctypes.byref(bwd), _lib.ptr(grads), _lib.ptr(stats), _lib.ptr(ws), need, ctypes.byref(bwd_s), 7,
                      0, 3, _lib.ptr(ws_s), need, _lib.stream_handle())
            _lib.call('acmi_kfac_output_stats_finish', ctypes.byref(net), B, ctypes.byref(acts), ctypes.byref(bwd_s),
                      _lib.ptr(stats), _lib.ptr(ws_s), need, _lib.stream_handle())
        else:
            _lib.call('acmi_backward', ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts),
                      ctypes.byref(bwd), _lib.ptr(grads), _lib.ptr(stats), _lib.ptr(ws), need, _lib.stream_handle())
            _lib.call('acmi_kfac_output_stats', ctypes.byref(net), B, ctypes.byref(acts), ctypes.byref(bwd_s), 7, 0,
                      3, _lib.ptr(stats), _lib.ptr(ws_s), need, _lib.stream_handle())
        torch.cuda.synchronize()
        out[stacked] = [grads, stats] + d + ds[1:]
    assert out[True][1].abs().sum() > 0
    for i, (a, b) in enumerate(zip(out[False], out[True])):
        assert torch.equal(a, b), i


def test_per_net_modes_override_the_process_default(lib, cuda):
    """acmi_net_t's mode fields (mode + 1; 0 = the process default): a net carrying
    ACMI_FWD_BF16 computes under an f32 process default exactly what the bf16
    process default computes, and the reverse; an invalid combination (bf16
    forward in f32 gemm mode) is refused.  (The modes are held per calling thread
    for the call, so nets in one process do not see each other's settings.)"""
    A, C3, B = 4, 32, 40
    g = torch.Generator().manual_seed(9)
    obs = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.uint8).to(cuda)
    params = rand_params(A, C3, cuda, seed=12)
    prep = torch.empty(int(lib.acmi_conv_prep_bytes(C3)), dtype=torch.uint8, device=cuda)

    def fwd(process_mode, net_field):
        prev = lib.acmi_get_forward_mode()
        _lib.call('acmi_set_forward_mode', process_mode)
        try:
            net = _lib.Net(A, C3, params.data_ptr(), prep.data_ptr(), 0, net_field, 0)
            _lib.call('acmi_conv_prepare', ctypes.byref(net), _lib.ptr(prep), _lib.stream_handle())
            t, acts = alloc_acts(B, A, C3, cuda, masks=True)
            _lib.call('acmi_forward', ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts), 1,
                      _lib.stream_handle())
            torch.cuda.synchronize()
            return [t[k].clone() for k in ('a1', 'a2', 'a3', 'logits', 'm1')]
        finally:
            _lib.call('acmi_set_forward_mode', prev)

    f32_default = fwd(_lib.FWD_F32, 0)
    bf16_default = fwd(_lib.FWD_BF16, 0)
    assert not torch.equal(f32_default[0], bf16_default[0])
    for a, b in zip(fwd(_lib.FWD_F32, _lib.FWD_BF16 + 1), bf16_default):
        assert torch.equal(a, b)
    for a, b in zip(fwd(_lib.FWD_BF16, _lib.FWD_F32 + 1), f32_default):
        assert torch.equal(a, b)
    bad = _lib.Net(A, C3, params.data_ptr(), prep.data_ptr(), _lib.GEMM_F32 + 1, _lib.FWD_BF16 + 1, 0)
    t, acts = alloc_acts(B, A, C3, cuda)
    assert lib.acmi_forward(ctypes.byref(bad), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts), 1,
                            _lib.stream_handle()) == -1
    assert b'mode' in lib.acmi_last_error()


def test_per_net_modes_hold_across_concurrent_threads(lib, cuda):
    """Two host threads call acmi_conv_prepare + acmi_forward at the same time, 25 times
    each, on their own HIP streams, one net carrying the bf16 forward and one the f32
    forward (process default f32): every output equals the single-threaded run of the
    same net bit for bit -- the per-call modes are held per thread (net.hip ModeScope),
    so concurrent calls with different nets do not see each other's settings (ctypes
    releases the GIL around each foreign call, so the calls overlap in the library)."""
    import threading
    A, C3, B = 4, 32, 40
    g = torch.Generator().manual_seed(21)
    obs = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.uint8).to(cuda)
    params = rand_params(A, C3, cuda, seed=22)
    torch.cuda.synchronize()  # the threads' streams do not wait on the default stream
    modes = (_lib.FWD_BF16 + 1, _lib.FWD_F32 + 1)

    def run(mode, stream, reps, out, errors, start=None):
        try:
            with torch.cuda.stream(stream):
                prep = torch.empty(int(lib.acmi_conv_prep_bytes(C3)), dtype=torch.uint8, device=cuda)
                net = _lib.Net(A, C3, params.data_ptr(), prep.data_ptr(), 0, mode, 0)
                t, acts = alloc_acts(B, A, C3, cuda, masks=True)
            h = ctypes.c_void_p(stream.cuda_stream)
            if start is not None:
                start.wait()
            for _ in range(reps):
                _lib.call('acmi_conv_prepare', ctypes.byref(net), _lib.ptr(prep), h)
                _lib.call('acmi_forward', ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts), 1, h)
            stream.synchronize()
            out.append([t[k].clone() for k in ('a1', 'a2', 'a3', 'logits', 'value', 'm1')])
        except Exception as e:  # surfaced by the main thread
            errors.append(e)

    refs = []
    for mode in modes:
        out, errors = [], []
        run(mode, torch.cuda.Stream(), 1, out, errors)
        assert not errors, errors
        refs.append(out[0])
    assert not torch.equal(refs[0][0], refs[1][0])  # the two modes really differ
    outs, errors = [[], []], []
    start = threading.Barrier(2)
    threads = [threading.Thread(target=run, args=(m, torch.cuda.Stream(), 25, outs[i], errors, start))
               for i, m in enumerate(modes)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not errors, errors
    for i in range(2):
        assert len(outs[i]) == 1
        for a, b in zip(outs[i][0], refs[i]):
            assert torch.equal(a, b)


@pytest.mark.parametrize('C3', [32, 64])
@pytest.mark.parametrize('fwd', ['f32', 'bf16'])
def test_split_tower_bit_identical_to_one_block_tower(lib, cuda, C3, fwd):
    """The small-batch split tower (towersplit.hpp: B <= kSplitMaxB = 64, each image
    over 7 workgroups) equals the one-block tower (tower.hpp) bit for bit -- a1..a3
    and the ReLU' words m1..m3 of the same images, once as a 5-image batch and once
    inside a 70-image batch -- in both forward modes and at both conv3 widths: every
    output pixel runs the same MFMA chain over the same K partition (conv1 pixels
    384..399, conv2 pixels 64..80 and conv3 at C3 = 32 as two K halves)."""
    A, B = 4, 5
    prev = lib.acmi_get_forward_mode()
    _lib.call('acmi_set_forward_mode', _lib.FWD_BF16 if fwd == 'bf16' else _lib.FWD_F32)
    try:
        params = rand_params(A, C3, cuda, seed=71)
        g = torch.Generator().manual_seed(72)
        big = torch.randint(0, 256, (70, 84, 84, 4), generator=g, dtype=torch.uint8).to(cuda)
        prep = torch.empty(int(lib.acmi_conv_prep_bytes(C3)), dtype=torch.uint8, device=cuda)
        net = _lib.Net(A, C3, params.data_ptr(), prep.data_ptr())
        _lib.call('acmi_conv_prepare', ctypes.byref(net), _lib.ptr(prep), _lib.stream_handle())
        out = []
        for obs in (big[17:17 + B].contiguous(), big):
            t, acts = alloc_acts(obs.shape[0], A, C3, cuda, masks=True)
            ws = torch.zeros(int(lib.acmi_forward_ws_floats(obs.shape[0])), device=cuda)
            acts.ws, acts.ws_floats = ws.data_ptr(), ws.numel()
            _lib.call('acmi_forward', ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, obs.shape[0],
                      ctypes.byref(acts), 1, _lib.stream_handle())
            torch.cuda.synchronize()
            out.append(t)
        for k in ('a1', 'a2', 'a3', 'm1', 'm2', 'm3'):
            assert torch.equal(out[0][k], out[1][k][17:17 + B]), k
        assert torch.equal(out[1]['m2'], _relu_bits(out[1]['a2'], 162))
    finally:
        _lib.call('acmi_set_forward_mode', prev)


@pytest.mark.parametrize('C3', [32, 64])
def test_conv3_dx_prepared_weights_bit_identical(lib, cuda, C3):
    """conv3's input gradient (convt3.hpp) on W3 fragments pre-split by
    acmi_conv_prepare equals the variant that stages and splits the f32 weights
    per block, bit for bit (same scale of max |W3|, same fragments, same MFMA
    order): d3 and d2 of one backward with and without net->conv_prep, on the
    same forward activations and head gradients."""
    A, B = 4, 300
    params = rand_params(A, C3, cuda, seed=61)
    g = torch.Generator().manual_seed(62)
    obs = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.uint8).to(cuda)
    prep = torch.empty(int(lib.acmi_conv_prep_bytes(C3)), dtype=torch.uint8, device=cuda)
    net_p = _lib.Net(A, C3, params.data_ptr(), prep.data_ptr())
    net_n = _lib.Net(A, C3, params.data_ptr(), None)
    _lib.call('acmi_conv_prepare', ctypes.byref(net_p), _lib.ptr(prep), _lib.stream_handle())
    ldh = 8
    dhead = torch.zeros(B, ldh)
    dhead[:, :A + 1] = torch.randn(B, A + 1, generator=g) / B
    dhead = dhead.to(cuda)
    z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=cuda)
    ws = z(lib.acmi_backward_ws_floats(B, A, C3))
    t, acts = alloc_acts(B, A, C3, cuda, masks=True)
    _lib.call('acmi_forward', ctypes.byref(net_p), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts), 1,
              _lib.stream_handle())
    out = []
    for net in (net_p, net_n):
        d = [z(B, 20, 20, 32), z(B, 9, 9, 64), z(B, 7, 7, C3), z(B, 512)]
        bwd = _lib.Bwd(*[x.data_ptr() for x in d], dhead.data_ptr(), ldh)
        grads = z(params.numel())
        _lib.call('acmi_backward', ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts),
                  ctypes.byref(bwd), _lib.ptr(grads), None, _lib.ptr(ws), ws.numel(), _lib.stream_handle())
        torch.cuda.synchronize()
        out.append((d[2].cpu(), d[1].cpu()))
    assert out[0][1].abs().max() > 0
    assert torch.equal(out[0][0], out[1][0]), 'd3'
    assert torch.equal(out[0][1], out[1][1]), 'd2'


@pytest.mark.parametrize('M,N,K', [(128, 128, 32), (300, 260, 200), (1, 4, 4), (1000, 64, 1568)])
def test_gemm_f32(lib, cuda, M, N, K):
    g = torch.Generator().manual_seed(1)
    a = torch.randn(M, K, generator=g)
    b = torch.randn(K, N, generator=g)
    c = torch.zeros(M, N, device=cuda)
    a_d, b_d = a.to(cuda), b.to(cuda)  # keep device copies alive until the kernel has run
    _lib.call('acmi_gemm_f32', _lib.ptr(a_d), _lib.ptr(b_d), _lib.ptr(c), M, N, K, _lib.stream_handle())
    torch.cuda.synchronize()
    ref = a.double() @ b.double()
    err = (c.cpu().double() - ref).abs().max().item()
    # exact-f32 fmaf chain: error ~ K * eps * max|a||b|
    assert err <= 2e-6 * K * ref.abs().max().item() / max(1.0, K ** 0.5), err


@pytest.mark.parametrize('A,C3,B', [(4, 32, 3), (18, 64, 5), (4, 32, 67)])
def test_forward_matches_torch(lib, cuda, A, C3, B):
    params = rand_params(A, C3, cuda)
    g = torch.Generator().manual_seed(2)
    obs = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.uint8)
    t, acts = alloc_acts(B, A, C3, cuda)
    net = _net(params, A, C3)
    obs_d = obs.to(cuda)
    _lib.call('acmi_forward', ctypes.byref(net), _lib.ptr(obs_d), 84 * 84 * 4, B, ctypes.byref(acts), 1,
              _lib.stream_handle())
    torch.cuda.synchronize()
    ref = torch_forward(params, obs, A, C3)
    names = ['a1', 'a2', 'a3', 'a4', 'logits', 'value']
    for name, r in zip(names, ref):
        got = t[name].cpu().double().reshape(r.shape)
        rel = (got - r).abs().max().item() / max(1e-6, r.abs().max().item())
        assert rel < 1e-5, (name, rel)


def _backward_errors(lib, cuda, B=6, seed=3):
    """max relative errors of acmi_backward's parameter gradients and A factors
    against float64 autograd / patch products"""
    errs = {}
    A, C3 = 4, 32
    params = rand_params(A, C3, cuda, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
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
    n = params.numel()
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
    torch.cuda.synchronize()
    # reference gradients by autograd in float64
    p64 = params.cpu().double().requires_grad_(True)
    a1, a2, a3f, a4, logits, value = torch_forward(p64, obs, A, C3)
    loss = (logits * dhead[:, :A].double()).sum() + (value * dhead[:, A].double()).sum()
    loss.backward()
    ref = p64.grad
    got = grads.cpu().double()
    off, _ = _layout(A, C3)
    ends = off[1:] + [n]
    for i, (o, e) in enumerate(zip(off, ends)):
        r = ref[o:e]
        errs[('param block', i)] = (got[o:e] - r).abs().max().item() / max(1e-12, r.abs().max().item())
    # A factors: mean over rows of [x;1][x;1]^T
    x = obs.double() / 255.0

    def patches(x, k, s):
        p = x.unfold(1, k, s).unfold(2, k, s)  # B, OH, OW, C, KH, KW
        return p.permute(0, 1, 2, 4, 5, 3).reshape(-1, k * k * x.shape[-1])

    ins = [patches(x, 8, 4), patches(a1.detach(), 4, 2), patches(a2.detach(), 3, 1), a3f.detach(), a4.detach()]
    a_host = astat.cpu().double()
    for f, xin in enumerate(ins):
        xb = torch.cat([xin, torch.ones(xin.shape[0], 1, dtype=xin.dtype)], 1)
        r = xb.t() @ xb / xb.shape[0]
        got_f = a_host[so[f]:so[f] + din[f] * din[f]].reshape(din[f], din[f])
        errs[('A factor', f)] = (got_f - r).abs().max().item() / r.abs().max().item()
    return errs


def _with_mode(lib, mode, fn, *a, **k):
    prev = lib.acmi_get_gemm_mode()
    _lib.call('acmi_set_gemm_mode', mode)
    try:
        return fn(*a, **k)
    finally:
        _lib.call('acmi_set_gemm_mode', prev)


def test_backward_and_astats_match_torch(lib, cuda):
    for key, rel in _backward_errors(lib, cuda).items():
        assert rel < 2e-5, (key, rel)


def test_x3_gemms_are_f32_class(lib, cuda):
    """The bf16x3 split-operand GEMMs (symred3.hpp, gemm3.hpp) are f32-class:
    against float64, every gradient block and A factor of the backward (whose
    conv input-gradient chain runs on gemm3) is within 5e-6 relative (the section 5
    gradient tolerance is 2e-5), within 10x of the v_mfma_f32_32x32x2_f32 path's
    error on the same inputs (floored at 5e-7, its typical gradient-block error),
    and the median block is within 3x.  Measured: A factors 0.8-1.3x; gradient
    blocks mostly 1-6x; the worst is the conv1 bias (3.5e-6 vs 4.2e-7), a plain
    sum of d1 over all conv1 locations whose cancellation magnifies d1's relative error
    (each 16-k step of the conv2 input gradient rounds six partial products into
    the accumulator)."""
    ex3 = _with_mode(lib, _lib.GEMM_X3, _backward_errors, lib, cuda, B=32, seed=21)
    ef32 = _with_mode(lib, _lib.GEMM_F32, _backward_errors, lib, cuda, B=32, seed=21)
    for key in ef32:
        print(key, 'x3 %.3g  f32 %.3g' % (ex3[key], ef32[key]))
    for key in ef32:
        assert ex3[key] <= 5e-6 and ex3[key] <= 10 * max(ef32[key], 5e-7), (key, ex3[key], ef32[key])
    ratios = sorted(ex3[k] / max(ef32[k], 5e-7) for k in ef32)
    assert ratios[len(ratios) // 2] <= 3.0, ratios


def _with_conv_stats(lib, mode, fn, *a, **k):
    prev = lib.acmi_get_conv_stats_mode()
    _lib.call('acmi_set_conv_stats_mode', mode)
    try:
        return fn(*a, **k)
    finally:
        _lib.call('acmi_set_conv_stats_mode', prev)


def test_band_conv_stats_match_float64(lib, cuda):
    """conv2 / conv3 weight gradients and A factors from the pixel-pair band
    reduction (band.hpp) vs float64 and vs the patch-row reduction: the same
    sums reassociated, so f32-class (<= 5e-6 relative) and within 10x of the
    patch path's error (floored at 5e-7)."""
    eb = _with_conv_stats(lib, _lib.CONV_STATS_BAND, _backward_errors, lib, cuda, B=24, seed=5)
    ep = _with_conv_stats(lib, _lib.CONV_STATS_PATCHES, _backward_errors, lib, cuda, B=24, seed=5)
    for key in ep:
        print(key, 'band %.3g  patches %.3g' % (eb[key], ep[key]))
    for key in ep:
        assert eb[key] <= 5e-6 and eb[key] <= 10 * max(ep[key], 5e-7), (key, eb[key], ep[key])


def _band_backward(lib, cuda, B, mode, reps=1, seed=8):
    """(grads, A-factor stats) of acmi_backward in conv-stats `mode`, `reps` times"""
    A, C3 = 4, 32
    params = rand_params(A, C3, cuda, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    obs = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.uint8).to(cuda)
    t, acts = alloc_acts(B, A, C3, cuda)
    net = _net(params, A, C3)
    _lib.call('acmi_forward', ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts), 1,
              _lib.stream_handle())
    ldh = 8
    dhead = torch.zeros(B, ldh)
    dhead[:, :A + 1] = torch.randn(B, A + 1, generator=g) / B
    dhead = dhead.to(cuda)
    z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=cuda)
    d = [z(B, 20, 20, 32), z(B, 9, 9, 64), z(B, 7, 7, C3), z(B, 512)]
    bwd = _lib.Bwd(*[x.data_ptr() for x in d], dhead.data_ptr(), ldh)
    din = (ctypes.c_int64 * 6)()
    so = (ctypes.c_int64 * 11)()
    tot = ctypes.c_int64()
    _lib.call('acmi_kfac_layout', A, C3, din, None, so, ctypes.byref(tot))
    ws = z(lib.acmi_backward_ws_floats(B, A, C3))
    outs = []
    for _ in range(reps):
        grads, astat = z(params.numel()), z(tot.value)
        _with_conv_stats(lib, mode, _lib.call, 'acmi_backward', ctypes.byref(net), _lib.ptr(obs),
                         84 * 84 * 4, B, ctypes.byref(acts), ctypes.byref(bwd), _lib.ptr(grads), _lib.ptr(astat),
                         _lib.ptr(ws), ws.numel(), _lib.stream_handle())
        torch.cuda.synchronize()
        outs.append((grads.cpu(), astat.cpu()))
    return outs, list(din), list(so), _layout(A, C3)[0]


def test_band_chunked_matches_patch_rows(lib, cuda):
    """At B = 1100 images the band reduction splits the images into chunks
    (per-chunk partials, in-order chunk reduction): conv2 / conv3 gradient blocks
    and A factors agree with the patch-row reduction to f32 accuracy."""
    B = 1100
    info = (ctypes.c_int64 * 5)()
    _lib.call('acmi_band_info', 1, 32, B, info)
    assert info[2] >= 2, list(info)
    (ob,), din, so, off = _band_backward(lib, cuda, B, _lib.CONV_STATS_BAND)
    (op,), _, _, _ = _band_backward(lib, cuda, B, _lib.CONV_STATS_PATCHES)
    for blk in (2, 3, 4, 5):  # conv2 W, b, conv3 W, b
        a, b = ob[0][off[blk]:off[blk + 1]].double(), op[0][off[blk]:off[blk + 1]].double()
        rel = (a - b).abs().max().item() / b.abs().max().item()
        assert rel < 1e-5, (blk, rel)
    for f in (1, 2):
        a = ob[1][so[f]:so[f] + din[f] * din[f]].double()
        b = op[1][so[f]:so[f] + din[f] * din[f]].double()
        rel = (a - b).abs().max().item() / b.abs().max().item()
        assert rel < 1e-5, (f, rel)


def test_band_backward_deterministic_and_symmetric(lib, cuda):
    """Two band backwards on the same inputs are bit-identical, and the band A
    factors are exactly symmetric (the upper triangle is mirrored)."""
    outs, din, so, _ = _band_backward(lib, cuda, 1100, _lib.CONV_STATS_BAND, reps=2)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    for f in (1, 2):
        F = outs[0][1][so[f]:so[f] + din[f] * din[f]].reshape(din[f], din[f])
        assert torch.equal(F, F.t()), f


def test_kfac_inverse_badly_conditioned(lib, cuda):
    """The pair sweep (two pivots per sweep, each 2 x 2 pivot block inverted in
    closed form, kfac.hip pivot_inverse) on damped factors of condition ~1e7:
    eigenvalues logspace(-9, 1) in a random basis, damping 1e-12 (sqrt 1e-6).
    Every 2 x 2 Schur-complement block of such an SPD matrix is SPD, and the fp64
    sweep keeps f32-output accuracy (max-abs error 1e-4 of max-abs value against
    numpy's float64 inverse of the same f32 factors)."""
    A, C3 = 4, 32
    din = (ctypes.c_int64 * 6)()
    dout = (ctypes.c_int64 * 6)()
    so = (ctypes.c_int64 * 11)()
    tot = ctypes.c_int64()
    _lib.call('acmi_kfac_layout', A, C3, din, dout, so, ctypes.byref(tot))
    rng = np.random.default_rng(17)
    fac = np.zeros(tot.value, np.float32)
    mats = []
    for f in range(11):
        n = din[f] if f < 5 else dout[f - 5]
        q, _ = np.linalg.qr(rng.standard_normal((n, n)))
        m = (q * np.logspace(-9, 1, n)) @ q.T
        m = ((m + m.T) / 2).astype(np.float32)
        fac[so[f]:so[f] + n * n] = m.ravel()
        mats.append(m.astype(np.float64))
    fac_d = torch.from_numpy(fac).to(cuda)
    inv = torch.zeros(lib.acmi_kfac_inverse_floats(A, C3), device=cuda)
    ws = torch.zeros(lib.acmi_kfac_inverse_ws_doubles(A, C3), dtype=torch.float64, device=cuda)
    damping = 1e-12
    _lib.call('acmi_kfac_inverse', A, C3, _lib.ptr(fac_d), ctypes.c_float(damping), 0, _lib.ptr(inv), _lib.ptr(ws),
              _lib.stream_handle())
    torch.cuda.synchronize()
    inv_h = inv.cpu().numpy().astype(np.float64)
    assert np.isfinite(inv_h).all()
    ioff = (ctypes.c_int64 * 12)()
    ild = (ctypes.c_int64 * 12)()
    _lib.call('acmi_kfac_inverse_layout', A, C3, ioff, ild)
    for l in range(6):
        Am, Gm = mats[min(l, 4)], mats[5 + l]
        da, dg = Am.shape[0], Gm.shape[0]
        lam = np.float64(np.float32(damping))
        pi = np.sqrt((np.trace(Am) / da) / (np.trace(Gm) / dg))
        for m, M, add in ((2 * l, Am, pi * np.sqrt(lam)), (2 * l + 1, Gm, np.sqrt(lam) / pi)):
            n = M.shape[0]
            ref = np.linalg.inv(M + add * np.eye(n))
            got = inv_h[ioff[m]:ioff[m] + n * ild[m]].reshape(n, ild[m])[:, :n]
            rel = np.abs(got - ref).max() / np.abs(ref).max()
            print('layer', l, 'AG'[m % 2], 'cond %.1e' % np.linalg.cond(M + add * np.eye(n)), 'rel %.2e' % rel)
            assert rel < 1e-4, (l, m % 2, rel)


def test_kfac_inverse_matches_numpy(lib, cuda):
    A, C3 = 4, 32
    din = (ctypes.c_int64 * 6)()
    dout = (ctypes.c_int64 * 6)()
    so = (ctypes.c_int64 * 11)()
    tot = ctypes.c_int64()
    _lib.call('acmi_kfac_layout', A, C3, din, dout, so, ctypes.byref(tot))
    rng = np.random.default_rng(5)
    fac = np.zeros(tot.value, np.float32)
    mats = []
    for f in range(11):
        n = din[f] if f < 5 else dout[f - 5]
        x = rng.standard_normal((max(n // 2, 1) + 3, n)).astype(np.float64)
        m = (x.T @ x / x.shape[0]).astype(np.float32)
        fac[so[f]:so[f] + n * n] = m.ravel()
        mats.append(m.astype(np.float64))
    fac_d = torch.from_numpy(fac).to(cuda)
    inv = torch.zeros(lib.acmi_kfac_inverse_floats(A, C3), device=cuda)
    ws = torch.zeros(lib.acmi_kfac_inverse_ws_doubles(A, C3), dtype=torch.float64, device=cuda)
    damping = 0.01
    _lib.call('acmi_kfac_inverse', A, C3, _lib.ptr(fac_d), ctypes.c_float(damping), 0, _lib.ptr(inv), _lib.ptr(ws),
              _lib.stream_handle())
    torch.cuda.synchronize()
    inv_h = inv.cpu().numpy().astype(np.float64)
    ioff = (ctypes.c_int64 * 12)()
    ild = (ctypes.c_int64 * 12)()
    _lib.call('acmi_kfac_inverse_layout', A, C3, ioff, ild)

    def block(m, n):
        o, ld = ioff[m], ild[m]
        b = inv_h[o:o + n * ld].reshape(n, ld)
        assert ld % 4 == 0 and ld >= n and not b[:, n:].any(), 'padding columns must be zero'
        return b[:, :n]

    for l in range(6):
        af = min(l, 4)
        Am, Gm = mats[af], mats[5 + l]
        da, dg = Am.shape[0], Gm.shape[0]
        pi = np.sqrt((np.trace(Am) / da) / (np.trace(Gm) / dg))
        ref_a = np.linalg.inv(Am + pi * np.sqrt(damping) * np.eye(da))
        ref_g = np.linalg.inv(Gm + np.sqrt(damping) / pi * np.eye(dg))
        got_a = block(2 * l, da)
        got_g = block(2 * l + 1, dg)
        for got, ref in ((got_a, ref_a), (got_g, ref_g)):
            rel = np.abs(got - ref).max() / np.abs(ref).max()
            assert rel < 1e-5, (l, rel)


def test_kfac_eigvals_match_numpy(lib, cuda):
    A, C3 = 4, 32
    din = (ctypes.c_int64 * 6)()
    dout = (ctypes.c_int64 * 6)()
    so = (ctypes.c_int64 * 11)()
    tot = ctypes.c_int64()
    _lib.call('acmi_kfac_layout', A, C3, din, dout, so, ctypes.byref(tot))
    rng = np.random.default_rng(6)
    fac = np.zeros(tot.value, np.float32)
    mats = []
    for f in range(11):
        n = din[f] if f < 5 else dout[f - 5]
        x = rng.standard_normal((n + 5, n))
        m = (x.T @ x / x.shape[0]).astype(np.float32)
        fac[so[f]:so[f] + n * n] = m.ravel()
        mats.append(m.astype(np.float64))
    fac_d = torch.from_numpy(fac).to(cuda)
    nev = sum(m.shape[0] for m in mats)
    ev = torch.zeros(nev, dtype=torch.float64, device=cuda)
    ws = torch.zeros(lib.acmi_kfac_eig_ws_doubles(A, C3), dtype=torch.float64, device=cuda)
    _lib.call('acmi_kfac_eigvals', A, C3, _lib.ptr(fac_d), _lib.ptr(ev), _lib.ptr(ws), _lib.stream_handle())
    got = ev.cpu().numpy()
    o = 0
    for m in mats:
        n = m.shape[0]
        ref = np.linalg.eigvalsh(0.5 * (m + m.T))
        rel = np.abs(got[o:o + n] - ref).max() / np.abs(ref).max()
        assert rel < 1e-10, rel
        # north_star: eigenvalues within 1e-4 relative (each eigenvalue)
        assert np.all(np.abs(got[o:o + n] - ref) <= 1e-4 * np.abs(ref) + 1e-12 * np.abs(ref).max())
        o += n


@pytest.mark.parametrize('C3', [32, 64])
def test_conv_prep_tower_matches_layer_kernels(lib, cuda, C3):
    """The fused conv tower on acmi_conv_prepare's f16x2 fragments (tower.hpp) and
    the per-layer kernels a net without conv_prep runs agree to f32 accuracy: every
    activation within 4e-6 of the other relative to its range (the value head,
    a 512-term sum, measured 2.1e-6), both within 1e-5 of the float64 forward."""
    A, B = 4, 37
    params = rand_params(A, C3, cuda, seed=4)
    obs = torch.randint(0, 256, (B, 84, 84, 4), generator=torch.Generator().manual_seed(6),
                        dtype=torch.uint8).to(cuda)
    prep = torch.empty(int(lib.acmi_conv_prep_bytes(C3)), dtype=torch.uint8, device=cuda)
    outs = []
    for use_prep in (False, True):
        t, acts = alloc_acts(B, A, C3, cuda)
        net = _lib.Net(A, C3, params.data_ptr(), prep.data_ptr() if use_prep else None)
        if use_prep:
            _lib.call('acmi_conv_prepare', ctypes.byref(net), _lib.ptr(prep), _lib.stream_handle())
        _lib.call('acmi_forward', ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts), 1,
                  _lib.stream_handle())
        torch.cuda.synchronize()
        outs.append({k: v.cpu() for k, v in t.items()})
    rel = lambda x, y: ((x.double() - y.double()).abs().max() / max(1e-6, y.double().abs().max())).item()
    for k in outs[0]:
        assert rel(outs[1][k], outs[0][k]) < 4e-6, (k, rel(outs[1][k], outs[0][k]))
    ref = torch_forward(params, obs.cpu(), A, C3)
    for name, r in zip(['a1', 'a2', 'a3', 'a4', 'logits', 'value'], ref):
        for o in outs:
            assert rel(o[name].reshape(r.shape), r) < 1e-5, name


@pytest.mark.parametrize('C3,B', [(32, 37), (32, 512), (64, 512)])
def test_fc4_rollout_matches_gemm3(lib, cuda, C3, B):
    """fc4's split-K slabs at rollout batches on the pre-split f16x2 W4
    (fc4roll.hpp, used when the net carries conv_prep and a forward workspace)
    agree with the staged bf16x3 gemm3 split-K launch to f32 accuracy (2e-6 of
    each tensor's range), and the forward matches float64 within 1e-5."""
    A = 4
    params = rand_params(A, C3, cuda, seed=21)
    obs = torch.randint(0, 256, (B, 84, 84, 4), generator=torch.Generator().manual_seed(22),
                        dtype=torch.uint8).to(cuda)
    prep = torch.empty(int(lib.acmi_conv_prep_bytes(C3)), dtype=torch.uint8, device=cuda)
    ws = torch.zeros(int(lib.acmi_forward_ws_floats(B)), device=cuda)
    outs = []
    for use_prep in (False, True):
        t, acts = alloc_acts(B, A, C3, cuda)
        acts.ws, acts.ws_floats = ws.data_ptr(), ws.numel()
        net = _lib.Net(A, C3, params.data_ptr(), prep.data_ptr() if use_prep else None)
        if use_prep:
            _lib.call('acmi_conv_prepare', ctypes.byref(net), _lib.ptr(prep), _lib.stream_handle())
        _lib.call('acmi_forward', ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts), 1,
                  _lib.stream_handle())
        torch.cuda.synchronize()
        outs.append({k: v.cpu() for k, v in t.items()})
    for k in ('a4', 'logits', 'value'):
        d = ((outs[1][k].double() - outs[0][k].double()).abs().max() / outs[0][k].double().abs().max()).item()
        assert d < 2e-6, (k, d)
    ref = torch_forward(params, obs.cpu(), A, C3)
    for name, r in zip(['a1', 'a2', 'a3', 'a4', 'logits', 'value'], ref):
        got = outs[1][name].double().reshape(r.shape)
        rel = (got - r).abs().max().item() / max(1e-6, r.abs().max().item())
        assert rel < 1e-5, (name, rel)


@pytest.mark.parametrize('B', [37, 1000])
def test_convt2_matches_gemm3_path(lib, cuda, B):
    """conv2's input gradient on pre-split f16x2 weights (convt2.hpp, used when the
    net carries conv_prep) agrees with the bf16x3 gemm3 path to f32 accuracy (both
    are f32-class: d1 within 2e-6 of each other relative to max |d1|), so do the
    parameter gradients and A factors of the whole backward (2e-6), and the
    sampled-loss chain's conv1 G factor -- reduced from the masked d1 tiles inside
    the kernel instead of stored and re-read -- is within 2e-6 of float64
    d1^T d1 / rows over the stored d1 (B = 1000: some blocks of the Gram grid take
    two column tiles)."""
    A, C3 = 4, 32
    params = rand_params(A, C3, cuda, seed=12)
    g = torch.Generator().manual_seed(13)
    obs = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.uint8).to(cuda)
    t, acts = alloc_acts(B, A, C3, cuda)
    prep = torch.empty(int(lib.acmi_conv_prep_bytes(C3)), dtype=torch.uint8, device=cuda)
    nets = {False: _lib.Net(A, C3, params.data_ptr(), None), True: _lib.Net(A, C3, params.data_ptr(), prep.data_ptr())}
    _lib.call('acmi_conv_prepare', ctypes.byref(nets[True]), _lib.ptr(prep), _lib.stream_handle())
    _lib.call('acmi_forward', ctypes.byref(nets[False]), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts), 1,
              _lib.stream_handle())
    ldh = 8
    dhead = torch.zeros(B, ldh)
    dhead[:, :A + 1] = torch.randn(B, A + 1, generator=g) / B
    dhead = dhead.to(cuda)
    z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=cuda)
    din = (ctypes.c_int64 * 6)()
    so = (ctypes.c_int64 * 11)()
    tot = ctypes.c_int64()
    _lib.call('acmi_kfac_layout', A, C3, din, None, so, ctypes.byref(tot))
    ws = z(lib.acmi_backward_ws_floats(B, A, C3))
    out = {}
    for use_prep in (False, True):
        d = [z(B, 20, 20, 32), z(B, 9, 9, 64), z(B, 7, 7, C3), z(B, 512)]
        bwd = _lib.Bwd(*[x.data_ptr() for x in d], dhead.data_ptr(), ldh)
        grads, astat = z(params.numel()), z(tot.value)
        _lib.call('acmi_backward', ctypes.byref(nets[use_prep]), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts),
                  ctypes.byref(bwd), _lib.ptr(grads), _lib.ptr(astat), _lib.ptr(ws), ws.numel(), _lib.stream_handle())
        torch.cuda.synchronize()
        d1_loss = d[0].clone()
        ds = [z(B, 20, 20, 32), z(B, 9, 9, 64), z(B, 7, 7, C3), z(B, 512)]
        bwd_s = _lib.Bwd(*[x.data_ptr() for x in ds], dhead.data_ptr(), ldh)
        gstat = z(tot.value)
        _lib.call('acmi_kfac_output_stats', ctypes.byref(nets[use_prep]), B, ctypes.byref(acts), ctypes.byref(bwd_s),
                  7, 0, 3, _lib.ptr(gstat), _lib.ptr(ws), ws.numel(), _lib.stream_handle())
        torch.cuda.synchronize()
        out[use_prep] = (d1_loss.cpu(), grads.cpu(), astat.cpu(), gstat.cpu(), ds[0].cpu())
    (d1a, ga, aa, sa, d1s), (d1b, gb, ab, sb, _) = out[False], out[True]
    rel = lambda x, y: ((x.double() - y.double()).abs().max() / y.double().abs().max()).item()
    assert rel(d1b, d1a) < 2e-6, rel(d1b, d1a)
    off, n = _layout(A, C3)
    ends = off[1:] + [n]
    for o, e in zip(off, ends):
        assert rel(gb[o:e], ga[o:e]) < 2e-6, (o, rel(gb[o:e], ga[o:e]))
    assert rel(ab, aa) < 2e-6
    # G factors: conv1's from the kernel's Gram, the rest unchanged
    o0 = so[5]
    ref = (d1s.double().reshape(-1, 32).t() @ d1s.double().reshape(-1, 32)) / (400 * B)
    got = sb[o0:o0 + 32 * 32].double().reshape(32, 32)
    err = (got - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err
    assert torch.equal(got, got.t())
    assert rel(sb[so[6]:], sa[so[6]:]) < 2e-6


@pytest.mark.parametrize('A,C3,B', [(4, 32, 29), (18, 64, 29), (18, 32, 1024)],
                         ids=['breakout', 'full-actions-c64', 'configs4-shard-1024x18'])
def test_bf16_forward_mode(lib, cuda, A, C3, B):
    """acmi_set_forward_mode(ACMI_FWD_BF16) (BASELINE configs[4] "bf16 forward"):
    the conv tower with one 16-bit MFMA per product (the scaled f16 h parts alone)
    stays within bf16 accuracy of the float64 forward (max error <= 1e-2 of each
    tensor's range), and
    switching back restores the f32-accurate tower bit for bit.  The last case is
    the configs[4] shard itself: 1024 images per launch, the full 18-action set,
    C3 = 32 (ACKTR)."""
    params = rand_params(A, C3, cuda, seed=31)
    obs = torch.randint(0, 256, (B, 84, 84, 4), generator=torch.Generator().manual_seed(32),
                        dtype=torch.uint8).to(cuda)
    prep = torch.empty(int(lib.acmi_conv_prep_bytes(C3)), dtype=torch.uint8, device=cuda)
    net = _lib.Net(A, C3, params.data_ptr(), prep.data_ptr())
    _lib.call('acmi_conv_prepare', ctypes.byref(net), _lib.ptr(prep), _lib.stream_handle())
    ref = torch_forward(params, obs.cpu(), A, C3)
    names = ['a1', 'a2', 'a3', 'a4', 'logits', 'value']
    outs = {}
    prev = lib.acmi_get_forward_mode()
    try:
        for mode in (_lib.FWD_F32, _lib.FWD_BF16, _lib.FWD_F32):
            _lib.call('acmi_set_forward_mode', mode)
            t, acts = alloc_acts(B, A, C3, cuda)
            _lib.call('acmi_forward', ctypes.byref(net), _lib.ptr(obs), 84 * 84 * 4, B, ctypes.byref(acts), 1,
                      _lib.stream_handle())
            torch.cuda.synchronize()
            outs.setdefault(mode, []).append({k: v.cpu() for k, v in t.items()})
    finally:
        _lib.call('acmi_set_forward_mode', prev)
    f32a, f32b = outs[_lib.FWD_F32]
    for k in f32a:
        assert torch.equal(f32a[k], f32b[k]), k
    bf = outs[_lib.FWD_BF16][0]
    for name, r in zip(names, ref):
        got = bf[name].double().reshape(r.shape)
        err = (got - r).abs().max().item() / max(1e-6, r.abs().max().item())
        print(name, 'bf16 forward rel err %.2e' % err)
        assert err < 1e-2, (name, err)
        assert not torch.equal(bf[name], f32a[name]), name  # the mode really changed the arithmetic


@pytest.mark.parametrize('B', [6, 300, 1000])
def test_conv1_afactor_and_weight_gradient_match_float64(lib, cuda, B):
    """The fused conv1 A-factor + weight-gradient kernel (conv1_afactor_roles_kernel:
    exact integer A partials, f16x2 weight gradient on the u8 patches as f16
    subnormals) against float64: the weight and bias gradients [P;1]^T d1 over the
    stored d1 within 2e-6 of their range, the A factor against the exact integer
    patch Gram within 1e-6 (B = 300).  B = 6: one stage per chunk (the odd tail
    only); 300: 4 stages (the paired loop only); 1000: 13 stages (both)."""
    A, C3 = 4, 32
    params = rand_params(A, C3, cuda, seed=31)
    g = torch.Generator().manual_seed(32)
    obs = torch.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=torch.uint8)
    obs_d = obs.to(cuda)
    t, acts = alloc_acts(B, A, C3, cuda)
    net = _net(params, A, C3)
    _lib.call('acmi_forward', ctypes.byref(net), _lib.ptr(obs_d), 84 * 84 * 4, B, ctypes.byref(acts), 1,
              _lib.stream_handle())
    ldh = 8
    dhead = torch.zeros(B, ldh)
    dhead[:, :A + 1] = torch.randn(B, A + 1, generator=g) / B
    dhead = dhead.to(cuda)
    z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=cuda)
    din = (ctypes.c_int64 * 6)()
    so = (ctypes.c_int64 * 11)()
    tot = ctypes.c_int64()
    _lib.call('acmi_kfac_layout', A, C3, din, None, so, ctypes.byref(tot))
    ws = z(lib.acmi_backward_ws_floats(B, A, C3))
    d = [z(B, 20, 20, 32), z(B, 9, 9, 64), z(B, 7, 7, C3), z(B, 512)]
    bwd = _lib.Bwd(*[x.data_ptr() for x in d], dhead.data_ptr(), ldh)
    grads, astat = z(params.numel()), z(tot.value)
    _lib.call('acmi_backward', ctypes.byref(net), _lib.ptr(obs_d), 84 * 84 * 4, B, ctypes.byref(acts),
              ctypes.byref(bwd), _lib.ptr(grads), _lib.ptr(astat), _lib.ptr(ws), ws.numel(), _lib.stream_handle())
    torch.cuda.synchronize()
    p = obs.double().unfold(1, 8, 4).unfold(2, 8, 4).permute(0, 1, 2, 4, 5, 3).reshape(-1, 256)
    d1 = d[0].cpu().double().reshape(-1, 32)
    off, _ = _layout(A, C3)
    gw = grads[off[0]:off[0] + 256 * 32].cpu().double().reshape(256, 32)
    gb = grads[off[1]:off[1] + 32].cpu().double()
    ref_w = (p / 255.0).t() @ d1
    ref_b = d1.sum(0)
    rw = ((gw - ref_w).abs().max() / ref_w.abs().max()).item()
    rb = ((gb - ref_b).abs().max() / ref_b.abs().max()).item()
    assert rw < 2e-6 and rb < 2e-6, (rw, rb)
    if B == 300:
        pb = torch.cat([p, torch.full((p.shape[0], 1), 255.0, dtype=torch.float64)], 1)
        ref = (pb.t() @ pb) / (65025.0 * p.shape[0])  # integer sums: exact in float64
        got = astat[so[0]:so[0] + 257 * 257].cpu().double().reshape(257, 257)
        rel = (got - ref).abs().max().item() / ref.abs().max().item()
        assert rel < 1e-6, rel


def test_kfac_pack_unpack_round_trip(lib, cuda):
    """acmi_kfac_pack / unpack (the data-parallel all-reduce of the factor statistics
    as upper triangles): the packed A and G parts are the factors' upper triangles
    row by row, back to back, and unpacking restores symmetric factors bit for bit
    (and mirrors the upper triangle into the lower one)."""
    A, C3 = 4, 32
    din = (ctypes.c_int64 * 6)()
    dout = (ctypes.c_int64 * 6)()
    so = (ctypes.c_int64 * 11)()
    tot = ctypes.c_int64()
    _lib.call('acmi_kfac_layout', A, C3, din, dout, so, ctypes.byref(tot))
    g = torch.Generator().manual_seed(3)
    stats = torch.zeros(tot.value)
    tris = {1: [], 2: []}
    for f in range(11):
        n = din[f] if f < 5 else dout[f - 5]
        m = torch.randn(n, n, generator=g)
        m = m + m.t()
        stats[so[f]:so[f] + n * n] = m.reshape(-1)
        iu = torch.triu_indices(n, n)
        tris[1 if f < 5 else 2].append(m[iu[0], iu[1]])
    ref = {w: torch.cat(tris[w]) for w in (1, 2)}
    ref[3] = torch.cat([ref[1], ref[2]])
    sd = stats.to(cuda)
    for which in (1, 2, 3):
        n = int(lib.acmi_kfac_packed_floats(A, C3, which))
        assert n == ref[which].numel()
        pk = torch.zeros(n, device=cuda)
        _lib.call('acmi_kfac_pack', A, C3, which, _lib.ptr(sd), _lib.ptr(pk), _lib.stream_handle())
        torch.cuda.synchronize()
        assert torch.equal(pk.cpu(), ref[which]), which
    pk = torch.zeros(ref[3].numel(), device=cuda)
    _lib.call('acmi_kfac_pack', A, C3, 3, _lib.ptr(sd), _lib.ptr(pk), _lib.stream_handle())
    back = torch.zeros(tot.value, device=cuda)
    _lib.call('acmi_kfac_unpack', A, C3, 3, _lib.ptr(pk), _lib.ptr(back), _lib.stream_handle())
    torch.cuda.synchronize()
    assert torch.equal(back.cpu(), stats)
