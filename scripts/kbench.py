"""Kernel micro-benchmarks (HIP events) for tuning: plain GEMM, and the update's
backward (wgrad + A-factor reductions) at the bench workload size.

  python scripts/kbench.py gemm 4096
  python scripts/kbench.py backward 10240
  python scripts/kbench.py backward1 10240   # two timed reps (profiling)
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'actor-critic_amd'))

import torch  # noqa: E402

from actorcritic import _lib  # noqa: E402


def timeit(fn, reps=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def gemm(n):
    lib = _lib.load()
    A = torch.randn(n, n, device='cuda')
    B = torch.randn(n, n, device='cuda')
    C = torch.empty(n, n, device='cuda')
    ms = timeit(lambda: _lib.call('acmi_gemm_f32', _lib.ptr(A), _lib.ptr(B), _lib.ptr(C), n, n, n,
                                  _lib.stream_handle()))
    print('gemm {}^3: {:.3f} ms  {:.1f} TFLOP/s'.format(n, ms, 2 * n ** 3 / ms / 1e9))


def backward(M, with_stats=True, site=1, reps=10):
    from actorcritic._engine import NetEngine, OBS_BYTES
    eng = NetEngine(4, 32)
    obs = torch.randint(0, 256, (M, 84, 84, 4), dtype=torch.uint8, device='cuda')
    acts = eng.activations(M)
    eng.forward(obs.data_ptr(), M, acts.struct)
    st = eng.update_state(M)
    st.dhead.normal_()
    st.dhead[:, 5:] = 0

    class F:
        pass
    f = F()
    f.obs, f.M, f.acts = obs, M, acts
    _lib.call('acmi_prof_enable', site, 64)
    ms = timeit(lambda: eng.backward(f, st, with_stats), reps=reps, warm=min(3, reps))
    tot, cnt = ctypes.c_double(), ctypes.c_int()
    _lib.call('acmi_prof_collect', ctypes.byref(tot), ctypes.byref(cnt))
    _lib.call('acmi_prof_enable', 0, 0)
    print('backward M={} stats={}: {:.3f} ms; site {} kernel avg {:.3f} ms over {}'.format(
        M, with_stats, ms, site, tot.value / max(1, cnt.value), cnt.value))


def stats_chain(M, reps=10):
    """conv2 dX of the sampled-loss chain (site 5 inside acmi_kfac_output_stats: the
    Gram epilogue), then of backward + output stats together (both epilogues)"""
    from actorcritic._engine import NetEngine
    eng = NetEngine(4, 32)
    obs = torch.randint(0, 256, (M, 84, 84, 4), dtype=torch.uint8, device='cuda')
    acts = eng.activations(M)
    eng.forward(obs.data_ptr(), M, acts.struct)
    st = eng.update_state(M)
    st.dhead.normal_()
    st.dhead[:, 5:] = 0

    class F:
        pass
    f = F()
    f.obs, f.M, f.acts = obs, M, acts
    eng.backward(f, st, True)
    for name, fn in (('stats', lambda: eng.output_stats(f, st, 7, 3)),
                     ('backward+stats', lambda: (eng.backward(f, st, True), eng.output_stats(f, st, 7, 3)))):
        _lib.call('acmi_prof_enable', 5, 64)
        ms = timeit(fn, reps=reps, warm=2)
        tot, cnt = ctypes.c_double(), ctypes.c_int()
        _lib.call('acmi_prof_collect', ctypes.byref(tot), ctypes.byref(cnt))
        _lib.call('acmi_prof_enable', 0, 0)
        print('{} M={}: {:.3f} ms; conv2 dX kernel avg {:.3f} ms over {} (sum per call {:.3f})'.format(
            name, M, ms, tot.value / max(1, cnt.value), cnt.value, tot.value / (reps + 2)))


def c2mix(M, reps=20):
    """conv2 dX of both K-FAC chains: the two launches of today (mode 0) against
    the stacked launch (mode 1, acmi_debug_convt2), same lease, HIP events; and
    the outputs (masked d1, max |d1|, Gram partials) compared bit for bit"""
    from actorcritic._engine import NetEngine
    K_AMAX = 64 * 64  # kAmaxWords
    eng = NetEngine(4, 32)
    obs = torch.randint(0, 256, (M, 84, 84, 4), dtype=torch.uint8, device='cuda')
    acts = eng.activations(M)
    eng.forward(obs.data_ptr(), M, acts.struct)
    st = eng.update_state(M)
    st.dhead.normal_()
    st.dhead[:, 5:] = 0

    class F:
        pass
    f = F()
    f.obs, f.M, f.acts = obs, M, acts
    sd = st.side(eng)
    eng.backward(f, st, True)
    eng.output_stats(f, st, 7, 3, side=sd)
    torch.cuda.synchronize()
    net = eng.net()
    m1 = ctypes.c_void_p(acts.struct.m1)
    d2max_a = st.bwd_ws[2 * K_AMAX:3 * K_AMAX]  # band scratch kBsMaxD2 (workspace prefix)
    d2max_b = sd.ws[2 * K_AMAX:3 * K_AMAX]
    nb = 768
    outs = {}
    for mode in (0, 1):
        d1 = torch.zeros_like(st.d1)
        gp = torch.zeros(nb * 33 * 32, device='cuda')
        d1max = torch.zeros(K_AMAX, dtype=torch.int32, device='cuda')
        run = lambda: _lib.call('acmi_debug_convt2', ctypes.byref(net), mode, _lib.ptr(st.d2), _lib.ptr(sd.d2), m1,
                                _lib.ptr(d1), M, _lib.ptr(gp), _lib.ptr(d2max_a), _lib.ptr(d2max_b),
                                _lib.ptr(d1max), _lib.stream_handle())
        run()
        torch.cuda.synchronize()
        outs[mode] = (d1.clone(), gp.clone(), d1max.max().item())
        ms = timeit(run, reps=reps, warm=3)
        print('conv2 dX both chains, mode {} ({}): {:.1f} us'.format(mode, 'two launches' if mode == 0 else 'stacked',
                                                                     1e3 * ms))
    print('bit-identical: d1', torch.equal(outs[0][0], outs[1][0]), 'gram', torch.equal(outs[0][1], outs[1][1]),
          'max|d1|', outs[0][2] == outs[1][2])


def inverse(A=4, C3=32, reps=10):
    lib = _lib.load()
    din = (ctypes.c_int64 * 6)()
    dout = (ctypes.c_int64 * 6)()
    so = (ctypes.c_int64 * 11)()
    tot = ctypes.c_int64()
    _lib.call('acmi_kfac_layout', A, C3, din, dout, so, ctypes.byref(tot))
    fac = torch.zeros(tot.value, device='cuda')
    for f in range(11):
        n = din[f] if f < 5 else dout[f - 5]
        x = torch.randn(2 * n, n, device='cuda')
        fac[so[f]:so[f] + n * n] = (x.t() @ x / (2 * n)).reshape(-1)
    inv = torch.zeros(lib.acmi_kfac_inverse_floats(A, C3), device='cuda')
    ws = torch.zeros(lib.acmi_kfac_inverse_ws_doubles(A, C3), dtype=torch.float64, device='cuda')
    ms = timeit(lambda: _lib.call('acmi_kfac_inverse', A, C3, _lib.ptr(fac), ctypes.c_float(0.01), 0,
                                  _lib.ptr(inv), _lib.ptr(ws), _lib.stream_handle()), reps=reps)
    print('kfac inverse (all 12 damped inverses): {:.3f} ms'.format(ms))


def forward(B=512, reps=50):
    """rollout-batch forward (site 3 = the conv tower / conv1 kernel)"""
    from actorcritic._engine import NetEngine
    eng = NetEngine(4, 32)
    obs = torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device='cuda')
    acts = eng.activations(B)
    _lib.call('acmi_prof_enable', 3, 256)
    ms = timeit(lambda: eng.forward(obs.data_ptr(), B, acts.struct), reps=reps)
    tot, cnt = ctypes.c_double(), ctypes.c_int()
    _lib.call('acmi_prof_collect', ctypes.byref(tot), ctypes.byref(cnt))
    _lib.call('acmi_prof_enable', 0, 0)
    print('forward B={}: {:.1f} us; site 3 kernel avg {:.1f} us over {}'.format(
        B, 1e3 * ms, 1e3 * tot.value / max(1, cnt.value), cnt.value))


def band_scaling(sizes=(1024, 2048, 4096, 10240)):
    """conv2 band kernel time vs images: against its MFMA-bound time (sum over
    groups of the busiest SIMD's sub-tiles x 4 x 3 f16x2 MFMAs of 32 cycles per 16
    image rows, over 256 CUs at 2.4 GHz) -- memory effects show as a growing ratio"""
    for M in sizes:
        info = (ctypes.c_int64 * 5)()
        _lib.call('acmi_band_info', 1, 32, M, info)
        bound_ms = info[4] * 4 * 3 * 32 * (M / 16.0) / 256 / 2.4e9 * 1e3
        _lib.call('acmi_prof_enable', 2, 64)
        backward(M, True, 2, reps=6)
        print('   M={} plan {} -> MFMA-bound {:.3f} ms'.format(M, list(info), bound_ms))


if __name__ == '__main__':
    what = sys.argv[1]
    if what == 'band':
        band_scaling()
    elif what == 'forward':
        forward(int(sys.argv[2]) if len(sys.argv) > 2 else 512)
    if what == 'inverse':
        inverse()
    elif what == 'gemm':
        gemm(int(sys.argv[2]) if len(sys.argv) > 2 else 4096)
    elif what == 'c2mix':
        c2mix(int(sys.argv[2]) if len(sys.argv) > 2 else 10240)
    elif what == 'c2g':  # conv2 dX site of the sampled-loss chain (Gram epilogue) and of both chains
        stats_chain(int(sys.argv[2]) if len(sys.argv) > 2 else 10240)
    elif what == 'fc4dx':  # fc4 dX site (ACMI_PROF_FC4_DX = 6), then conv3 dX (7)
        M = int(sys.argv[2]) if len(sys.argv) > 2 else 10240
        backward(M, False, 6, reps=10)
        backward(M, False, 7, reps=10)
    elif what == 'af':  # conv1 A factor + weight gradient site (ACMI_PROF_CONV1_AFACTOR = 4)
        backward(int(sys.argv[2]) if len(sys.argv) > 2 else 10240, True, 4, reps=10)
    elif what == 'c2':  # conv2 dX site (ACMI_PROF_CONV2_DX = 5)
        backward(int(sys.argv[2]) if len(sys.argv) > 2 else 10240, False, 5, reps=10)
    elif what == 'backward1x':  # the conv2 band launch alone (site 2), ten timed reps
        backward(int(sys.argv[2]) if len(sys.argv) > 2 else 10240, True, 2, reps=10)
    elif what == 'backward1':  # a short run for PMC passes
        backward(int(sys.argv[2]) if len(sys.argv) > 2 else 10240, True, 2, reps=2)
    elif what == 'backward':
        M = int(sys.argv[2]) if len(sys.argv) > 2 else 10240
        for site in (1, 2, 4):
            backward(M, True, site)
        backward(M, False, 1)
