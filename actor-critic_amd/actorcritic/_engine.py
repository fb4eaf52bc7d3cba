"""Device-resident state of the Nature-CNN actor-critic on one GPU.

One flat fp32 parameter vector in the C-ABI layout (include/acmi.h: each layer's
homogeneous [W; b] block is one contiguous slice), activation buffers keyed by batch
size, and the update workspaces.  Every arithmetic call goes through libacmi.so.
"""

import ctypes
import os
import weakref

import numpy as np
import torch

from actorcritic import _lib

OBS_SHAPE = (84, 84, 4)
OBS_BYTES = 84 * 84 * 4


def _roundup4(x):
    return (x + 3) // 4 * 4


def _orthogonal(shape, gain, rng):
    """tf.orthogonal_initializer semantics (envs/atari/model.py:132-135)."""
    rows = int(np.prod(shape[:-1]))
    cols = shape[-1]
    a = rng.standard_normal((max(rows, cols), min(rows, cols)))
    q, r = np.linalg.qr(a)
    q = q * np.sign(np.diag(r))
    if rows < cols:
        q = q.T
    return (gain * q[:rows, :cols]).reshape(shape)


class Layout(object):
    def __init__(self, A, C3):
        lib = _lib.load()
        self.A, self.C3 = A, C3
        self.nparams = int(lib.acmi_param_count(A, C3))
        if self.nparams <= 0:
            raise ValueError('unsupported model: num_actions={} conv3_filters={}'.format(A, C3))
        off = (ctypes.c_int64 * 12)()
        _lib.call('acmi_param_offsets', A, C3, off)
        self.offsets = list(off)
        din = (ctypes.c_int64 * 6)()
        dout = (ctypes.c_int64 * 6)()
        so = (ctypes.c_int64 * 11)()
        tot = ctypes.c_int64()
        _lib.call('acmi_kfac_layout', A, C3, din, dout, so, ctypes.byref(tot))
        self.din, self.dout, self.stat_off, self.stat_total = list(din), list(dout), list(so), tot.value
        self.inv_total = int(lib.acmi_kfac_inverse_floats(A, C3))
        ioff = (ctypes.c_int64 * 12)()
        ild = (ctypes.c_int64 * 12)()
        _lib.call('acmi_kfac_inverse_layout', A, C3, ioff, ild)
        self.inv_off, self.inv_ld = list(ioff), list(ild)
        self.shapes = [(8, 8, 4, 32), (32,), (4, 4, 32, 64), (64,), (3, 3, 64, C3), (C3,), (49 * C3, 512), (512,),
                       (512, A), (A,), (512, 1), (1,)]
        self.names = ['conv1', 'conv2', 'conv3', 'fc4', 'fc_policy', 'fc_baseline']

    def inverse_block(self, inv, m):
        """[n, n] view of inverse block m (2l: Ainv_l, 2l+1: Ginv_l) of a flat
        inverse buffer (rows padded to inv_ld[m], acmi_kfac_inverse_layout)."""
        n = self.dout[m // 2] if m % 2 else self.din[m // 2]
        o, ld = self.inv_off[m], self.inv_ld[m]
        return inv[o:o + n * ld].view(n, ld)[:, :n]

    def init_params(self, seed=0):
        """Orthogonal init with gains sqrt(2) / 0.01 / 1.0 and zero biases."""
        rng = np.random.default_rng(seed)
        gains = [np.sqrt(2.0)] * 4 + [0.01, 1.0]
        parts = []
        for l in range(6):
            parts.append(_orthogonal(self.shapes[2 * l], gains[l], rng).ravel())
            parts.append(np.zeros(int(np.prod(self.shapes[2 * l + 1]))))
        return np.concatenate(parts).astype(np.float32)

    def split(self, flat):
        ends = self.offsets[1:] + [self.nparams]
        return [flat[o:e].reshape(s) for o, e, s in zip(self.offsets, ends, self.shapes)]


class Activations(object):
    """a1..a4, logits, value for a batch of B images (row-major, env-major)."""

    def __init__(self, B, layout, device):
        z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=device)
        self.B = B
        self.a1 = z(B, 20, 20, 32)
        self.a2 = z(B, 9, 9, 64)
        self.a3 = z(B, 7, 7, layout.C3)
        self.a4 = z(B, 512)
        self.logits = z(B, layout.A)
        self.value = z(B)
        # ReLU' bit masks (acmi_acts_t m1..m3): one uint32 per 32 channels of a pixel
        zi = lambda *s: torch.zeros(*s, dtype=torch.int32, device=device)
        self.m1 = zi(B, 400)
        self.m2 = zi(B, 81 * 2)
        self.m3 = zi(B, 49 * (layout.C3 // 32))
        self.ws = None
        self.struct = self.view(0, 1)

    def view(self, row, stride, ws_rows=None):
        """Acts struct whose batch row b is image row + b*stride (rollout step view);
        ws_rows: batch size the forward workspace must serve (default B / stride)."""
        el = lambda t, per: t.data_ptr() + 4 * row * per
        A = self.logits.shape[1]
        rows = ws_rows if ws_rows is not None else max(1, self.B // stride)
        need = int(_lib.load().acmi_forward_ws_floats(rows))
        if self.ws is None or self.ws.numel() < need:
            self.ws = torch.zeros(max(need, 1), dtype=torch.float32, device=self.a1.device)
        return _lib.Acts(el(self.a1, 400 * 32), el(self.a2, 81 * 64), el(self.a3, self.a3[0].numel()),
                         el(self.a4, 512), el(self.logits, A), el(self.value, 1), A, self.ws.data_ptr(),
                         self.ws.numel(), el(self.m1, 400), el(self.m2, 162), el(self.m3, self.m3.shape[1]))


class UpdateState(object):
    """Workspaces of one update over M = N*T rows.

    ``red`` is the one buffer a data-parallel update all-reduces:
    [grads (nparams) | loss scalars (4) | factor stats (A factors, then G factors)].
    """

    def __init__(self, eng, M):
        L = eng.layout
        dev = eng.device
        z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=dev)
        n, S = L.nparams, L.stat_total
        self.M = M
        self.red = z(n + 4 + S)
        self.grads = self.red[:n]
        self.loss = self.red[n:n + 4]
        # acmi_backward writes the A part and acmi_kfac_output_stats the G part of one
        # stats vector laid out like the factors (acmi_kfac_layout)
        self.stats = self.red[n + 4:]
        self.astat = self.stats
        self.gstat = self.stats
        self.n_grad_red = n + 4
        self.targets = z(M)
        self.adv = z(M)
        self.dhead = z(M, eng.ldh)
        self.d1 = z(M, 20, 20, 32)
        self.d2 = z(M, 9, 9, 64)
        self.d3 = z(M, 7, 7, L.C3)
        self.d4 = z(M, 512)
        self.bwd_ws = z(int(eng.lib.acmi_backward_ws_floats(M, L.A, L.C3)))
        self.loss_ws = z(int(eng.lib.acmi_a2c_loss_ws_floats(M)))
        self.bwd = _lib.Bwd(self.d1.data_ptr(), self.d2.data_ptr(), self.d3.data_ptr(), self.d4.data_ptr(),
                            self.dhead.data_ptr(), eng.ldh)
        self.actions = None
        self.fwd = None
        self.loss_reduced = True  # loss slots hold global means (see objectives._Loss)
        self._side = None

    def side(self, eng):
        """Second backward workspace (d1..d4, dhead, ws) and a side stream: the sampled-
        loss backward (acmi_kfac_output_stats) runs there concurrently with the loss
        backward (acmi_backward) -- the two chains share only read-only inputs (the
        rollout activations, the parameters) and write disjoint parts of ``stats``."""
        if self._side is None:
            L, dev, M = eng.layout, eng.device, self.M
            z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=dev)
            sd = type('SideState', (), {})()
            sd.dhead = z(M, eng.ldh)
            sd.d1, sd.d2, sd.d3, sd.d4 = z(M, 20, 20, 32), z(M, 9, 9, 64), z(M, 7, 7, L.C3), z(M, 512)
            sd.ws = z(int(eng.lib.acmi_backward_ws_floats(M, L.A, L.C3)))
            sd.bwd = _lib.Bwd(sd.d1.data_ptr(), sd.d2.data_ptr(), sd.d3.data_ptr(), sd.d4.data_ptr(),
                              sd.dhead.data_ptr(), eng.ldh)
            sd.stream = torch.cuda.Stream(device=dev)
            self._side = sd
        return self._side


class NetEngine(object):
    """Parameters + kernels of one AtariModel on one device."""

    def __init__(self, num_actions, conv3_filters, device=None, seed=0, params=None, forward_mode=None,
                 gemm_mode=None):
        _lib.require_gpu()
        self.lib = _lib.load()
        self.device = torch.device(device) if device is not None else torch.device('cuda',
                                                                                    torch.cuda.current_device())
        self.layout = Layout(num_actions, conv3_filters)
        self.A, self.C3 = num_actions, conv3_filters
        init = self.layout.init_params(seed) if params is None else np.asarray(params, np.float32)
        self.params = torch.from_numpy(init).to(self.device)
        from actorcritic import parallel
        self.rank = parallel.rank()
        self.world_size = parallel.world_size()
        # the per-update exchange runs when there are ranks to exchange with -- or,
        # test-only (ACMI_FORCE_COLLECTIVE=1 with a process group of one rank), through
        # the same RCCL calls at world size 1, where the sum must leave every bit as is
        # this net's arithmetic (acmi_net_t mode fields; None: the process default at each call)
        self.forward_mode, self.gemm_mode = forward_mode, gemm_mode
        self.collective = self.world_size > 1 or (
            os.environ.get('ACMI_FORCE_COLLECTIVE') == '1' and parallel.is_initialized())
        if self.world_size > 1:  # identical initial parameters on every rank
            parallel.broadcast_(self.params)
        self.version = 0  # bumped by every parameter update (activation-cache key)
        self.ldh = max(8, _roundup4(num_actions + 1))
        self._acts = {}
        self._updates = {}
        self._rollout_cache = None
        self._bad_rows = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._prep, self._prep_version = None, None
        self.sample_counter = 0
        self._comm = None  # comm_timing: [(start event, end event, bytes)] per update

    # -- update plumbing -------------------------------------------------------
    def update_state(self, M):
        if M not in self._updates:
            self._updates[M] = UpdateState(self, M)
        return self._updates[M]

    def bump_version(self):
        self.version += 1

    def register_rollout(self, obs, fwd_out):
        """Marks `obs` ([N,T,84,84,4] device buffer) as already forwarded with the current
        parameters: the update re-uses the rollout activations instead of recomputing the
        tower on identical (params, obs) (DESIGN.md §Rollout/update fusion).

        The key holds a weak reference to `obs`: once the registered tensor is freed
        (a copy_batches clone the caller dropped), its address may be handed to a
        different tensor of the same shape by the caching allocator, so the entry dies
        with it instead of matching that tensor."""
        self._rollout_cache = (weakref.ref(obs), obs.data_ptr(), tuple(obs.shape), self.version, fwd_out)

    def lookup_rollout(self, x):
        c = self._rollout_cache
        if c is None or not isinstance(x, torch.Tensor) or not x.is_cuda:
            return None
        ref = c[0]()
        if ref is None:  # the registered buffer is gone: its address means nothing now
            self._rollout_cache = None
            return None
        if x.data_ptr() == c[1] and tuple(x.shape) == c[2] and c[3] == self.version:
            return c[4]
        return None

    def backward(self, fwd, st, with_stats):
        net = self.net()
        _lib.call('acmi_backward', ctypes.byref(net), ctypes.c_void_p(fwd.obs.data_ptr()), OBS_BYTES, fwd.M,
                  ctypes.byref(fwd.acts.struct), ctypes.byref(st.bwd), _lib.ptr(st.grads),
                  _lib.ptr(st.astat) if with_stats else None, _lib.ptr(st.bwd_ws), st.bwd_ws.numel(), self.stream())

    def backward_stacked(self, fwd, st, sd, seed, counter):
        """acmi_backward + the sampled-loss chain's input gradients into the side
        buffers ``sd``, conv2's input gradient of both chains as one launch (on this
        stream); output_stats_finish then forms the G factors."""
        net = self.net()
        _lib.call('acmi_backward_stacked', ctypes.byref(net), ctypes.c_void_p(fwd.obs.data_ptr()), OBS_BYTES, fwd.M,
                  ctypes.byref(fwd.acts.struct), ctypes.byref(st.bwd), _lib.ptr(st.grads), _lib.ptr(st.astat),
                  _lib.ptr(st.bwd_ws), st.bwd_ws.numel(), ctypes.byref(sd.bwd), seed, self.rank * fwd.M, counter,
                  _lib.ptr(sd.ws), sd.ws.numel(), self.stream())

    def output_stats_finish(self, fwd, st, sd):
        net = self.net()
        _lib.call('acmi_kfac_output_stats_finish', ctypes.byref(net), fwd.M, ctypes.byref(fwd.acts.struct),
                  ctypes.byref(sd.bwd), _lib.ptr(st.gstat), _lib.ptr(sd.ws), sd.ws.numel(), self.stream())

    def output_stats(self, fwd, st, seed, counter, side=None):
        """side: run on UpdateState.side()'s stream and workspace (see there)."""
        net = self.net()
        bwd, ws = (side.bwd, side.ws) if side is not None else (st.bwd, st.bwd_ws)
        _lib.call('acmi_kfac_output_stats', ctypes.byref(net), fwd.M, ctypes.byref(fwd.acts.struct),
                  ctypes.byref(bwd), seed, self.rank * fwd.M, counter, _lib.ptr(st.gstat), _lib.ptr(ws),
                  ws.numel(), self.stream())

    # the G chain on a side stream: '1' always, '0' never, unset: at batches up to
    # CONCURRENT_STATS_ROWS.  Round 6 at the bench shard (512 x 20, same lease):
    # side stream 2.772-2.792 ms per update against 2.842-2.856 on one stream (the
    # band reduction slows 0.57 -> 0.64 ms beside it, the rest more than pays);
    # rounds 2-4 had measured one stream faster with the kernels of then
    concurrent_stats = {'1': True, '0': False}.get(os.environ.get('ACMI_CONCURRENT_STATS', ''))
    CONCURRENT_STATS_ROWS = 1 << 30
    # measured (ACKTR 512x20, one box): plain update 5.25 ms with the G chain started
    # next to the whole backward, 5.16 ms started after the backward's dX chain
    stats_after_dx = os.environ.get('ACMI_STATS_AFTER_DX', '1') != '0'
    # on one stream (larger batches): the two chains' conv2 input gradients as one
    # launch (acmi_backward_stacked) with ACMI_STACKED_DX=1.  Off by default: the
    # stacked launch is 11 % faster than the two launches back to back (kbench
    # c2mix, 564 vs 632 us, bit-identical), but in the update it moves the sampled
    # chain's dX ahead of the loss chain's reductions, which then re-read d1 / d2
    # from further away: update 2.914-2.925 vs 2.885-2.897 ms (same lease, 512 x 20)
    stacked_dx = os.environ.get('ACMI_STACKED_DX', '0') == '1'

    def backward_and_stats(self, fwd, st, with_stats, seed, counter):
        """acmi_backward (+ A stats) and, with stats, acmi_kfac_output_stats (G stats);
        starts the data-parallel all-reduce of the backward's prefix of ``red`` as soon
        as it is enqueued and returns its handle (allreduce_end completes it).  With
        ``concurrent_stats`` the G chain runs on a side stream next to the backward."""
        conc = self.concurrent_stats if self.concurrent_stats is not None else fwd.M <= self.CONCURRENT_STATS_ROWS
        if with_stats and not conc and self.stacked_dx:
            sd = st.side(self)  # (its d1..d4 and workspace; the work stays on this stream)
            self.backward_stacked(fwd, st, sd, seed, counter)
            pending = self.allreduce_begin(st, True)
            self.output_stats_finish(fwd, st, sd)
            return pending
        if not (with_stats and conc):
            self.backward(fwd, st, with_stats)
            pending = self.allreduce_begin(st, with_stats)
            if with_stats:
                self.output_stats(fwd, st, seed, counter)
            return pending
        main = torch.cuda.current_stream(self.device)
        sd = st.side(self)
        self.net()  # (any pending prepare on main, ahead of the fork)
        sd.stream.wait_stream(main)
        if self.stats_after_dx:
            # the sampled-loss chain starts where the loss backward's input-gradient
            # chain ends, next to its weight-gradient reductions
            self.backward(fwd, st, True)
            _lib.call('acmi_stream_wait_backward_dx', ctypes.c_void_p(sd.stream.cuda_stream))
            with torch.cuda.stream(sd.stream):
                self.output_stats(fwd, st, seed, counter, side=sd)
        else:
            with torch.cuda.stream(sd.stream):
                self.output_stats(fwd, st, seed, counter, side=sd)
            self.backward(fwd, st, True)
        pending = self.allreduce_begin(st, True)
        main.wait_stream(sd.stream)
        return pending

    def allreduce(self, st, with_stats):
        """Sums [grads | losses (| factor stats)] over ranks (RCCL); the 1/world scale is
        folded into the loss gradient and the factor EMA."""
        if self.collective:
            from actorcritic import parallel
            k = st.red.numel() if with_stats else st.n_grad_red
            parallel.allreduce_sum_(st.red[:k], force=True)
            st.loss_reduced = True

    def _packed(self, st):
        """[grads | losses | A stats | G stats] with the (symmetric) factor statistics
        as upper triangles (acmi_kfac_pack): what a K-FAC update all-reduces, 10.8 MB
        instead of 18.1 at C3 = 32."""
        if getattr(st, 'pk', None) is None:
            L = self.layout
            st.pk_na = int(self.lib.acmi_kfac_packed_floats(L.A, L.C3, 1))
            st.pk_ng = int(self.lib.acmi_kfac_packed_floats(L.A, L.C3, 2))
            st.pk = torch.zeros(st.n_grad_red + st.pk_na + st.pk_ng, dtype=torch.float32, device=self.device)
        return st.pk

    def allreduce_begin(self, st, with_stats):
        """Starts summing what acmi_backward produced -- [grads | losses (| A factor
        stats, packed)] -- over ranks without waiting: RCCL runs it on its own stream
        while the sampled-loss backward (acmi_kfac_output_stats, which writes only the
        G part) computes on this one.  Returns the pending handle (None on one rank);
        allreduce_end completes ``red``."""
        st.pk_active = False
        if not self.collective:
            return None
        from actorcritic import parallel
        st.loss_reduced = True
        if not with_stats:
            st.comm_bytes = 4 * st.n_grad_red
            return parallel.allreduce_sum_async(st.red[:st.n_grad_red])
        pk, ng, L = self._packed(st), st.n_grad_red, self.layout
        pk[:ng].copy_(st.red[:ng])
        _lib.call('acmi_kfac_pack', L.A, L.C3, 1, ctypes.c_void_p(st.stats.data_ptr()),
                  ctypes.c_void_p(pk[ng:].data_ptr()), self.stream())
        st.pk_active = True
        st.comm_bytes = 4 * (ng + st.pk_na + st.pk_ng)
        return parallel.allreduce_sum_async(pk[:ng + st.pk_na])

    def allreduce_end(self, st, with_stats, pending):
        """Sums the G factor stats (packed, if the prefix carried the A stats) and makes
        this stream wait for the pending prefix sum, then unpacks: ``red`` is fully
        reduced for the kernels enqueued next."""
        if not self.collective:
            return
        from actorcritic import parallel
        marks = self._comm_mark() if self._comm is not None else None
        if not st.pk_active:
            pending.wait()
        else:
            pk, ng, L = st.pk, st.n_grad_red, self.layout
            _lib.call('acmi_kfac_pack', L.A, L.C3, 2, ctypes.c_void_p(st.stats.data_ptr()),
                      ctypes.c_void_p(pk[ng + st.pk_na:].data_ptr()), self.stream())
            parallel.allreduce_sum_(pk[ng + st.pk_na:], force=True)
            pending.wait()
            st.red[:ng].copy_(pk[:ng])
            _lib.call('acmi_kfac_unpack', L.A, L.C3, 3, ctypes.c_void_p(pk[ng:].data_ptr()),
                      ctypes.c_void_p(st.stats.data_ptr()), self.stream())
            st.pk_active = False
        if marks is not None:
            marks[1].record()
            self._comm.append((marks[0], marks[1], st.comm_bytes))

    # -- communication timing (bench.py allreduce_ms) ----------------------------
    def comm_timing(self, on):
        """Records HIP events on the compute stream around allreduce_end -- from the end
        of the sampled-loss backward to the reduced buffer being ready (G-tail pack and
        sum, the wait for the asynchronous prefix sum, unpack): the time the update's
        compute stream stands still on the exchange step, skew between ranks included."""
        self._comm = [] if on else None

    def _comm_mark(self):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        return e0, e1

    def comm_collect(self):
        """(mean ms per update, bytes all-reduced per update, updates seen) of the
        exchanges recorded since comm_timing(True); call after a synchronize."""
        if not self._comm:
            return 0.0, 0, 0
        ms = [a.elapsed_time(b) for a, b, _ in self._comm]
        return sum(ms) / len(ms), self._comm[-1][2], len(ms)

    # -- plumbing ------------------------------------------------------------
    def net(self, force_prepare=False):
        """The C-ABI net: parameters + the conv tower's pre-split weights, re-prepared
        (acmi_conv_prepare, stream-ordered, on the CURRENT stream) at the first use after
        a parameter update, or always with ``force_prepare`` (a hipGraph capture: every
        replay re-prepares from the parameters as they are then).  A caller that forks
        work onto a second stream calls this on the parent stream BEFORE the fork, so the
        prepare is ordered ahead of both chains."""
        if self._prep is None:
            self._prep = torch.empty(int(self.lib.acmi_conv_prep_bytes(self.C3)), dtype=torch.uint8,
                                     device=self.device)
        net = _lib.Net(self.A, self.C3, self.params.data_ptr(), self._prep.data_ptr(),
                       0 if self.gemm_mode is None else self.gemm_mode + 1,
                       0 if self.forward_mode is None else self.forward_mode + 1, 0)
        if force_prepare or self._prep_version != (self.version, self.params.data_ptr()):
            _lib.call('acmi_conv_prepare', ctypes.byref(net), ctypes.c_void_p(self._prep.data_ptr()), self.stream())
            self._prep_version = (self.version, self.params.data_ptr())
        return net

    def activations(self, B, key='default'):
        k = (key, B)
        if k not in self._acts:
            self._acts[k] = Activations(B, self.layout, self.device)
        return self._acts[k]

    def stream(self):
        return _lib.stream_handle(self.device)

    # -- ops -----------------------------------------------------------------
    def forward(self, obs_ptr, B, acts_struct, want_value=True, img_stride=OBS_BYTES, act_stride=1):
        net = self.net()
        _lib.call('acmi_forward_strided', ctypes.byref(net), ctypes.c_void_p(obs_ptr), img_stride, B,
                  ctypes.byref(acts_struct), 1 if want_value else 0, act_stride, self.stream())

    def forward_obs(self, obs, key='default'):
        """obs: uint8 device tensor [B, 84, 84, 4] (contiguous)."""
        obs = _as_obs(obs, self.device)
        B = obs.shape[0]
        acts = self.activations(B, key)
        self.forward(obs.data_ptr(), B, acts.struct)
        return acts, obs

    def sample(self, logits, B, out, mode=False, seed=0, stream_id=0, uniforms=None, ld=None):
        _lib.call('acmi_sample_actions', ctypes.c_void_p(logits.data_ptr()), ld or self.A, B, self.A, seed,
                  stream_id, self.sample_counter, _lib.ptr(uniforms), 1 if mode else 0,
                  ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(self._bad_rows.data_ptr()), self.stream())
        self.sample_counter += 1

    def check_bad_rows(self):
        """Raises like the reference's out-of-range label error if any logits were NaN."""
        bad = int(self._bad_rows.item())
        if bad:
            self._bad_rows.zero_()
            raise FloatingPointError('{} policy rows had non-finite logits (reference: InvalidArgumentError '
                                     '"Received a label value ... outside the valid range", README.md:53)'
                                     .format(bad))


def _as_obs(obs, device):
    if isinstance(obs, torch.Tensor):
        t = obs
    else:
        t = torch.from_numpy(np.asarray(obs, dtype=np.uint8))
    if t.dtype != torch.uint8:
        raise TypeError('observations must be uint8 (model.py:172-186 placeholder dtype)')
    t = t.reshape(-1, *OBS_SHAPE)
    if t.device != device:
        t = t.to(device, non_blocking=True)
    return t.contiguous()
