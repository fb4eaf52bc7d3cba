"""K-FAC for the Atari model (reference: actorcritic/kfac_utils.py:1-53 over the
un-vendored tensorflow/kfac; conventions pinned in DESIGN.md §K-FAC).

Per update (all libacmi, no host round trips):
  * acmi_backward fuses the weight gradient with the A-factor statistics
    ([P;1]^T [P | dY | 1] over every conv location / fc row),
  * acmi_kfac_output_stats samples the predictive distributions (categorical on the
    logits, normal var=1 on the value) and back-propagates them for the G factors,
  * one all-reduce of [grads | losses | A | G] when data-parallel,
  * acmi_kfac_ema: zero-initialised EMA with zero-debias,
  * every `invert_every` updates acmi_kfac_inverse: pi-adjusted factored damping and
    fp64 block Gauss-Jordan inverses,
  * acmi_kfac_step: Delta = Ainv [dW;db] Ginv, trust-region coefficient on the device,
    momentum, parameter update.
"""

import ctypes

import numpy as np
import torch

from actorcritic import _lib
from actorcritic.nn import OptimizeOp, Optimizer


class LayerCollection(object):
    """kfac.LayerCollection stand-in: records the registrations of
    AtariModel.register_layers / register_predictive_distributions."""

    EXPECTED = ('conv1', 'conv2', 'conv3', 'fc4', 'fc_policy', 'fc_baseline')

    def __init__(self):
        self.layers = []
        self.losses = []
        self.model = None

    def register_conv2d(self, params, strides, padding, inputs, outputs, approx=None):
        if padding != 'VALID':
            raise NotImplementedError('only VALID convolutions are registered by the reference')
        self.layers.append(('conv2d', params, tuple(strides)))

    def register_fully_connected(self, params, inputs, outputs, approx=None):
        self.layers.append(('fully_connected', params, None))

    def register_categorical_predictive_distribution(self, logits, seed=None, targets=None, name=None):
        self.losses.append(('categorical', seed))

    def register_normal_predictive_distribution(self, mean, var=0.5, seed=None, targets=None, name=None):
        if float(var) != 1.0:
            raise NotImplementedError('the reference registers var=1.0 (baselines.py:66)')
        self.losses.append(('normal', seed))

    def validate(self):
        names = tuple(l[1] for l in self.layers)
        if names != self.EXPECTED:
            raise ValueError('K-FAC blocks must be the six Atari layers {} (got {})'.format(self.EXPECTED, names))
        kinds = sorted(l[0] for l in self.losses)
        if kinds != ['categorical', 'normal']:
            raise ValueError('register_predictive_distributions must register the categorical policy and the '
                             'normal(var=1) baseline (got {})'.format(kinds))
        if self.model is None:
            raise ValueError('register_layers was not called')


class KfacOptimizer(Optimizer):
    """kfac.KfacOptimizer (regular momentum, trust region = norm_constraint)."""

    def __init__(self, learning_rate, cov_ema_decay, damping, layer_collection, momentum=0.9,
                 norm_constraint=None, momentum_type='regular', cov_devices=None, inv_devices=None,
                 estimation_mode='gradients', conv_damping_normalize=False, name='KFAC', **unused):
        super().__init__(learning_rate, name)
        if momentum_type != 'regular':
            raise NotImplementedError('momentum_type {!r}'.format(momentum_type))
        if estimation_mode != 'gradients':
            raise NotImplementedError('estimation_mode {!r} (the reference uses the default '
                                      '"gradients")'.format(estimation_mode))
        self._cov_ema_decay = float(cov_ema_decay)
        self._damping = float(damping)
        self._layers = layer_collection
        self._momentum = float(momentum)
        self._norm_constraint = float(norm_constraint) if norm_constraint is not None else None
        self._conv_normalize = bool(conv_damping_normalize)
        self._state = None
        self.cov_updates = 0       # number of EMA updates so far (zero-debias exponent)
        self.inverse_updates = 0
        self.last_coeff = None

    # -- state -------------------------------------------------------------------
    def _init_state(self, eng):
        if self._state is not None:
            return self._state
        self._layers.validate()
        L = eng.layout
        dev = eng.device
        z = lambda n, dt=torch.float32: torch.zeros(int(n), dtype=dt, device=dev)
        s = dict(
            biased=z(L.stat_total), factors=z(L.stat_total), inv=z(L.inv_total),
            inv_ws=z(eng.lib.acmi_kfac_inverse_ws_doubles(L.A, L.C3), torch.float64),
            velocity=z(L.nparams), precon=z(L.nparams), step_ws=z(eng.lib.acmi_kfac_step_ws_floats(L.A, L.C3)),
            coeff=z(1))
        # kfac initialises the inverse variables to the identity (used until the first
        # inverse update, i.e. between the cold start and gs = cold + invert_every)
        for m in range(12):
            L.inverse_block(s['inv'], m).fill_diagonal_(1.0)
        self._state = s
        return s

    @property
    def state(self):
        return self._state

    # -- the three K-FAC phases ------------------------------------------------------
    def _cov_update(self, eng, st):
        s = self._state
        self.cov_updates += 1
        debias = 1.0 / (1.0 - self._cov_ema_decay ** self.cov_updates)
        _lib.call('acmi_kfac_ema', _lib.ptr(s['biased']), _lib.ptr(s['factors']), _lib.ptr(st.stats),
                  eng.layout.stat_total, self._cov_ema_decay, debias, 1.0 / eng.world_size, eng.stream())

    def _inv_update(self, eng):
        s = self._state
        L = eng.layout
        _lib.call('acmi_kfac_inverse', L.A, L.C3, _lib.ptr(s['factors']), self._damping,
                  1 if self._conv_normalize else 0, _lib.ptr(s['inv']), _lib.ptr(s['inv_ws']), eng.stream())
        self.inverse_updates += 1

    def _kfac_apply(self, eng, grads, lr):
        s = self._state
        L = eng.layout
        nc = self._norm_constraint if self._norm_constraint is not None else float('inf')
        _lib.call('acmi_kfac_step', L.A, L.C3, _lib.ptr(eng.params), _lib.ptr(s['velocity']), _lib.ptr(grads),
                  _lib.ptr(s['inv']), lr, self._momentum, nc, _lib.ptr(s['precon']), _lib.ptr(s['step_ws']),
                  _lib.ptr(s['coeff']), eng.stream())
        self.last_coeff = s['coeff']

    def _stats(self, eng, fwd, st, counter):
        eng.output_stats(fwd, st, seed=0x4b464143, counter=counter)

    def _update(self, ctx, objective, global_step, clip_norm=0.0):
        """Plain KfacOptimizer: covariance update every step, inverse every step."""
        eng = objective.model.engine
        s = self._init_state(eng)
        st = eng.update_state(ctx.eval(objective.model._forward).M)
        lr = self._lr(ctx)
        gs = global_step.value if global_step is not None else self.cov_updates
        pending = eng.backward_and_stats(st.fwd, st, True, seed=0x4b464143, counter=gs)
        eng.allreduce_end(st, True, pending)
        self._cov_update(eng, st)
        self._inv_update(eng)
        self._kfac_apply(eng, st.grads, lr)
        eng.bump_version()
        if global_step is not None:
            global_step.assign(global_step.value + 1)
        return s


def schedule(global_step, num_cold_updates, invert_every):
    """The flags of one ColdStartPeriodicInvUpdateKfacOpt.apply_gradients
    (kfac_utils.py:38-53) with TF1 reads of the ref variable after each control
    dependency: (cold, cov, inv, global_step_after)."""
    gs = int(global_step)
    cold = gs < num_cold_updates
    if cold:
        gs += 1  # the cold optimizer's apply_gradients increments global_step
    cov = not cold
    inv = gs > num_cold_updates and (gs - num_cold_updates) % invert_every == 0
    gs += 1      # KfacOptimizer.apply_gradients increments global_step
    return cold, cov, inv, gs


class ColdStartPeriodicInvUpdateKfacOpt(KfacOptimizer):
    """K-FAC with a cold start and periodic inverses (kfac_utils.py:7-53).

    While global_step < num_cold_updates the cold optimizer AND the K-FAC apply (with the
    initial identity inverses) both run and global_step advances by 2; afterwards the
    covariances update every step and the inverses when
    global_step > num_cold_updates and (global_step - num_cold_updates) % invert_every == 0.
    """

    def __init__(self, num_cold_updates, cold_optimizer, invert_every, **kwargs):
        self._num_cold_updates = int(num_cold_updates)
        self._cold_optimizer = cold_optimizer
        self._invert_every = int(invert_every)
        super().__init__(**kwargs)
        self.last_flags = None

    def _update(self, ctx, objective, global_step, clip_norm=0.0):
        if global_step is None:
            raise ValueError('ColdStartPeriodicInvUpdateKfacOpt needs global_step')
        eng = objective.model.engine
        self._init_state(eng)
        st = eng.update_state(ctx.eval(objective.model._forward).M)
        lr = self._lr(ctx)  # learning_rate read once, from the pre-update global_step
        cold, cov, inv, gs_after = schedule(global_step.value, self._num_cold_updates, self._invert_every)
        self.last_flags = (cold, cov, inv)
        pending = eng.backward_and_stats(st.fwd, st, cov, seed=0x4b464143, counter=global_step.value)
        eng.allreduce_end(st, cov, pending)
        if cold:
            self._cold_optimizer._apply_dense(ctx, eng, st.grads, 0.0)
        else:
            self._cov_update(eng, st)
        if inv:
            self._inv_update(eng)
        self._kfac_apply(eng, st.grads, lr)
        eng.bump_version()
        global_step.assign(gs_after)
