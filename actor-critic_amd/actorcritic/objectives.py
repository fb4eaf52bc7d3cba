"""Objectives (reference: actorcritic/objectives.py:10-214).

:class:`A2CObjective` keeps the reference's maths — n-step discounted targets with
terminal cuts and a bootstrap from V(s_T) (objectives.py:123-126, closures :178-214),
stop-gradient advantage (:128-130), no advantage normalisation, policy loss
``-(mean(adv*log pi) + beta*mean(H))`` (:132-149) and baseline loss
``mean((target-V)^2/2)`` (:151-154) — evaluated by libacmi (acmi_returns,
acmi_a2c_loss).  The py_func discount-matrix closures become one reverse scan per
env whose gamma tables are the exact float32 values the closures produce.

Two options go beyond the reference (BASELINE.json's north_star names them; both
off by default, so the defaults are the reference's objective): ``gae_lambda``
(GAE(lambda) targets/advantages, acmi_gae; lambda = 1 is the n-step target in
exact arithmetic) and ``normalize_advantages`` (batch-normalised advantages for
the policy loss, acmi_adv_moments / acmi_adv_normalize; under data parallelism
the moments are summed over ranks, so every rank normalises with the global
batch's mean and std).
"""

from abc import ABCMeta, abstractmethod

import numpy as np
import torch

from actorcritic import _lib
from actorcritic.session import Node, as_node


def gamma_tables(gamma, T):
    """gamma_pow[k] = f32(gamma)**f32(k) (numpy float32 power: the D-matrix entries of
    objectives.py:183-187); boot_pow[k] = k-fold sequential float32 product (the
    float32 cumprod of objectives.py:211)."""
    g = np.float32(gamma)
    gp = (g ** np.arange(T, dtype=np.float32)).astype(np.float32)
    bp = np.ones(T + 1, np.float32)
    for k in range(1, T + 1):
        bp[k] = np.float32(bp[k - 1] * g)
    return gp, bp


class ActorCriticObjective(object, metaclass=ABCMeta):
    @property
    @abstractmethod
    def policy_loss(self):
        pass

    @property
    @abstractmethod
    def baseline_loss(self):
        pass

    def optimize_separate(self, policy_optimizer, baseline_optimizer, policy_kwargs=None, baseline_kwargs=None):
        """Separate optimisation of the two losses (objectives.py:31-54) is not supported for the
        shared-trunk Atari model on this engine (out of the hot-path scope)."""
        raise NotImplementedError('optimize_separate is not supported; use optimize_shared')

    def optimize_shared(self, optimizer, baseline_loss_weight=0.5, **kwargs):
        """optimizer.minimize(policy_loss + baseline_loss_weight * baseline_loss) (objectives.py:56-79)."""
        shared_loss = SharedLoss(self, baseline_loss_weight)
        return optimizer.minimize(shared_loss, **kwargs)


class SharedLoss(Node):
    """policy_loss + w * baseline_loss: the differentiable loss of optimize_shared."""

    def __init__(self, objective, weight):
        self.objective = objective
        self.weight = float(weight)
        self.name = 'shared_loss'
        objective._vcoef = self.weight

    def _eval(self, ctx):
        # the loss vector itself: the update needs only its kernels to have run (the
        # gradient comes from acmi_a2c_loss's dhead), and a fetched value is formed
        # by _finalize -- no two device launches per update for the scalar
        return ctx.eval(self.objective._loss_node)

    def _finalize(self, ctx, value):
        loss = self.objective._loss_node.scalars(ctx)
        return loss[0] + self.weight * loss[1]


class _Targets(Node):
    name = 'target_values'

    def __init__(self, objective):
        self.objective = objective

    def _eval(self, ctx):
        obj = self.objective
        model = obj._model
        eng = model.engine
        fwd = ctx.eval(model._forward)
        boot = ctx.eval(model._bootstrap_forward)
        N, T = fwd.batch, fwd.steps
        if boot.batch != N:
            raise ValueError('bootstrap observations must have one row per environment ({} != {})'
                             .format(boot.batch, N))
        rewards = _device(ctx.eval(model.rewards_placeholder), torch.float32, eng.device).reshape(N, T)
        terminals = _device_bool_u8(ctx.eval(model.terminals_placeholder), eng.device).reshape(N, T)
        st = eng.update_state(N * T)
        if obj._gae_lambda is None:
            gp, bp = obj._tables(T, eng.device)
            _lib.call('acmi_returns', _lib.ptr(rewards), _lib.ptr(terminals), _lib.ptr(fwd.flat_value),
                      _lib.ptr(boot.flat_value), N, T, _lib.ptr(gp), _lib.ptr(bp), _lib.ptr(st.targets),
                      _lib.ptr(st.adv), eng.stream())
        else:
            _lib.call('acmi_gae', _lib.ptr(rewards), _lib.ptr(terminals), _lib.ptr(fwd.flat_value),
                      _lib.ptr(boot.flat_value), N, T, obj._gamma, obj._gae_lambda, _lib.ptr(st.targets),
                      _lib.ptr(st.adv), eng.stream())
        if obj._normalize:
            _normalize_advantages(eng, st.adv, N * T, obj._adv_eps)
        st.fwd = fwd
        return st


def _normalize_advantages(eng, adv, M, eps):
    """adv <- (adv - mean) / (std + eps) over the global batch (all ranks)."""
    ws = getattr(eng, '_adv_ws', None)
    need = int(eng.lib.acmi_adv_moments_ws_doubles(M))
    if ws is None or ws.numel() < need:
        ws = torch.zeros(need, dtype=torch.float64, device=eng.device)
        eng._adv_ws = ws
        eng._adv_moments = torch.zeros(2, dtype=torch.float64, device=eng.device)
    mom = eng._adv_moments
    _lib.call('acmi_adv_moments', _lib.ptr(adv), M, _lib.ptr(ws), _lib.ptr(mom), eng.stream())
    if eng.world_size > 1:
        from actorcritic import parallel
        parallel.allreduce_sum_(mom)
    _lib.call('acmi_adv_normalize', _lib.ptr(adv), M, _lib.ptr(mom), float(M * eng.world_size), float(eps),
              eng.stream())


class _Loss(Node):
    """Loss scalars [policy, baseline, entropy] + head gradients in the update state."""
    name = 'losses'

    def __init__(self, objective):
        self.objective = objective

    def _eval(self, ctx):
        obj = self.objective
        model = obj._model
        eng = model.engine
        st = ctx.eval(obj._targets_node)
        fwd = ctx.eval(model._forward)
        actions = _device(ctx.eval(model.actions_placeholder), torch.int32, eng.device).reshape(-1)
        M = fwd.M
        if actions.numel() != M:
            raise ValueError('actions must have the shape of the observations batch [env, step]')
        st.actions = actions
        # the kernel scales the loss scalars by 1/world like dhead; they hold the
        # global means once the update's all-reduce has summed them (loss_reduced)
        st.loss_reduced = eng.world_size == 1
        _lib.call('acmi_a2c_loss', _lib.ptr(fwd.flat_logits), eng.A, _lib.ptr(fwd.flat_value), _lib.ptr(actions),
                  _lib.ptr(st.targets), _lib.ptr(st.adv), M, eng.A, float(obj._beta), float(obj._vcoef),
                  1.0 / eng.world_size, _lib.ptr(st.dhead), eng.ldh, _lib.ptr(st.loss_ws), _lib.ptr(st.loss),
                  eng.stream())
        st.fwd = fwd
        return st.loss

    def scalars(self, ctx):
        """[policy, baseline, entropy] of this run as fetched: the global means when
        the run's optimize op all-reduced them, else (no update in the run) this
        rank's means -- the kernel's 1/world scale undone."""
        loss = ctx.eval(self)
        st = ctx.eval(self.objective._targets_node)
        if getattr(st, 'loss_reduced', True):
            return loss[:3]
        return loss[:3] * float(self.objective._model.engine.world_size)


class _LossScalar(Node):
    def __init__(self, loss_node, index, name):
        self.loss_node, self.index, self.name = loss_node, index, name

    def _eval(self, ctx):
        return ctx.eval(self.loss_node)[self.index]

    def _finalize(self, ctx, value):
        return self.loss_node.scalars(ctx)[self.index]


class A2CObjective(ActorCriticObjective):
    """A2C/ACKTR objective (objectives.py:82-175)."""

    def __init__(self, model, discount_factor=0.99, entropy_regularization_strength=0.01, name=None,
                 gae_lambda=None, normalize_advantages=False, advantage_epsilon=1e-8):
        """The reference's arguments (objectives.py:100); ``gae_lambda`` (None: the
        reference's n-step targets; a float in [0, 1]: GAE(lambda)) and
        ``normalize_advantages`` are extensions beyond it (module docstring)."""
        if gae_lambda is not None and not 0.0 <= float(gae_lambda) <= 1.0:
            raise ValueError('gae_lambda must be in [0, 1] or None, got {}'.format(gae_lambda))
        self._model = model
        self._gamma = float(discount_factor)
        self._gae_lambda = None if gae_lambda is None else float(gae_lambda)
        self._normalize = bool(normalize_advantages)
        self._adv_eps = float(advantage_epsilon)
        self._beta = float(entropy_regularization_strength)
        self._vcoef = 0.5
        self._name = name or 'A2CObjective'
        self._table_cache = {}
        self._targets_node = _Targets(self)
        self._loss_node = _Loss(self)
        self._policy_loss = _LossScalar(self._loss_node, 0, 'policy_loss')
        self._baseline_loss = _LossScalar(self._loss_node, 1, 'baseline_loss')
        self._mean_entropy = _LossScalar(self._loss_node, 2, 'mean_entropy')

    def _tables(self, T, device):
        if T not in self._table_cache:
            gp, bp = gamma_tables(self._gamma, T)
            self._table_cache[T] = (torch.from_numpy(gp).to(device), torch.from_numpy(bp).to(device))
        return self._table_cache[T]

    @property
    def model(self):
        return self._model

    @property
    def target_values(self):
        return _TargetView(self._targets_node, 'targets')

    @property
    def advantage(self):
        return _TargetView(self._targets_node, 'adv')

    @property
    def policy_loss(self):
        return self._policy_loss

    @property
    def baseline_loss(self):
        return self._baseline_loss

    @property
    def mean_entropy(self):
        return self._mean_entropy


class _TargetView(Node):
    def __init__(self, node, attr):
        self.node, self.attr, self.name = node, attr, attr

    def _eval(self, ctx):
        st = ctx.eval(self.node)
        fwd = st.fwd if hasattr(st, 'fwd') else None
        v = getattr(st, self.attr)
        if fwd is not None:
            return v.reshape(fwd.batch, fwd.steps)
        return v


def _device(x, dtype, device):
    if isinstance(x, torch.Tensor):
        t = x
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(x)))
    if t.dtype == torch.bool:
        t = t.to(torch.uint8)
    return t.to(device=device, dtype=dtype).contiguous()


def _device_bool_u8(x, device):
    if isinstance(x, torch.Tensor):
        t = x
        if t.dtype == torch.bool:
            t = t.view(torch.uint8) if t.is_contiguous() else t.to(torch.uint8)
        elif t.dtype != torch.uint8:
            t = (t != 0).to(torch.uint8)
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(x, dtype=bool)).view(np.uint8))
    return t.to(device).contiguous()
