"""Optimizers and schedules (reference: actorcritic/nn.py:129-189 and the TF1 optimizers
the example uses, a2c_acktr.py:233-251).

Every update is: backward through the tower (acmi_backward) -> one all-reduce of the
gradient buffer when data-parallel -> a fused optimizer kernel
(acmi_momentum_apply / acmi_rmsprop_apply, global-norm clipping computed on the
device, no host round trip).
"""

from actorcritic import _lib
from actorcritic.session import Node, as_node


class LinearDecay(Node):
    """tf.train.polynomial_decay(power=1, cycle=False) (nn.py:129-156):
    ``(start - end) * (1 - min(step, total) / total) + end``."""

    def __init__(self, start_value, end_value, step, total_steps, name=None):
        self.start = start_value
        self.end = end_value
        self.step = step
        self.total = total_steps
        self.name = name or 'linear_decay'

    def _eval(self, ctx):
        start = float(ctx.eval(as_node(self.start)))
        end = float(ctx.eval(as_node(self.end)))
        total = float(ctx.eval(as_node(self.total)))
        step = min(float(ctx.eval(as_node(self.step))), total)
        return (start - end) * (1.0 - step / total) + end


def linear_decay(start_value, end_value, step, total_steps, name=None):
    return LinearDecay(start_value, end_value, step, total_steps, name)


class OptimizeOp(Node):
    """The op returned by ``optimizer.minimize``: forward (or the rollout's cached
    activations), targets, losses, backward and the parameter update."""

    def __init__(self, optimizer, loss, global_step):
        self.optimizer = optimizer
        self.loss = loss
        self.global_step = global_step
        self.name = 'optimize'

    def _eval(self, ctx):
        objective = getattr(self.loss, 'objective', None)
        if objective is None:
            raise NotImplementedError('only the shared A2C loss (objective.optimize_shared) is differentiable '
                                      'on this engine')
        ctx.eval(self.loss)
        self.optimizer._update(ctx, objective, self.global_step)
        return None


class Optimizer(object):
    """tf.train.Optimizer protocol subset: ``minimize(loss, global_step=None)``."""

    def __init__(self, learning_rate, name):
        self._learning_rate = learning_rate
        self._name = name

    def minimize(self, loss, global_step=None, name=None):
        return OptimizeOp(self, loss, global_step)

    def apply_gradients(self, grads_and_vars, global_step=None, name=None):
        raise NotImplementedError('gradients are engine buffers here; use minimize()')

    # -- engine hooks ----------------------------------------------------------
    def _lr(self, ctx):
        return float(ctx.eval(as_node(self._learning_rate)))

    def _update(self, ctx, objective, global_step, clip_norm=0.0):
        eng = objective.model.engine
        st = eng.update_state(ctx.eval(objective.model._forward).M)
        fwd = st.fwd
        eng.backward(fwd, st, with_stats=False)
        eng.allreduce(st, with_stats=False)
        self._apply_dense(ctx, eng, st.grads, clip_norm)
        eng.bump_version()
        if global_step is not None:
            global_step.assign(global_step.value + 1)

    def _apply_dense(self, ctx, eng, grads, clip_norm):  # pragma: no cover - abstract
        raise NotImplementedError

    # -- slot variables (tf.train.Optimizer slots: saved and restored by checkpoint) --
    _slot_names = ()

    def _ensure_slots(self, eng):
        """Allocates the slot variables with their TF initial values (first
        _apply_dense, or a checkpoint restore before it)."""

    def slots(self):
        """{name: tensor} of the allocated slot variables."""
        out = {}
        for name in self._slot_names:
            v = getattr(self, name, None)
            if v is not None:
                out[name] = v
        return out

    def restore_slots(self, eng, values):
        """Copies checkpointed slot values in, allocating the slots first."""
        unknown = set(values) - set(self._slot_names)
        if unknown:
            raise ValueError('{} has no slots {}'.format(type(self).__name__, sorted(unknown)))
        self._ensure_slots(eng)
        for name, v in values.items():
            dst = getattr(self, name)
            if tuple(dst.shape) != tuple(v.shape):
                raise ValueError('slot {} has shape {} in the checkpoint, {} here'.format(
                    name, tuple(v.shape), tuple(dst.shape)))
            dst.copy_(v.to(dst.device))


class MomentumOptimizer(Optimizer):
    """TF1 MomentumOptimizer: accum = m*accum + g;  var -= lr*accum."""

    def __init__(self, learning_rate, momentum, use_locking=False, name='Momentum', use_nesterov=False):
        super().__init__(learning_rate, name)
        if use_nesterov:
            raise NotImplementedError('nesterov momentum is not used by the reference')
        self._momentum = float(momentum)
        self._accum = None
        self._ws = None
        self.last_norm = None

    _slot_names = ('_accum',)

    def _ensure_slots(self, eng):
        import torch
        if self._accum is None:
            self._accum = torch.zeros_like(eng.params)  # TF 'momentum' slot: zeros
            self._ws = torch.zeros(int(eng.lib.acmi_opt_ws_floats(eng.params.numel())), device=eng.device)
            self.last_norm = torch.zeros(1, device=eng.device)

    def _apply_dense(self, ctx, eng, grads, clip_norm):
        self._ensure_slots(eng)
        _lib.call('acmi_momentum_apply', _lib.ptr(eng.params), _lib.ptr(self._accum), _lib.ptr(grads),
                  eng.params.numel(), self._lr(ctx), self._momentum, float(clip_norm), _lib.ptr(self._ws),
                  _lib.ptr(self.last_norm), eng.stream())


class RMSPropOptimizer(Optimizer):
    """TF1 RMSPropOptimizer (decay .9, momentum 0, epsilon 1e-10, ms initialised to 1):
    ms = d*ms + (1-d)*g^2;  mom = m*mom + lr*g/sqrt(ms+eps);  var -= mom."""

    def __init__(self, learning_rate, decay=0.9, momentum=0.0, epsilon=1e-10, use_locking=False, centered=False,
                 name='RMSProp'):
        super().__init__(learning_rate, name)
        if centered:
            raise NotImplementedError('centered RMSProp is not used by the reference')
        self._decay, self._momentum, self._eps = float(decay), float(momentum), float(epsilon)
        self._ms = self._mom = self._ws = None
        self.last_norm = None

    _slot_names = ('_ms', '_mom')

    def _ensure_slots(self, eng):
        import torch
        if self._ms is None:
            self._ms = torch.ones_like(eng.params)  # TF1 RMSProp 'rms' slot starts at 1
            self._mom = torch.zeros_like(eng.params)
            self._ws = torch.zeros(int(eng.lib.acmi_opt_ws_floats(eng.params.numel())), device=eng.device)
            self.last_norm = torch.zeros(1, device=eng.device)

    def _apply_dense(self, ctx, eng, grads, clip_norm):
        self._ensure_slots(eng)
        _lib.call('acmi_rmsprop_apply', _lib.ptr(eng.params), _lib.ptr(self._ms), _lib.ptr(self._mom),
                  _lib.ptr(grads), eng.params.numel(), self._lr(ctx), self._decay, self._momentum, self._eps,
                  float(clip_norm), _lib.ptr(self._ws), _lib.ptr(self.last_norm), eng.stream())


class ClipGlobalNormOptimizer(Optimizer):
    """Clips the gradients by their global norm before the wrapped optimizer
    (nn.py:159-189; tf.clip_by_global_norm: g *= c * min(1/||g||, 1/c))."""

    def __init__(self, optimizer, clip_norm, name=None):
        super().__init__(None, name or 'ClipGlobalNormOptimizer')
        self._optimizer = optimizer
        self._clip_norm = float(clip_norm)

    @property
    def optimizer(self):
        return self._optimizer

    @property
    def clip_norm(self):
        return self._clip_norm

    def _lr(self, ctx):
        return self._optimizer._lr(ctx)

    def _apply_dense(self, ctx, eng, grads, clip_norm):
        self._optimizer._apply_dense(ctx, eng, grads, self._clip_norm)

    def _ensure_slots(self, eng):
        self._optimizer._ensure_slots(eng)

    def slots(self):
        return self._optimizer.slots()

    def restore_slots(self, eng, values):
        self._optimizer.restore_slots(eng, values)
