"""Checkpoint round trips on the CPU (no GPU, no kernels): everything
``tf.train.Saver`` would restore (a2c_acktr.py:101-102, 256-275) comes back --
parameters, global step, the first-order optimizer's slot variables (RMSProp ms/mom,
cold-start Momentum accumulator) and the K-FAC state (factors, inverses, velocity,
EMA counters) -- including into a fresh optimizer whose slots were never allocated."""
import types

import pytest
import torch

from actorcritic import _lib, checkpoint
from actorcritic._engine import Layout
from actorcritic.kfac_utils import ColdStartPeriodicInvUpdateKfacOpt, LayerCollection
from actorcritic.nn import ClipGlobalNormOptimizer, MomentumOptimizer, RMSPropOptimizer
from actorcritic.session import Variable


class _CpuEngine(object):
    """The attributes of NetEngine the optimizer state and the checkpoint touch."""

    def __init__(self, A, C3, seed):
        self.lib = _lib.load()
        self.device = torch.device('cpu')
        self.layout = Layout(A, C3)
        g = torch.Generator().manual_seed(seed)
        self.params = torch.randn(self.layout.nparams, generator=g)
        self.version = 0

    def bump_version(self):
        self.version += 1


def _model(A, C3, seed):
    eng = _CpuEngine(A, C3, seed)
    return types.SimpleNamespace(params=eng.params, num_actions=A, conv3_num_filters=C3, engine=eng)


def _layers():
    lc = LayerCollection()
    for name, s in (('conv1', 4), ('conv2', 2), ('conv3', 1)):
        lc.register_conv2d(name, (1, s, s, 1), 'VALID', None, None)
    for name in ('fc4', 'fc_policy', 'fc_baseline'):
        lc.register_fully_connected(name, None, None)
    lc.register_categorical_predictive_distribution(None)
    lc.register_normal_predictive_distribution(None, var=1.0)
    lc.model = object()
    return lc


def _acktr():
    cold = ClipGlobalNormOptimizer(MomentumOptimizer(learning_rate=3e-4, momentum=0.9), clip_norm=0.5)
    return ColdStartPeriodicInvUpdateKfacOpt(
        num_cold_updates=30, cold_optimizer=cold, invert_every=10, learning_rate=0.25, cov_ema_decay=0.99,
        damping=0.01, layer_collection=_layers(), momentum=0.9, norm_constraint=1e-4)


def _a2c():
    return ClipGlobalNormOptimizer(RMSPropOptimizer(learning_rate=7e-4), clip_norm=0.5)


def _randomise(tensors, seed):
    g = torch.Generator().manual_seed(seed)
    for t in tensors:
        t.copy_(torch.randn(t.shape, generator=g, dtype=t.dtype))


def test_a2c_rmsprop_slots_round_trip(tmp_path):
    model = _model(4, 64, seed=1)
    opt = _a2c()
    opt._ensure_slots(model.engine)
    assert set(opt.slots()) == {'_ms', '_mom'}
    _randomise(opt.slots().values(), seed=2)
    path = checkpoint.save(str(tmp_path / 'Atari'), 123, model, opt)
    assert checkpoint.latest(str(tmp_path)) == path

    fresh_model = _model(4, 64, seed=9)
    fresh = _a2c()
    assert fresh.slots() == {}  # never applied: slots not allocated yet
    gs = Variable(0, 'global_step')
    checkpoint.load(path, fresh_model, fresh, gs)
    assert gs.value == 123
    assert torch.equal(fresh_model.params, model.params)
    assert fresh_model.engine.version == 1
    for name, v in opt.slots().items():
        assert torch.equal(fresh.slots()[name], v), name


def test_acktr_cold_slots_and_kfac_state_round_trip(tmp_path):
    model = _model(4, 32, seed=3)
    opt = _acktr()
    st = opt._init_state(model.engine)
    _randomise([v for v in st.values() if v.is_floating_point()], seed=4)
    opt._cold_optimizer._ensure_slots(model.engine)
    _randomise(opt._cold_optimizer.slots().values(), seed=5)
    opt.cov_updates, opt.inverse_updates = 17, 2
    path = checkpoint.save(str(tmp_path / 'Atari'), 47, model, opt)

    fresh_model = _model(4, 32, seed=8)
    fresh = _acktr()
    gs = Variable(0, 'global_step')
    checkpoint.load(path, fresh_model, fresh, gs)
    assert gs.value == 47
    assert torch.equal(fresh_model.params, model.params)
    assert (fresh.cov_updates, fresh.inverse_updates) == (17, 2)
    assert set(fresh.state) == set(st)
    for k, v in st.items():
        assert torch.equal(fresh.state[k], v), k
    assert set(fresh._cold_optimizer.slots()) == {'_accum'}
    assert torch.equal(fresh._cold_optimizer.slots()['_accum'], opt._cold_optimizer.slots()['_accum'])


def test_checkpoint_rejects_mismatched_optimizer_or_model(tmp_path):
    model = _model(4, 64, seed=1)
    opt = _a2c()
    opt._ensure_slots(model.engine)
    path = checkpoint.save(str(tmp_path / 'm'), 5, model, opt)
    # an RMSProp checkpoint has no Momentum accumulator
    wrong = ClipGlobalNormOptimizer(MomentumOptimizer(1e-3, 0.9), 0.5)
    with pytest.raises(ValueError):
        checkpoint.load(path, _model(4, 64, seed=2), wrong)
    with pytest.raises(ValueError):
        checkpoint.load(path, _model(4, 32, seed=2), _a2c())
