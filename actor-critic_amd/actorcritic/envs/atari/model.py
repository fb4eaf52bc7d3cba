"""Nature-CNN actor-critic for Atari (reference: actorcritic/envs/atari/model.py:14-246).

conv 8x8 s4 (32) -> ReLU -> conv 4x4 s2 (64) -> ReLU -> conv 3x3 s1 (conv3_num_filters)
-> ReLU -> NHWC flatten -> fc 512 -> ReLU -> {policy logits, value}.  The tower runs in
libacmi (acmi_forward); parameters live in one flat fp32 device vector
(:class:`actorcritic._engine.NetEngine`).  A2C uses 64 conv3 filters, ACKTR 32.
"""

import torch

from actorcritic import spaces
from actorcritic._engine import NetEngine, _as_obs
from actorcritic import _lib
from actorcritic.baselines import StateValueFunction
from actorcritic.model import ActorCriticModel
from actorcritic.policies import SoftmaxPolicy
from actorcritic.session import Node


class ForwardOut(object):
    """Result of the tower on a fed [batch, steps] observation block."""

    def __init__(self, engine, acts, batch, steps, obs):
        self.engine = engine
        self.acts = acts
        self.batch = batch
        self.steps = steps
        self.M = batch * steps
        self.obs = obs  # device uint8 [M, 84, 84, 4]

    @property
    def flat_logits(self):
        return self.acts.logits[:self.M]

    @property
    def flat_value(self):
        return self.acts.value[:self.M]

    def logits(self):
        return self.flat_logits.reshape(self.batch, self.steps, -1)

    def value(self):
        return self.flat_value.reshape(self.batch, self.steps)

    def entropy(self):
        out = torch.empty(self.M, dtype=torch.float32, device=self.engine.device)
        _lib.call('acmi_categorical', _lib.ptr(self.flat_logits), self.engine.A, self.M, self.engine.A, None,
                  _lib.ptr(out), None, self.engine.stream())
        return out.reshape(self.batch, self.steps)

    def log_prob(self, actions):
        a = _actions_tensor(actions, self.engine.device).reshape(-1)
        if a.numel() != self.M:
            raise ValueError('actions shape does not match the observations')
        out = torch.empty(self.M, dtype=torch.float32, device=self.engine.device)
        _lib.call('acmi_categorical', _lib.ptr(self.flat_logits), self.engine.A, self.M, self.engine.A, _lib.ptr(a),
                  None, _lib.ptr(out), self.engine.stream())
        return out.reshape(self.batch, self.steps)


def _actions_tensor(actions, device):
    if isinstance(actions, torch.Tensor):
        t = actions
    else:
        import numpy as np
        t = torch.from_numpy(np.asarray(actions).astype(np.int32))
    return t.to(device=device, dtype=torch.int32).contiguous()


class _TowerForward(Node):
    """Forward of the tower on one of the two observation placeholders."""

    def __init__(self, model, placeholder, bootstrap):
        self.model = model
        self.placeholder = placeholder
        self.bootstrap = bootstrap
        self.name = 'bootstrap_forward' if bootstrap else 'forward'

    def _eval(self, ctx):
        eng = self.model._engine
        x = ctx.eval(self.placeholder)
        cached = eng.lookup_rollout(x) if not self.bootstrap else None
        if cached is not None:
            return cached
        obs = _as_obs(x, eng.device)
        if self.bootstrap:
            batch, steps = obs.shape[0], 1
        else:
            shape = tuple(x.shape) if hasattr(x, 'shape') else None
            if shape is None or len(shape) < 2:
                import numpy as np
                shape = np.shape(x)
            batch, steps = int(shape[0]), int(shape[1])
        M = batch * steps
        acts = eng.activations(M, 'boot' if self.bootstrap else 'feed')
        eng.forward(obs.data_ptr(), M, acts.struct, want_value=True)
        return ForwardOut(eng, acts, batch, steps, obs)


class _Logits(Node):
    def __init__(self, fwd):
        self.fwd = fwd
        self.name = 'logits'

    def _eval(self, ctx):
        return ctx.eval(self.fwd)


class _Value(Node):
    def __init__(self, fwd, bootstrap):
        self.fwd = fwd
        self.bootstrap = bootstrap
        self.name = 'bootstrap_values' if bootstrap else 'value'

    def _eval(self, ctx):
        out = ctx.eval(self.fwd)
        return out.flat_value if self.bootstrap else out.value()


class AtariModel(ActorCriticModel):
    """The A3C/ACKTR Atari model on MI355X.

    Args mirror the reference (envs/atari/model.py:45); ``device``, ``params`` (a flat
    float32 vector in the acmi layout), ``init_seed`` and ``forward_mode`` (this
    model's conv-tower precision, acmi ``FWD_F32`` / ``FWD_BF16``; None: the
    process default) are extensions.
    """

    def __init__(self, observation_space, action_space, conv3_num_filters=64, random_seed=None, name=None,
                 device=None, params=None, init_seed=0, forward_mode=None):
        super().__init__(observation_space, action_space)
        assert spaces.is_discrete(action_space)
        assert spaces.is_box(observation_space)
        if tuple(observation_space.shape) != (84, 84, 4):
            raise ValueError('AtariModel expects 84x84x4 stacked frames, got {}'.format(observation_space.shape))
        self._num_actions = action_space.n
        self._conv3_num_filters = conv3_num_filters
        self._name = name or 'AtariModel'
        self._random_seed = random_seed
        self._engine = NetEngine(self._num_actions, conv3_num_filters, device=device, seed=init_seed,
                                 params=params, forward_mode=forward_mode)

        self._forward = _TowerForward(self, self.observations_placeholder, bootstrap=False)
        self._bootstrap_forward = _TowerForward(self, self.bootstrap_observations_placeholder, bootstrap=True)
        self._policy = SoftmaxPolicy(_Logits(self._forward), self.actions_placeholder, random_seed)
        self._baseline = StateValueFunction(_Value(self._forward, False))
        self._bootstrap_values = _Value(self._bootstrap_forward, True)
        self._registered_layers = None

    @property
    def num_actions(self):
        return self._num_actions

    @property
    def conv3_num_filters(self):
        return self._conv3_num_filters

    @property
    def engine(self):
        return self._engine

    @property
    def params(self):
        """The flat fp32 parameter vector (device tensor)."""
        return self._engine.params

    def named_params(self):
        """{'conv1/weights': tensor view, ...} in the reference's variable naming."""
        views = self._engine.layout.split(self._engine.params)
        out = {}
        for l, n in enumerate(self._engine.layout.names):
            out[n + '/weights'] = views[2 * l]
            out[n + '/bias'] = views[2 * l + 1]
        return out

    def register_layers(self, layer_collection):
        """Registers the six K-FAC blocks of envs/atari/model.py:219-246."""
        layer_collection.register_conv2d('conv1', strides=[1, 4, 4, 1], padding='VALID', inputs='observations',
                                         outputs='conv1_pre')
        layer_collection.register_conv2d('conv2', strides=[1, 2, 2, 1], padding='VALID', inputs='conv1',
                                         outputs='conv2_pre')
        layer_collection.register_conv2d('conv3', strides=[1, 1, 1, 1], padding='VALID', inputs='conv2',
                                         outputs='conv3_pre')
        layer_collection.register_fully_connected('fc4', inputs='conv3', outputs='fc4_pre')
        layer_collection.register_fully_connected('fc_policy', inputs='fc4', outputs='fc_policy')
        layer_collection.register_fully_connected('fc_baseline', inputs='fc4', outputs='fc_baseline')
        layer_collection.model = self
        self._registered_layers = layer_collection
