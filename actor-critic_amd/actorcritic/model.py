"""Base class of actor-critic models (reference: actorcritic/model.py:10-186).

Placeholders are feed keys of :class:`actorcritic.session.Session` with the
reference's dtypes and shapes (`_space_placeholder`, model.py:172-186); the policy,
baseline and bootstrap values are graph nodes evaluated by libacmi kernels.
"""

from abc import ABCMeta

import numpy as np

from actorcritic import spaces
from actorcritic.session import Placeholder


class ActorCriticModel(object, metaclass=ABCMeta):
    """A model that provides a policy, a baseline and bootstrap values, plus the five
    placeholders of the reference (model.py:97-105)."""

    def __init__(self, observation_space, action_space):
        self._observations_placeholder = None
        self._bootstrap_observations_placeholder = None
        self._actions_placeholder = None
        self._rewards_placeholder = None
        self._terminals_placeholder = None

        self._setup_placeholders(observation_space, action_space)

        self._policy = None
        self._baseline = None
        self._bootstrap_values = None

    @property
    def observations_placeholder(self):
        return self._observations_placeholder

    @property
    def bootstrap_observations_placeholder(self):
        return self._bootstrap_observations_placeholder

    @property
    def actions_placeholder(self):
        return self._actions_placeholder

    @property
    def rewards_placeholder(self):
        return self._rewards_placeholder

    @property
    def terminals_placeholder(self):
        return self._terminals_placeholder

    @property
    def policy(self):
        return self._policy

    @property
    def baseline(self):
        return self._baseline

    @property
    def bootstrap_values(self):
        return self._bootstrap_values

    def _setup_placeholders(self, observation_space, action_space):
        self._observations_placeholder = _space_placeholder(observation_space, [None, None], 'observations')
        self._bootstrap_observations_placeholder = _space_placeholder(observation_space, [None],
                                                                      'bootstrap_observations')
        self._actions_placeholder = _space_placeholder(action_space, [None, None], 'actions')
        self._rewards_placeholder = Placeholder(np.float32, [None, None], 'rewards')
        self._terminals_placeholder = Placeholder(np.bool_, [None, None], 'terminals')

    def register_layers(self, layer_collection):
        raise NotImplementedError()

    def register_predictive_distributions(self, layer_collection, random_seed=None):
        self._policy.register_predictive_distribution(layer_collection, random_seed)
        self._baseline.register_predictive_distribution(layer_collection, random_seed)

    def sample_actions(self, observations, session):
        """session.run(policy.sample) on [batch, 1]-shaped observations -> list (model.py:135-151)."""
        return _tolist(session.run(self.policy.sample, feed_dict={self.observations_placeholder: observations}))

    def select_max_actions(self, observations, session):
        """session.run(policy.mode) -> list (model.py:153-169)."""
        return _tolist(session.run(self.policy.mode, feed_dict={self.observations_placeholder: observations}))


def _tolist(x):
    return x.tolist() if hasattr(x, 'tolist') else list(x)


def _space_placeholder(space, batch_shape=None, name=None):
    """Placeholder for a space (model.py:172-186): Discrete -> min scalar dtype of n,
    Box -> the space dtype and shape; anything else raises TypeError."""
    if batch_shape is None:
        batch_shape = [None]
    if spaces.is_discrete(space):
        return Placeholder(np.min_scalar_type(space.n), batch_shape, name)
    if spaces.is_box(space):
        if np.dtype(space.low.dtype) != np.dtype(space.high.dtype) or space.low.shape != space.high.shape:
            raise TypeError()
        return Placeholder(space.low.dtype, list(batch_shape) + list(space.low.shape), name)
    raise TypeError('Unsupported space')
