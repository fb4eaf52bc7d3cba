"""Baselines (reference: actorcritic/baselines.py:6-69)."""

from abc import ABCMeta, abstractmethod


class Baseline(object, metaclass=ABCMeta):
    @property
    @abstractmethod
    def value(self):
        pass

    def register_predictive_distribution(self, layer_collection, random_seed=None):
        raise NotImplementedError()


class StateValueFunction(Baseline):
    """A state-value baseline whose K-FAC predictive distribution is a normal with
    var=1.0 — vanilla Gauss-Newton (baselines.py:55-69)."""

    def __init__(self, value):
        self._value = value

    @property
    def value(self):
        return self._value

    def register_predictive_distribution(self, layer_collection, random_seed=None):
        layer_collection.register_normal_predictive_distribution(mean=self._value, var=1.0, seed=random_seed)
