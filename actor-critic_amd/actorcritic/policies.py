"""Policies (reference: actorcritic/policies.py:10-158).

:class:`SoftmaxPolicy` is a categorical distribution over the logits node of a model;
its ``sample`` / ``mode`` / ``entropy`` / ``log_prob`` are graph nodes evaluated by
libacmi (acmi_sample_actions, acmi_categorical).
"""

from abc import ABCMeta, abstractmethod

import torch

from actorcritic.session import Node


class Policy(object, metaclass=ABCMeta):
    @property
    @abstractmethod
    def sample(self):
        pass

    @property
    @abstractmethod
    def mode(self):
        pass

    @property
    @abstractmethod
    def entropy(self):
        pass

    @property
    @abstractmethod
    def log_prob(self):
        pass

    def register_predictive_distribution(self, layer_collection, random_seed=None):
        raise NotImplementedError()


class _Sample(Node):
    """Categorical.sample squeezed on the last axis (policies.py:86): valid for a
    [batch, 1] observation feed, returns [batch] actions."""

    def __init__(self, logits, mode, seed):
        self.logits, self.mode, self.seed = logits, mode, seed
        self.name = 'mode' if mode else 'sample'

    def _eval(self, ctx):
        out = ctx.eval(self.logits)  # LogitsValue
        if out.steps != 1:
            raise ValueError('Can not squeeze dim[1], expected a dimension of 1, got {} (policies.py:86)'
                             .format(out.steps))
        eng = out.engine
        B = out.batch
        actions = torch.empty(B, dtype=torch.int32, device=eng.device)
        eng.sample(out.flat_logits, B, actions, mode=self.mode, seed=self.seed or 0, stream_id=eng.rank)
        eng.check_bad_rows()
        return actions


class _Entropy(Node):
    name = 'entropy'

    def __init__(self, logits):
        self.logits = logits

    def _eval(self, ctx):
        out = ctx.eval(self.logits)
        return out.entropy()


class _LogProb(Node):
    name = 'log_prob'

    def __init__(self, logits, actions):
        self.logits, self.actions = logits, actions

    def _eval(self, ctx):
        out = ctx.eval(self.logits)
        return out.log_prob(ctx.eval(self.actions))


class DistributionPolicy(Policy, metaclass=ABCMeta):
    def __init__(self, logits, actions, random_seed=None):
        self._logits = logits
        self._sample = _Sample(logits, False, random_seed)
        self._mode = _Sample(logits, True, random_seed)
        self._entropy = _Entropy(logits)
        self._log_prob = _LogProb(logits, actions)

    @property
    def logits(self):
        return self._logits

    @property
    def sample(self):
        return self._sample

    @property
    def mode(self):
        return self._mode

    @property
    def entropy(self):
        return self._entropy

    @property
    def log_prob(self):
        return self._log_prob


class SoftmaxPolicy(DistributionPolicy):
    """Categorical(logits) policy (policies.py:124-158)."""

    def __init__(self, logits, actions, random_seed=None, name=None):
        super().__init__(logits, actions, random_seed)
        self.name = name or 'SoftmaxPolicy'

    def register_predictive_distribution(self, layer_collection, random_seed=None):
        return layer_collection.register_categorical_predictive_distribution(logits=self._logits, seed=random_seed)
