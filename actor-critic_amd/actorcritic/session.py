"""A tf.Session stand-in for the reference's graph-mode call pattern.

The reference builds a TF1 graph and evaluates it with
``session.run(fetches, feed_dict)`` (model.py:149-151, a2c_acktr.py:117-126).  Here
graph nodes are small Python objects whose ``_eval(ctx)`` enqueues libacmi kernels on
the current HIP stream; a ``_RunContext`` memoises each node once per ``run`` exactly
like a TF step, so fetching ``[summary_op, global_step, optimize_op]`` runs the forward,
loss, backward and optimizer once.
"""

import numbers

import numpy as np
import torch


class Node(object):
    """Base class of every fetchable object."""

    name = 'node'

    def _eval(self, ctx):  # pragma: no cover - abstract
        raise NotImplementedError

    def _finalize(self, ctx, value):
        """The fetched value once every node of the run is enqueued (Session.run calls
        it for each fetch); nodes whose value depends on later ops of the same run --
        the loss scalars, reduced over ranks only if the optimize op ran -- override it."""
        return value

    def __add__(self, other):
        return _Sum(self, other)

    def __radd__(self, other):
        return _Sum(other, self)

    def __mul__(self, other):
        return _Scale(self, other)

    __rmul__ = __mul__

    def __neg__(self):
        return _Scale(self, -1.0)


class Placeholder(Node):
    """tf.placeholder: a feed key with a dtype and a shape (None = any)."""

    def __init__(self, dtype, shape, name):
        self.dtype = dtype
        self.shape = tuple(shape)
        self.name = name

    def _eval(self, ctx):
        if self not in ctx.feeds:
            raise KeyError('You must feed a value for placeholder {!r}'.format(self.name))
        return ctx.feeds[self]

    def __repr__(self):
        return '<Placeholder {} {} {}>'.format(self.name, np.dtype(self.dtype).name, self.shape)


class Constant(Node):
    def __init__(self, value, name='const'):
        self.value = value
        self.name = name

    def _eval(self, ctx):
        return self.value


class NoOp(Node):
    name = 'no_op'

    def _eval(self, ctx):
        return None


def no_op():
    return NoOp()


def as_node(x):
    return x if isinstance(x, Node) else Constant(x)


class _Sum(Node):
    def __init__(self, a, b):
        self.a, self.b = as_node(a), as_node(b)

    def _eval(self, ctx):
        return ctx.eval(self.a) + ctx.eval(self.b)

    def _finalize(self, ctx, value):
        return self.a._finalize(ctx, ctx.eval(self.a)) + self.b._finalize(ctx, ctx.eval(self.b))


class _Scale(Node):
    def __init__(self, a, k):
        self.a, self.k = as_node(a), as_node(k)

    def _eval(self, ctx):
        return ctx.eval(self.a) * ctx.eval(self.k)

    def _finalize(self, ctx, value):
        return self.a._finalize(ctx, ctx.eval(self.a)) * self.k._finalize(ctx, ctx.eval(self.k))


class Variable(Node):
    """A host-side scalar variable (global_step)."""

    def __init__(self, value, name):
        self.value = value
        self.name = name

    def _eval(self, ctx):
        return self.value

    def assign(self, value):
        self.value = value


_GLOBAL_STEP = None


def get_or_create_global_step():
    """tf.train.get_or_create_global_step (a2c_acktr.py:59)."""
    global _GLOBAL_STEP
    if _GLOBAL_STEP is None:
        _GLOBAL_STEP = Variable(0, 'global_step')
    return _GLOBAL_STEP


def reset_default_graph():
    global _GLOBAL_STEP
    _GLOBAL_STEP = None


class _RunContext(object):
    def __init__(self, session, feeds):
        self.session = session
        self.feeds = feeds
        self.cache = {}

    def eval(self, node):
        if not isinstance(node, Node):
            return node
        key = id(node)
        if key not in self.cache:
            self.cache[key] = (node, node._eval(self))
        return self.cache[key][1]


def _to_host(v):
    if isinstance(v, torch.Tensor):
        v = v.detach()
        if v.dim() == 0:
            return v.item()
        return v.cpu().numpy()
    return v


class Session(object):
    """Evaluates nodes; values come back as numpy arrays / Python scalars like TF.

    ``run(..., host=False)`` keeps tensor results on the device (used by the hot loop).
    """

    def __init__(self, device=None):
        self.device = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
        self.closed = False

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def close(self):
        self.closed = True

    def run(self, fetches, feed_dict=None, host=True):
        if self.closed:
            raise RuntimeError('Attempted to use a closed Session.')
        ctx = _RunContext(self, dict(feed_dict or {}))
        single = not isinstance(fetches, (list, tuple))
        items = [fetches] if single else list(fetches)
        out = [ctx.eval(f) if f is not None else None for f in items]
        out = [f._finalize(ctx, v) if isinstance(f, Node) else v for f, v in zip(items, out)]
        if host:
            out = [_to_host(v) for v in out]
        return out[0] if single else out


def global_variables_initializer():
    return NoOp()


def is_number(x):
    return isinstance(x, numbers.Number)
