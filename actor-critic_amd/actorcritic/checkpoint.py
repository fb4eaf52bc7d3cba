"""Checkpoints and scalar summaries (reference: a2c_acktr.py:83-143, 256-303 —
tf.train.Saver files ``<path>/<model_name>-<step>`` + TensorBoard scalars).

TF checkpoints are unreadable without TensorFlow, so this engine writes its own:
``<prefix>-<step>.pt`` holding tensors and scalars only (loadable with
``torch.load(weights_only=True)``) and a ``checkpoint`` index file naming the latest,
like TF's.  Summaries are JSON lines (step, policy_loss, baseline_loss,
policy_entropy, episode_reward).
"""

import json
import os

import torch


def _first_order(optimizer):
    """The optimizer whose slot variables a checkpoint carries: the optimizer itself
    (A2C: clip-wrapped RMSProp) or, for ACKTR, its cold-start optimizer (clip-wrapped
    Momentum); the K-FAC state is saved separately under kfac/."""
    if optimizer is None:
        return None
    cold = getattr(optimizer, '_cold_optimizer', None)
    return cold if cold is not None else optimizer


def _optimizer_state(optimizer):
    out = {}
    if optimizer is None:
        return out
    st = getattr(optimizer, 'state', None)
    if isinstance(st, dict):
        for k, v in st.items():
            out['kfac/' + k] = v.detach().cpu()
    for attr in ('cov_updates', 'inverse_updates'):
        if hasattr(optimizer, attr):
            out['kfac_meta/' + attr] = torch.tensor(getattr(optimizer, attr))
    for name, v in _first_order(optimizer).slots().items():
        out['opt/' + name] = v.detach().cpu()
    return out


def save(prefix, step, model, optimizer=None):
    path = '{}-{}.pt'.format(prefix, int(step))
    blob = {'params': model.params.detach().cpu(), 'global_step': torch.tensor(int(step)),
            'num_actions': torch.tensor(model.num_actions), 'conv3_filters': torch.tensor(model.conv3_num_filters)}
    blob.update(_optimizer_state(optimizer))
    tmp = path + '.tmp'
    torch.save(blob, tmp)
    os.replace(tmp, path)
    with open(os.path.join(os.path.dirname(prefix) or '.', 'checkpoint'), 'w') as f:
        json.dump({'model_checkpoint_path': os.path.basename(path)}, f)
    return path


def latest(directory):
    idx = os.path.join(directory, 'checkpoint')
    if not os.path.exists(idx):
        return None
    with open(idx) as f:
        name = json.load(f)['model_checkpoint_path']
    path = os.path.join(directory, name)
    return path if os.path.exists(path) else None


def load(path, model, optimizer=None, global_step=None):
    blob = torch.load(path, map_location='cpu', weights_only=True)
    if int(blob['num_actions']) != model.num_actions or int(blob['conv3_filters']) != model.conv3_num_filters:
        raise ValueError('checkpoint was written for a different model')
    model.params.copy_(blob['params'].to(model.params.device))
    model.engine.bump_version()
    if global_step is not None:
        global_step.assign(int(blob['global_step']))
    if optimizer is not None:
        eng = model.engine
        slots = {k[4:]: v for k, v in blob.items() if k.startswith('opt/')}
        if slots:
            # tf.train.Saver restores the slot variables too (a2c_acktr.py:101-102)
            _first_order(optimizer).restore_slots(eng, slots)
        if any(k.startswith('kfac/') for k in blob) and hasattr(optimizer, '_init_state'):
            st = optimizer._init_state(eng)
            for k, v in blob.items():
                if k.startswith('kfac/'):
                    st[k[5:]].copy_(v.to(eng.device))
            for attr in ('cov_updates', 'inverse_updates'):
                if 'kfac_meta/' + attr in blob:
                    setattr(optimizer, attr, int(blob['kfac_meta/' + attr]))
    return blob


class ScalarLog(object):
    """Append-only JSON-lines scalar summaries (the TensorBoard scalars of a2c_acktr.py:83-92)."""

    def __init__(self, directory):
        os.makedirs(directory, exist_ok=True)
        self._f = open(os.path.join(directory, 'scalars.jsonl'), 'a')

    def add(self, step, **scalars):
        rec = {'step': int(step)}
        rec.update({k: (None if v != v else float(v)) for k, v in scalars.items()})
        self._f.write(json.dumps(rec) + '\n')
        if int(step) % 10 == 0:
            self._f.flush()

    def close(self):
        self._f.close()
