"""Checkpoints in the reference format, plus an exact-resume sidecar.

Reference (``/root/reference/train.py:67-93, 386-418``): ``torch.save({'model':
state_dict, 'infos': dict, 'opt': argparse.Namespace}, model_file)`` on every
new best (score ``>=`` best), a base checkpoint when none exists, and a
``_history.json`` of per-epoch infos.  Resume (``--start_from`` file or
directory + the same basename) restores weights and infos only.

Additions: ``<model>_last.pth`` holding optimizer, RNG and
loader state so a killed run continues bit-exactly (``save_last``), written
atomically (temp file + rename).
"""
import argparse
import json
import logging
import os

import numpy as np
import torch

logger = logging.getLogger(__name__)


def _atomic_save(obj, path):
    tmp = path + '.tmp'
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_checkpoint(model, infos, opt, path):
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    _atomic_save({'model': model.state_dict(), 'infos': _encode(infos), 'opt': _encode(opt)},
                 path)
    logger.info('Wrote checkpoint to: %s', path)


def _encode(obj):
    """Make a state tree loadable with ``weights_only=True``: numpy arrays
    become tagged tensors, numpy scalars Python numbers, numpy RNG state
    tuples tagged dicts."""
    if isinstance(obj, np.ndarray):
        return {'__ndarray__': torch.from_numpy(np.ascontiguousarray(obj))}
    if isinstance(obj, np.generic):
        return obj.item()
    if (isinstance(obj, tuple) and len(obj) == 5 and isinstance(obj[0], str)
            and obj[0] == 'MT19937'):
        return {'__np_rng__': [obj[0], torch.from_numpy(obj[1].astype(np.int64)), int(obj[2]),
                               int(obj[3]), float(obj[4])]}
    if isinstance(obj, argparse.Namespace):
        return argparse.Namespace(**_encode(vars(obj)))
    if isinstance(obj, dict):
        return {k: _encode(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_encode(v) for v in obj)
    return obj


def _decode(obj):
    if isinstance(obj, np.generic):  # numpy scalars of a reference checkpoint
        return obj.item()
    if isinstance(obj, argparse.Namespace):
        return argparse.Namespace(**_decode(vars(obj)))
    if isinstance(obj, dict):
        if set(obj) == {'__ndarray__'}:
            return obj['__ndarray__'].cpu().numpy()
        if set(obj) == {'__np_rng__'}:
            name, keys, pos, has_gauss, cached = obj['__np_rng__']
            return (name, keys.cpu().numpy().astype(np.uint32), pos, has_gauss, cached)
        return {k: _decode(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_decode(v) for v in obj)
    return obj


def _safe_globals():
    """Classes a reference checkpoint needs beyond tensors and containers:
    ``opt`` is a pickled ``argparse.Namespace`` (``/root/reference/train.py:87-91``)
    and the best-model ``infos`` carry numpy float64 scores from coco-caption
    (``train.py:403-407`` after ``infos.update(scores)``).  numpy scalars
    unpickle through ``multiarray.scalar(dtype, bytes)`` and the dtype
    classes: reconstructors that only rebuild a value, they run no code from
    the file."""
    out = [argparse.Namespace, np.dtype]
    try:
        from numpy._core.multiarray import scalar  # numpy >= 2
    except ImportError:  # pragma: no cover - numpy 1.x
        from numpy.core.multiarray import scalar
    out.append(scalar)
    dtypes = getattr(np, 'dtypes', None)
    if dtypes is not None:
        out += [getattr(dtypes, n) for n in dir(dtypes) if n.endswith('DType')]
    return out


def load_checkpoint(path, map_location='cpu'):
    """Load a checkpoint with ``torch.load(weights_only=True)`` -- nothing in
    the file is executed.  Allow-listed: ``argparse.Namespace`` and the numpy
    scalar reconstructors (:func:`_safe_globals`); numpy scalars come back as
    Python numbers.  Files this framework writes hold only tensors, containers
    and numbers (numpy state is tagged by :func:`_encode`)."""
    with torch.serialization.safe_globals(_safe_globals()):
        s = torch.load(path, map_location=map_location, weights_only=True)
    return _decode(s)


def resolve_start_from(start_from, model_file):
    if not start_from or not os.path.exists(start_from):
        return None
    if os.path.isdir(start_from):
        return os.path.join(start_from, os.path.basename(model_file))
    return start_from


def last_path(model_file):
    return model_file.replace('.pth', '_last.pth', 1) if model_file.endswith('.pth') \
        else model_file + '_last.pth'


def rng_state(extra=None):
    return {'torch': torch.get_rng_state(), 'numpy': np.random.get_state(),
            'cuda': torch.cuda.get_rng_state_all() if torch.cuda.is_available() else None,
            'extra': extra}


def save_last(path, model, optimizer, infos, opt, loader, rng_extra=None, per_rank=None,
              extra=None):
    """``per_rank``: optional list (one entry per DP rank) of
    ``{'loader': state, 'rng': state}``; rank r resumes from entry r.
    ``extra``: trainer state beyond ``infos`` (history, resolved schedule
    epochs)."""
    state = {'model': model.state_dict(), 'infos': infos, 'opt': opt,
             'optimizer': optimizer.state_dict(), 'loader': loader.state_dict(),
             'rng': rng_state(rng_extra)}
    if per_rank is not None:
        state['per_rank'] = per_rank
    if extra is not None:
        state['extra'] = extra
    _atomic_save(_encode(state), path)


def restore_rng(rng):
    torch.set_rng_state(rng['torch'])
    np.random.set_state(rng['numpy'])
    if rng.get('cuda') is not None and torch.cuda.is_available():
        torch.cuda.set_rng_state_all(rng['cuda'])


def write_history(history_file, history):
    if not history_file:
        return
    with open(history_file, 'w') as f:
        json.dump(history, f)
