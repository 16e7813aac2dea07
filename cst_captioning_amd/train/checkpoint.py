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
    _atomic_save({'model': model.state_dict(), 'infos': infos, 'opt': opt}, path)
    logger.info('Wrote checkpoint to: %s', path)


def load_checkpoint(path, map_location='cpu', trusted=True):
    """Load a checkpoint.  Reference checkpoints pickle an argparse Namespace,
    so they need ``weights_only=False``: only do that for files this
    framework (or a trusted reference run) wrote.  ``trusted=False`` loads
    with ``weights_only=True`` and returns only what that allows."""
    if not trusted:
        return torch.load(path, map_location=map_location, weights_only=True)
    return torch.load(path, map_location=map_location, weights_only=False)


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


def save_last(path, model, optimizer, infos, opt, loader, rng_extra=None, per_rank=None):
    """``per_rank``: optional list (one entry per DP rank) of
    ``{'loader': state, 'rng': state}``; rank r resumes from entry r."""
    state = {'model': model.state_dict(), 'infos': infos, 'opt': opt,
             'optimizer': optimizer.state_dict(), 'loader': loader.state_dict(),
             'rng': rng_state(rng_extra)}
    if per_rank is not None:
        state['per_rank'] = per_rank
    _atomic_save(state, path)


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
