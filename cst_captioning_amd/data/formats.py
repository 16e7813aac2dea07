"""On-disk formats for labels and features.

The reference stores labels and features in HDF5 (``create_sequencelabel.py:
87-103``, ``dataloader.py:33-49``).  h5py is not installed in this image, so
the native format is ``.npz`` with the same dataset names; ``.h5`` files are
read/written through h5py when it is importable (drop-in compatibility with
reference artefacts on machines that have it).

Feature files: reference layout is one dataset per ``str(video_id)`` holding
a ``(dim,)`` vector, broadcast to ``(num_chunks, dim)``
(``dataloader.py:109-110``).  The native layout is one array ``feats`` of
shape ``(N, dim)`` or ``(N, C, dim)`` aligned with a ``videos`` array.
"""
import numpy as np

try:  # optional dependency
    import h5py  # noqa: F401
    HAVE_H5PY = True
except ImportError:  # pragma: no cover - depends on the image
    HAVE_H5PY = False

LABEL_KEYS = ('labels', 'label_start_ix', 'label_end_ix', 'label_length', 'label_to_video')


def _need_h5(path):
    if not HAVE_H5PY:
        raise RuntimeError('%s is HDF5 but h5py is not installed; convert it to .npz '
                           '(cst_captioning_amd.data.formats) on a machine with h5py' % path)


def save_label_file(path, store):
    if path.endswith('.h5'):
        _need_h5(path)
        import h5py
        with h5py.File(path, 'w') as f:
            for k in LABEL_KEYS:
                if k in store:
                    f.create_dataset(k, data=store[k])
            f['videos'] = np.array([s.encode() for s in store['videos']])
            f['vocab'] = np.array([s.encode() for s in store['vocab']])
        return path
    out = dict(store)
    out['videos'] = np.asarray(store['videos'], dtype=str)
    out['vocab'] = np.asarray(store['vocab'], dtype=str)
    np.savez(path, **out)
    return path if path.endswith('.npz') else path + '.npz'


def load_label_file(path):
    """Dict with 'vocab' (list of str), 'videos' (list of str) and, when
    present, the label arrays as int64 numpy arrays."""
    if path.endswith('.h5'):
        _need_h5(path)
        import h5py
        with h5py.File(path, 'r') as f:
            out = {k: np.asarray(f[k], dtype=np.int64) for k in LABEL_KEYS if k in f}
            out['vocab'] = [v.decode() if isinstance(v, bytes) else str(v) for v in f['vocab']]
            out['videos'] = [v.decode() if isinstance(v, bytes) else str(v) for v in f['videos']]
        return out
    z = np.load(path, allow_pickle=False)
    out = {k: np.asarray(z[k], dtype=np.int64) for k in LABEL_KEYS if k in z.files}
    out['vocab'] = [str(v) for v in z['vocab']]
    out['videos'] = [str(v) for v in z['videos']]
    return out


def save_feature_file(path, videos, feats):
    feats = np.asarray(feats, dtype=np.float32)
    if path.endswith('.h5'):
        _need_h5(path)
        import h5py
        with h5py.File(path, 'w') as f:
            for v, x in zip(videos, feats):
                f[str(v)] = x
        return path
    np.savez(path, videos=np.asarray(videos, dtype=str), feats=feats)
    return path if path.endswith('.npz') else path + '.npz'


def load_feature_file(path, videos, num_chunks=1):
    """``(N, num_chunks, dim)`` float32 aligned with ``videos``."""
    if path.endswith('.h5'):
        _need_h5(path)
        import h5py
        with h5py.File(path, 'r') as f:
            arr = np.stack([np.asarray(f[str(v)], dtype=np.float32) for v in videos])
    else:
        z = np.load(path, allow_pickle=False)
        pos = {str(v): i for i, v in enumerate(z['videos'])}
        arr = np.asarray(z['feats'], dtype=np.float32)[[pos[str(v)] for v in videos]]
    if arr.ndim == 2:
        arr = np.repeat(arr[:, None, :], num_chunks, axis=1)
    elif arr.shape[1] != num_chunks:
        raise ValueError('%s has %d chunks, num_chunks=%d' % (path, arr.shape[1], num_chunks))
    return arr
