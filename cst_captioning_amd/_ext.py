"""Loader for the native extension ``cst_captioning_amd._C``.

``_C`` is built in-tree (``python setup.py build_ext --inplace`` or
``__graft_entry__.build()``) from ``csrc/``: gfx950 HIP kernels plus the C++
host runtime (decoder time-loop executor, CIDEr-D table builder, native CPU
scorer).

Policy: on a machine with a GPU the extension is REQUIRED -- a missing or
broken build raises instead of silently falling back to PyTorch ops (set
``CSTCAP_ALLOW_TORCH_FALLBACK=1`` to opt out, e.g. to measure the
reference-semantics baseline).  On a CPU-only machine the torch paths are
used.
"""
import os

_mod = None
_err = None


def _load():
    global _mod, _err
    if _mod is not None or _err is not None:
        return
    try:
        import torch  # noqa: F401  (libtorch must be loaded first)
        if os.environ.get('CSTCAP_EXT') == 'san':  # host-sanitized build (setup.py)
            from . import _C_san as _C  # type: ignore
        else:
            from . import _C  # type: ignore
        _mod = _C
    except Exception as e:  # pragma: no cover - depends on build state
        _err = e


def available():
    _load()
    if _mod is not None:
        return True
    import torch
    if torch.cuda.is_available() and os.environ.get('CSTCAP_ALLOW_TORCH_FALLBACK') != '1':
        raise RuntimeError(
            'cst_captioning_amd._C (HIP kernels) failed to load on a GPU machine: %r. '
            'Build it with `python setup.py build_ext --inplace`, or set '
            'CSTCAP_ALLOW_TORCH_FALLBACK=1 to run the plain PyTorch path.' % (_err,))
    return False


def host_available():
    """True if the extension loaded (its CPU-side functions work without a GPU)."""
    _load()
    return _mod is not None


def ops():
    _load()
    if _mod is None:
        raise RuntimeError('cst_captioning_amd._C is not built: %r' % (_err,))
    return _mod
