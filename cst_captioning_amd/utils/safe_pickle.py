"""Restricted unpickler for the reference's data pickles.

The reference stores CIDEr-D document frequencies
(``/root/reference/compute_ciderdf.py:123-129``: ``{'document_frequency':
{tuple[str]: float}, 'ref_len': float}``) and GT consensus scores
(``/root/reference/compute_scores.py:105-108``: ``{metric: ndarray}``) as
pickles.  A plain ``pickle.load`` runs whatever callable the file names, so
these files are read with an unpickler that resolves only plain containers,
numbers, strings and numpy array / scalar reconstruction; any other global
raises :class:`pickle.UnpicklingError`.
"""
import io
import os
import pickle

_ALLOWED = {
    ('builtins', 'dict'), ('builtins', 'list'), ('builtins', 'tuple'), ('builtins', 'set'),
    ('builtins', 'frozenset'), ('builtins', 'str'), ('builtins', 'bytes'),
    ('builtins', 'int'), ('builtins', 'float'), ('builtins', 'bool'), ('builtins', 'complex'),
    ('collections', 'defaultdict'), ('collections', 'OrderedDict'),
    ('numpy', 'ndarray'), ('numpy', 'dtype'),
    ('numpy.core.multiarray', '_reconstruct'), ('numpy._core.multiarray', '_reconstruct'),
    ('numpy.core.multiarray', 'scalar'), ('numpy._core.multiarray', 'scalar'),
}
# numpy >= 1.25 pickles dtypes as numpy.dtypes.<Name>DType classes
_NUMPY_DTYPE_MODULES = ('numpy.dtypes',)


class RestrictedUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED or (module in _NUMPY_DTYPE_MODULES
                                          and name.endswith('DType')):
            return super().find_class(module, name)
        raise pickle.UnpicklingError('refusing to load global %s.%s from a data pickle'
                                     % (module, name))


def safe_load(f):
    """Unpickle from a binary file object, or from a path."""
    if isinstance(f, (str, os.PathLike)):
        with open(f, 'rb') as fh:
            return RestrictedUnpickler(fh).load()
    return RestrictedUnpickler(f).load()


def safe_loads(data):
    return RestrictedUnpickler(io.BytesIO(data)).load()
