"""Build the native extension in-tree:  python setup.py build_ext --inplace

Produces cst_captioning_amd/_C*.so from csrc/: gfx950 HIP kernels (hipcc,
--offload-arch=gfx950 only) plus the C++ host runtime (decoder executor,
CIDEr-D table builder and CPU scorer).
"""
import glob
import os

from setuptools import setup

os.environ.setdefault('PYTORCH_ROCM_ARCH', 'gfx950')
from torch.utils.cpp_extension import BuildExtension, CUDAExtension  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sources = (sorted(glob.glob(os.path.join('csrc', 'kernels', '*.hip'))) +
           ['csrc/engine.cpp', 'csrc/bindings.cpp', 'csrc/host/cider_host.cpp'])

setup(
    name='cst_captioning_amd',
    version='0.1.0',
    packages=['cst_captioning_amd'],
    ext_modules=[CUDAExtension(
        'cst_captioning_amd._C', sources,
        include_dirs=[os.path.join(HERE, 'csrc')],
        extra_compile_args={'cxx': ['-O3', '-std=c++17'],
                            'nvcc': ['-O3', '-std=c++17', '--offload-arch=gfx950',
                                     '-munsafe-fp-atomics']})],
    cmdclass={'build_ext': BuildExtension.with_options(use_ninja=True)},
)
