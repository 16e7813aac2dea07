"""Build the native extension in-tree:  python setup.py build_ext --inplace

Produces ``cst_captioning_amd/_C*.so`` from ``csrc/``:

  * ``csrc/kernels/*.hip`` -- gfx950 kernels, compiled directly by
    ``hipcc --offload-arch=gfx950`` (no hipify pass: torch's CUDAExtension
    would rewrite the sources into *_hip copies, so it is not used);
  * ``csrc/*.cpp``, ``csrc/host/*.cpp`` -- the C++ host runtime (decoder
    executor, CIDEr-D table builder / CPU scorer, bindings), compiled as a
    regular torch C++ extension against the ROCm headers and linked with the
    HIP objects and ``libamdhip64``.
"""
import glob
import os
import subprocess
import sys

from setuptools import setup

os.environ.setdefault('PYTORCH_ROCM_ARCH', 'gfx950')
from torch.utils.cpp_extension import (BuildExtension, CppExtension,  # noqa: E402
                                       include_paths, ROCM_HOME)

HERE = os.path.dirname(os.path.abspath(__file__))
ROCM = ROCM_HOME or '/opt/rocm'
HIPCC = os.path.join(ROCM, 'bin', 'hipcc')
OBJ_DIR = os.path.join(HERE, 'build', 'hip_objs')
HIP_SOURCES = sorted(glob.glob(os.path.join(HERE, 'csrc', 'kernels', '*.hip')))
HIP_FLAGS = ['--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-munsafe-fp-atomics',
             '-I' + os.path.join(HERE, 'csrc')]
# Debug build of the kernels: CSTCAP_KERNEL_DEBUG=1 compiles the
# device-side CST_DCHECK bounds checks in (separate object directory).  Pair it
# with CSTCAP_LAUNCH_CHECK=2 at run time to synchronise after every launch.
if os.environ.get('CSTCAP_KERNEL_DEBUG') == '1':
    HIP_FLAGS += ['-DCST_KERNEL_DEBUG', '-g']
    OBJ_DIR = os.path.join(HERE, 'build', 'hip_objs_debug')


def hip_objects():
    return [os.path.join(OBJ_DIR, os.path.basename(s)[:-4] + '.o') for s in HIP_SOURCES]


def compile_hip(jobs=8):
    """hipcc every kernel source (parallel, incremental on mtime)."""
    os.makedirs(OBJ_DIR, exist_ok=True)
    headers = glob.glob(os.path.join(HERE, 'csrc', '**', '*.h'), recursive=True)
    newest_header = max([os.path.getmtime(h) for h in headers] or [0])
    procs = []
    for src, obj in zip(HIP_SOURCES, hip_objects()):
        if os.path.exists(obj) and os.path.getmtime(obj) > max(os.path.getmtime(src),
                                                              newest_header):
            continue
        cmd = [HIPCC] + HIP_FLAGS + ['-c', src, '-o', obj]
        print(' '.join(cmd), flush=True)
        procs.append((src, subprocess.Popen(cmd)))
        while len([p for _, p in procs if p.poll() is None]) >= jobs:
            procs[0][1].wait()
    for src, p in procs:
        if p.wait() != 0:
            sys.exit('hipcc failed on %s' % src)


class BuildWithHip(BuildExtension):
    def run(self):
        compile_hip(int(os.environ.get('MAX_JOBS', '8')))
        super().run()


# Host-sanitized variant of the same extension: the C++ host
# runtime (decoder executor, bindings, CIDEr-D host code) under UBSan with
# abort-on-error plus libstdc++ container bounds checks, linked against the
# same gfx950 kernel objects.  CSTCAP_HOST_SANITIZE=1 python setup.py
# build_ext --inplace builds cst_captioning_amd._C_san; CSTCAP_EXT=san loads it
# instead of _C (tests/test_gpu_debug.py runs the engine through it).  UBSan
# needs no preloaded runtime (libubsan is an ordinary shared-library
# dependency), unlike ASan, which the host-only tests cover
# (tests/test_native_sanitizers.py).
SANITIZE = os.environ.get('CSTCAP_HOST_SANITIZE') == '1'
ext = CppExtension(
    'cst_captioning_amd._C_san' if SANITIZE else 'cst_captioning_amd._C',
    ['csrc/engine.cpp', 'csrc/bindings.cpp', 'csrc/host/cider_host.cpp',
     'csrc/host/blaslt_tuned.cpp'],
    include_dirs=[os.path.join(HERE, 'csrc')] + include_paths(device_type='cuda'),
    define_macros=[('__HIP_PLATFORM_AMD__', '1'), ('USE_ROCM', '1')]
    + ([('_GLIBCXX_ASSERTIONS', '1')] if SANITIZE else []),
    extra_compile_args=(['-O1', '-g', '-std=c++17', '-fsanitize=undefined',
                         '-fno-sanitize-recover=all', '-fno-omit-frame-pointer']
                        if SANITIZE else ['-O3', '-std=c++17']),
    extra_link_args=['-fsanitize=undefined'] if SANITIZE else [],
    extra_objects=hip_objects(),
    library_dirs=[os.path.join(ROCM, 'lib')],
    libraries=['amdhip64', 'c10_hip', 'torch_hip', 'hipblaslt'],
)

setup(
    name='cst_captioning_amd',
    version='0.1.0',
    packages=['cst_captioning_amd'],
    ext_modules=[ext],
    cmdclass={'build_ext': BuildWithHip.with_options(use_ninja=True)},
)
