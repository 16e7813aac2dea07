"""Sanitizer runs of the native host code.

GPU AddressSanitizer is not available on the MI355X pool, so the native
host-side runtime -- the CIDEr-D table builder and CPU scorer
(``csrc/host/cider_host.cpp``: open-addressing hash table, ragged offset
arrays) -- is compiled here with ``-fsanitize=address,undefined`` (no
recovery) and driven through random datasets and edge cases by
``tests/native/cider_host_check.cpp``.
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which('g++') is None, reason='needs g++')
def test_cider_host_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / 'cider_host_check')
    cmd = ['g++', '-std=c++17', '-O1', '-g', '-fno-omit-frame-pointer',
           '-fsanitize=address,undefined', '-fno-sanitize-recover=all',
           '-I' + os.path.join(REPO, 'csrc'),
           os.path.join(REPO, 'csrc', 'host', 'cider_host.cpp'),
           os.path.join(REPO, 'tests', 'native', 'cider_host_check.cpp'), '-o', exe]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=0',
               UBSAN_OPTIONS='print_stacktrace=1')
    res = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.strip().endswith('ok'), res.stdout
    assert 'runtime error' not in res.stderr, res.stderr
