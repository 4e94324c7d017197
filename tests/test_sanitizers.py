"""Host runtime under AddressSanitizer + UBSan: builds the sanitized extension and
exercises the libsvm parser, tokenizer, vocab encoder and shuffles in a preloaded child."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_runtime_clean_under_asan_ubsan():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sanitize_runtime.py")], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "clean" in r.stdout
