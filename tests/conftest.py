"""Shared test setup.

- `gpu` marker: tests that need an MI355X (run with -m gpu on the GPU box).
- torch is imported first (when present) so that a process which also uses
  torch has exactly one HIP runtime: libasr_amd.so then binds to the
  libamdhip64.so.7 torch already loaded.
- asr (the product's Python host mirror) and oracle (the CPU checker) are
  loaded by path: the package directory name is not a Python identifier.
"""
import importlib.util
import os
import sys
from pathlib import Path

# No GPU_MAX_HW_QUEUES override (round 6): the pipeline's CU-masked streams
# get hardware queues of their own, and the tests run at whatever the box
# exports (HIP's default is 4); tests/test_pipeline_gpu.py checks the
# library's fit of its unmasked streams by setting what asr_pipeline_create
# reads.

try:
    import torch  # noqa: F401  (see module docstring)
except Exception:  # pragma: no cover
    torch = None

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "gpu-accelerated-speech-recognition_amd"
GOLDEN = Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(ROOT))


def _load(name, path):
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


asr = _load("asr_amd", PKG / "asr_amd.py")
oracle = _load("ctc_oracle", ROOT / "oracle" / "ctc_oracle.py")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950)")


def cpu_threads():
    return max(1, min(16, os.cpu_count() or 1))
