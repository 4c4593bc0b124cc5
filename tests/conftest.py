"""pytest configuration: registers the `gpu` marker and puts the repo root (oracle/)
and the product package directory on sys.path."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "dino-video-summarization-transformer_amd")
for p in (ROOT, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs under `pytest -m gpu` on the GPU box)")
    config.addinivalue_line("markers", "slow: CPU test that takes more than ~10 s")
