import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line(
        "markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


import pytest  # noqa: E402


@pytest.fixture(autouse=True, scope="session")
def _torch_hip_first(request):
    """torch ships its own HIP runtime (torch/lib): in a process where the
    engine's (/opt/rocm) runtime came up first, torch's later finds no GPU
    ("No HIP GPUs are available").  A GPU session brings torch's up first;
    the tests that copy planes with torch need it."""
    if request.config.getoption("-m", default="") and \
            "not gpu" in request.config.getoption("-m"):
        return
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass
