import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: large inputs")


def pytest_collection_modifyitems(config, items):
    """GPU runs: bring up torch's HIP runtime before the scan library's (some GPU
    tests use torch for device buffers; torch's bundled runtime fails to
    initialise when /opt/rocm's was initialised first in the process)."""
    if any(it.get_closest_marker("gpu") for it in items):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass
