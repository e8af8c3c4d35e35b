"""Debug: tools/probe_py.py with torch's HIP runtime brought up first (as tests/conftest.py does)."""
import os, runpy, sys
import torch
torch.cuda.init()
print("torch", torch.__version__, torch.cuda.is_available(), flush=True)
sys.argv = ["probe_py.py"] + sys.argv[1:]
runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "probe_py.py"), run_name="__main__")
