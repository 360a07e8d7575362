"""Reference file name (code/3d_reconstruction.py) for the BA linearisation; the module itself is
reconstruction.py because a Python identifier cannot start with a digit (the reference comments
its import out for that reason, code/pipeline.py:4).  Load with importlib if needed."""
from reconstruction import *  # noqa: F401,F403
