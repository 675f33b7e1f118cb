"""gslm -- host side of the MI355X Gaussian-splat LM hot path (render wrappers, solver, sharding).

Import order: `gslm._lib` loads libgslm.so eagerly (and fails loudly if it is missing); the
camera / model helpers are pure PyTorch host code and import without a GPU."""
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)
