"""Drop-in for ``consensus.cfa_ge_4stage`` (tensorflow1_implementations/consensus/cfa_ge_4stage.py).

The reference file is the first 385 lines of cfa_ge_2stage.py (the 4-stage negotiation
``getFederatedWeight_gradients`` without the fast variant); the same class serves both."""
from .cfa_ge_2stage import CFA_ge_process  # noqa: F401

__all__ = ["CFA_ge_process"]
