"""federated_amd — MI355X-native consensus-reduction engine for CFA / CFA-GE federated learning.

Drop-in for the mixing step of labRadioVision/federated's ``consensus`` package: the Python
call surface is kept (``federated_amd.consensus``), the arithmetic runs in hand-written HIP
kernels for gfx950 (``federated_amd/csrc``) reached through the C-ABI in
``include/cfa_engine.h`` (``libcfa.so``), and sharded populations exchange buckets over RCCL.
"""
__version__ = "1.0.0"
