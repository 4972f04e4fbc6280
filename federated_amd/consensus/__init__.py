"""Drop-in replacement of labRadioVision/federated's ``consensus`` package.

Same module names, classes, method signatures, argument orders, file protocol and return
tuples as the reference (tensorflow1_implementations/consensus and
tensorflow2_implementations/*/consensus); the mixing arithmetic runs in libcfa's HIP kernels.

TF1: cfa, cfa_mobilenet, cfa_ongraphs, cfa_ge_2stage, cfa_ge_4stage, cfa_ge_2stage_mobilenet
TF2: consensus_v2, consensus_v3, consensus_v3_threading, consensus_v4, parameter_server,
     parameter_server_v2

Use: replace ``from consensus.cfa import CFA_process`` with
``from federated_amd.consensus.cfa import CFA_process`` (or put federated_amd/ on sys.path
first and alias the package).
"""

import importlib
import sys

_TF1 = ("cfa", "cfa_mobilenet", "cfa_ongraphs", "cfa_ge_2stage", "cfa_ge_4stage", "cfa_ge_2stage_mobilenet")
_TF2 = ("consensus_v2", "consensus_v3", "consensus_v3_threading", "consensus_v4", "parameter_server",
        "parameter_server_v2")
_VARIANTS = {
    None: {},
    "fl_radar": {"consensus_v3": "fl_radar.consensus_v3", "consensus_v4": "fl_radar.consensus_v4",
                 "parameter_server": "parameter_server_099"},
    "fl_over_mqtt": {"consensus_v3": "fl_over_mqtt.consensus_v3", "parameter_server": "parameter_server_099"},
    "cifar100": {"parameter_server": "parameter_server_099"},
}


def install_as_consensus(variant=None):
    """Register these modules under the reference's import names, so an unmodified driver's
    ``from consensus.cfa_ongraphs import CFA_process`` (TF1) or
    ``from consensus.consensus_v3 import CFA_process`` (TF2) resolves to the GPU engine.
    ``variant`` selects a dataset directory's copy where they differ ("fl_radar",
    "fl_over_mqtt"). Call it before the driver imports ``consensus``."""
    if variant not in _VARIANTS:
        raise ValueError(f"unknown variant {variant!r}; expected one of {sorted(k for k in _VARIANTS if k)}")
    pkg = sys.modules[__name__]
    sys.modules["consensus"] = pkg
    for name in _TF1 + _TF2:
        target = _VARIANTS[variant].get(name, name)
        mod = importlib.import_module(f"{__name__}.{target}")
        sys.modules[f"consensus.{name}"] = mod
        setattr(pkg, name, mod)
    return pkg
