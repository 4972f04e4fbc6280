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
