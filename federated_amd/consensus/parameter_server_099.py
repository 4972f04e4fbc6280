"""Drop-in for the CIFAR100 / FL_radar / FL_over_MQTT copies of ``consensus.parameter_server``:
the MNIST module with update_factor defaulting to 0.99 (those copies lack
``federated_metalearning``; it is kept here as a harmless superset)."""
from __future__ import annotations

from .parameter_server import Parameter_Server as _PS


class Parameter_Server(_PS):
    def __init__(self, devices, model_parameters, active_device_per_round, federated=True, graph=0, update_factor=0.99):
        super().__init__(devices, model_parameters, active_device_per_round, federated, graph, update_factor)
