"""Drop-in for ``consensus.parameter_server`` (tensorflow2_implementations/MNIST_dataset/consensus/
parameter_server.py; identical in CIFAR_crossentropy). FedAvg over ``active`` devices drawn with
``random.sample`` (Python's RNG, consumed exactly as the reference), aggregation on the GPU.
The CIFAR100 / FL_radar / FL_over_MQTT copies (update_factor 0.99, no metalearning) are in
``parameter_server_099``."""
from __future__ import annotations

import os
import random

import numpy as np

from ._ps import PSBase, fedavg_into, load_retry
from ._runtime import pause


class Parameter_Server(PSBase):
    def __init__(self, devices, model_parameters, active_device_per_round, federated=True, graph=0, update_factor=1):
        self._init_common(devices, model_parameters, active_device_per_round, federated, graph, update_factor)
        self.outfile_gradients = ["results/dump_train_grad{}.npy".format(k) for k in range(devices)]

    def _fedavg_files(self, paths):
        stop = False
        models = []
        combined = 0
        for k in random.sample(range(self.devices), self.active):
            while not os.path.isfile(paths[k]):
                print("waiting")
                pause(1)
            m, ok = load_retry(paths[k], slot=("ps", len(models)))
            if ok:
                models.append(m)
            else:
                stop = True
            if not stop:
                combined += 1
        if combined > 0:
            print("Received models on the PS to combine {}".format(combined))
            fedavg_into(self.model_parameters, models[:combined], self.update_factor)
        return self.model_parameters

    def federated_metalearning(self, epoch=0, aggregation_type=0):
        """parameter_server.py:38-78: FedAvg of the devices' published gradients into the model."""
        if aggregation_type == 0:
            return self._fedavg_files(self.outfile_gradients)
        return self.model_parameters

    def federated_target_weights_aggregation(self, epoch=0, aggregation_type=0):
        """parameter_server.py:80-158: type 1 = copy the best device's model, type 0 = FedAvg."""
        if aggregation_type == 1:
            self._best_device(random.sample(range(self.devices), self.active))
            return self.model_parameters
        if aggregation_type == 0:
            return self._fedavg_files(self.outfile_models)
        return self.model_parameters
