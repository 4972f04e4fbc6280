"""Drop-in for ``consensus.parameter_server_v2`` (identical in all five TF2 dataset directories):
FedAvg over the scheduled devices ``indexes_tx[:, epoch]`` with staleness and training_end
handling (parameter_server_v2.py:39-165); the aggregation is one libcfa launch."""
from __future__ import annotations

import os
import random

import numpy as np

from .. import npyfile
from ._ps import PSBase, fedavg_into, load_retry
from ._runtime import pause


class Parameter_Server(PSBase):
    def __init__(self, devices, model_parameters, active_device_per_round, indexes_tx, federated=True, graph=0,
                 update_factor=0.99):
        self._init_common(devices, model_parameters, active_device_per_round, federated, graph, update_factor)
        self.indexes_tx = indexes_tx
        self.training_end = np.zeros(self.devices, dtype=bool)
        self.epoch_count = 0

    def _load_status(self, k):
        d = npyfile.load(self.outfile[k])
        return d["epoch_count"], d["training_end"]

    def federated_target_weights_aggregation(self, epoch, aggregation_type=0):
        if aggregation_type == 1:
            self._best_device(random.sample(range(self.devices), self.active))
            return self.model_parameters
        if aggregation_type != 0:
            return self.model_parameters
        stop = False
        combined = 0
        models, ended = [], []
        nbr_count = 0
        for k in self.indexes_tx[:, epoch]:
            while not os.path.isfile(self.outfile[k]):
                print("waiting on server")
                pause(1)
            try:
                nbr_count, self.training_end[k] = self._load_status(k)
            except Exception:
                pause(5)
                print("retrying opening variables on server")
                try:
                    nbr_count, self.training_end[k] = self._load_status(k)
                except Exception:
                    print("failed opening variables on server")
            while not os.path.isfile(self.outfile_models[k]) or nbr_count < epoch and not self.training_end[k]:
                print("waiting")
                pause(1)
                try:
                    nbr_count, self.training_end[k] = self._load_status(k)
                except Exception:
                    pause(5)
                    print("retrying opening variables on server")
                    try:
                        nbr_count, self.training_end[k] = self._load_status(k)
                    except Exception:
                        print("failed opening variables on server")
            m, ok = load_retry(self.outfile_models[k], slot=("ps", len(models)))
            if ok:
                models.append(m)
            else:
                stop = True
            if not stop:
                combined += 1
                ended.append(self.training_end[k])
        if combined > 0:
            print("Received models on the PS to combine {}".format(combined))
            ended = np.asarray(ended)
            if np.sum(ended) > 0:
                print("Training ended on below devices, transfer learning active:")
                first = int(np.asarray(np.nonzero(ended), dtype=int)[0][0])
                print(first)
                # p <- p + u * (x_first_ended - p), no division (:150-157)
                fedavg_into(self.model_parameters, [models[first]], self.update_factor, divide=False)
            else:
                fedavg_into(self.model_parameters, models[:combined], self.update_factor)
        return self.model_parameters
