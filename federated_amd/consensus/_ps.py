"""FedAvg parameter server shared by the parameter_server / parameter_server_v2 drop-ins.

The reference aggregates the C received models into the global model layer by layer:
p[q] <- p[q] + u * (x_k[q] - p[q]) / C for k = 0..C-1 (parameter_server_v2.py:159-161,
parameter_server.py:154). Here every received model is one bucket and the whole fold is ONE
libcfa launch (``cfa_mix_seq_div_f32``), rounding step for step like the fp32 numpy chain.
"""
from __future__ import annotations

import math
import os
import random

import numpy as np

from .. import npyfile
from ._runtime import mixer, pause


def fedavg_into(params, models, update_factor, divide=True):
    """params[q] <- fold_k(params[q] + u * (models[k][q] - params[q]) [/ C]) for every layer q,
    assigned into ``params`` (object array) as the reference does."""
    C = len(models)
    local = [np.asarray(params[q]) for q in range(len(params))]
    nbrs = [[np.asarray(m[q]) for q in range(len(params))] for m in models]
    out, _ = mixer().mix(local, nbrs, [update_factor] * C,
                         divisors=[float(C)] * C if divide else [1.0] * C)
    for q in range(len(params)):
        params[q] = out[q].reshape(np.shape(local[q]))


def load_retry(path, slot=None):
    """np.load of a peer's published object array (native reader, federated_amd/npyfile.py) with
    one retry after pause(5); ``slot`` as in npyfile.load (models the aggregation consumes)."""
    try:
        return npyfile.load(path, slot=slot), True
    except Exception:
        pause(5)
        print("retrying opening model on server")
        try:
            return npyfile.load(path, slot=slot), True
        except Exception:
            print("halting aggregation on server")
            return None, False


class PSBase:
    def _init_common(self, devices, model_parameters, active_device_per_round, federated, graph, update_factor):
        self.federated = federated
        self.devices = devices
        self.active = active_device_per_round
        self.model_parameters = model_parameters
        self.layers = self.model_parameters.size
        self.graph = graph
        self.update_factor = update_factor
        self.file_paths = []
        self.outfile_models = []
        self.outfile = []
        self.global_model = "results/model_global.npy"
        self.eps_t_control = 1 / devices
        self.loss = math.inf * np.ones(self.devices, dtype=float)
        for k in range(devices):
            self.outfile_models.append("results/dump_train_model{}.npy".format(k))
            self.outfile.append("results/dump_train_variables{}.npz".format(k))

    def _best_device(self, candidates):
        """aggregation_type 1 (parameter_server.py:83-116): copy the model of argmax(loss)."""
        stop = False
        for k in candidates:
            while not os.path.isfile(self.outfile[k]):
                print("waiting on server")
                pause(1)
            try:
                self.loss[k] = npyfile.load(self.outfile[k])["loss"]
            except Exception:
                pause(5)
                print("retrying opening variables on server")
                try:
                    self.loss[k] = npyfile.load(self.outfile[k])["loss"]
                except Exception:
                    print("failed opening variables on server")
        best = np.argmax(self.loss)
        print("Using model {} as target with running reward {}".format(best, self.loss[best]))
        while not os.path.isfile(self.outfile_models[int(best)]):
            print("waiting")
            pause(1)
        try:
            w = npyfile.load(self.outfile_models[int(best)])
        except Exception:
            pause(5)
            print("retrying opening model")
            try:
                w = npyfile.load(self.outfile_models[int(best)])
            except Exception:
                print("halting aggregation")
                stop = True
        if not stop:
            for q in range(self.layers):
                self.model_parameters[q] = w[q]

    def publish_global_model(self):
        np.save(self.global_model, self.model_parameters)
