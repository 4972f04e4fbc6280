"""Drop-in for ``consensus.cfa_ongraphs`` (tensorflow1_implementations/consensus/cfa_ongraphs.py):
CFA on time-varying graphs with consensus modes 0/1 and the parameter-compression epilogue, as
driven by ``FL_CFA_CNN_tf2.py:159-266``.

The neighbour mix and the compression epilogue run fused in ONE libcfa kernel
(``cfa_mix_seq_compress_f32``): the W2 segment of the bucket is compressed against the pre-mix
local W2 while the mixed value is still in registers, and the kept-parameter count is reduced
on the GPU (the reference runs a Python double loop, ~3 us/element, :225-273).
"""
from __future__ import annotations

import time

import numpy as np

from . import _tf1
from ._runtime import loadmat_retry, mixer, pause, savemat_retry, wait_for

W2 = 2  # layer index of weights2 in the (W1, b1, W2, b2) bucket


class CFA_process:
    def getRandomNetwork_connectivity(self, ii_saved_local, neighbors, devices, epoch):
        """cfa_ongraphs.py:18-31."""
        return _tf1.random_neighbors(ii_saved_local, neighbors, devices)

    def getMobileNetwork_connectivity(self, ii_saved_local, max_neighbors, devices, graph):
        """cfa_ongraphs.py:33-52 (vGraph row, random.choices with replacement above max)."""
        return _tf1.mobile_neighbors(ii_saved_local, max_neighbors, devices, graph)

    def get_connectivity(self, ii_saved_local, neighbors, devices):
        """cfa_ongraphs.py:54-72 (k-regular)."""
        return _tf1.kregular(ii_saved_local, neighbors, devices)

    def federated_weights_computing2(self, filename, filename2, ii, ii2, epoch, devices, neighbors,
                                     eps_t_control):
        """Single-neighbour step of cfa_ongraphs.py:75-136 (alpha = eps * b/(b + n b)); returns
        (W1, b1, W2, b2, parameters_received, time_info). Kept for API compatibility."""
        pause(2)
        wait_for(filename2)
        cur = _tf1.model_from_mat(loadmat_retry(filename2))
        start = time.time()
        wait_for(filename)
        content = loadmat_retry(filename)
        received = content["counter_param"]
        a = eps_t_control * _tf1.weight_factor(devices, ii, ii2, neighbors)
        (W1, b1, W2_, b2), _ = _tf1.gpu_mix(cur, [_tf1.model_from_mat(content)], [a])
        time_info = time.time() - start
        savemat_retry("temp_datamat{}_{}.mat".format(ii, epoch),
                      {"weights1": W1, "biases1": b1, "weights2": W2_, "biases2": b2})
        return W1, b1, W2_, b2, received, time_info

    def __init__(self, federated, devices, ii_saved_local, neighbors, graph, compression, consensus_mode):
        self.federated = federated
        self.devices = devices
        self.ii_saved_local = ii_saved_local
        self.compression = compression
        self.max_neighbors = neighbors
        self.graph = graph
        self.neighbor_vec = np.asarray(0, dtype=int)
        self.neighbors = self.neighbor_vec.size  # = 1 until the first mixing call (:145-146)
        self.consensus_mode = consensus_mode

    def disable_consensus(self, federated):
        self.federated = federated

    def _select_neighbors(self, current_neighbor, stop_consensus):
        """cfa_ongraphs.py:173-187."""
        if self.graph == 0:  # k-degree network, degree = the previous call's neighbour count
            self.neighbor_vec = self.get_connectivity(self.ii_saved_local, self.neighbors, self.devices)
        elif self.consensus_mode == 0:
            if stop_consensus:
                self.neighbor_vec = np.asarray(current_neighbor, dtype=int)
            else:
                self.neighbor_vec = np.zeros(1, dtype=int)
                self.neighbor_vec[0] = current_neighbor
        elif self.consensus_mode == 1:
            self.neighbor_vec = np.asarray(current_neighbor, dtype=int)
        else:
            print("Unknown consensus mode profile, exiting")
            exit(1)
        self.neighbors = self.neighbor_vec.size

    def getFederatedWeight(self, n_W_l1, n_W_l2, n_b_l1, n_b_l2, epoch, v_loss, eps_t_control,
                           current_neighbor, stop_consensus):
        """cfa_ongraphs.py:152-314. Returns (W1, b1, W2, b2, counter_param, time_info,
        compression_time)."""
        ii = self.ii_saved_local
        if not self.federated:
            _tf1.publish(ii, epoch, n_W_l1, n_b_l1, n_W_l2, n_b_l2, epoch=epoch, loss_sample=v_loss,
                         counter_param=0)
            return n_W_l1, n_b_l1, n_W_l2, n_b_l2, 0, 0, 0
        if self.devices <= 1:
            return n_W_l1, n_b_l1, n_W_l2, n_b_l2, 0, 0, 0
        if epoch == 0:
            counter_param = n_W_l2.shape[0] * n_W_l2.shape[1]
            _tf1.publish(ii, epoch, n_W_l1, n_b_l1, n_W_l2, n_b_l2, epoch=epoch, loss_sample=v_loss,
                         counter_param=counter_param)
            return n_W_l1, n_b_l1, n_W_l2, n_b_l2, counter_param, 0, 0

        self._select_neighbors(current_neighbor, stop_consensus)
        compression_time = 0
        time_info = 0
        if self.neighbors > 0:
            models, _, waited = _tf1.load_neighbour_models(self.neighbor_vec, epoch - 1,
                                                           sleep_before=2, sleep_after=5)
            alphas = [eps_t_control * _tf1.weight_factor(self.devices, ii, int(j), self.neighbors)
                      for j in self.neighbor_vec]
            start = time.time()
            mode = self.compression if self.compression in (1, 2, 3, 4) else 0
            (W1, b1, W2_, b2), kept = _tf1.gpu_mix([n_W_l1, n_b_l1, n_W_l2, n_b_l2], models, alphas,
                                                   compress=(mode, W2))
            time_info = waited + (time.time() - start)
            if self.compression in (1, 2, 3, 4):
                compression_time = time.time() - start  # fused: the epilogue has no separate pass
            counter_param = kept
            W_up_l1, n_up_l1, W_up_l2, n_up_l2 = _tf1.squeeze_out(W1, b1, W2_, b2)
        else:
            # no neighbour: W_up_l2 IS the caller's n_W_l2, so the compression modifies it in
            # place, and the published model below carries the compressed W2 (:219-273, :282-291)
            W_up_l1, n_up_l1, W_up_l2, n_up_l2 = n_W_l1, n_b_l1, n_W_l2, n_b_l2
            if self.compression in (1, 2, 3, 4):
                start = time.time()
                y, counter_param = mixer().compress(n_W_l2, n_W_l2, self.compression)
                n_W_l2[...] = y
                compression_time = time.time() - start
            else:
                counter_param = n_W_l2.shape[0] * n_W_l2.shape[1]
        time_info = time_info + compression_time
        if stop_consensus:
            _tf1.publish(ii, epoch, n_W_l1, n_b_l1, n_W_l2, n_b_l2, counter_param=counter_param)
        return W_up_l1, n_up_l1, W_up_l2, n_up_l2, counter_param, time_info, compression_time
