"""Drop-in for ``consensus.cfa_ge_2stage`` (tensorflow1_implementations/consensus/cfa_ge_2stage.py):
CFA with gradient exchange (CFA-GE), 4-stage (``getFederatedWeight_gradients``) and 2-stage/fast
(``getFederatedWeight_gradients_fast``) negotiation, as driven by
``federated_sample_CNN_CFA-GE.py:124-190``.

Stage 1 (CFA mix of the neighbours' models) and the gradient-bucket update (MEWMA filter + SGD
step with the neighbours' gradients) are libcfa kernels on fp64 buckets, the reference's own
numpy-2 arithmetic: ``cfa_mix_tf1_f64`` folds all neighbours in one pass,
``cfa_mewma_tf1_f64`` applies every neighbour's gradient and updates every saved state in one
pass ((3n + 2) * P * 8 bytes). Outputs are the reference's fp64 arrays, bit for bit. The neighbour-gradient
evaluation (a model forward/backward, not a reduction) runs through ``self.grad_fn``
(default: the torch restatement of the TF1 graph in ``_tf1_models``).
"""
from __future__ import annotations

import glob
import os

import numpy as np

from . import _tf1, _tf1_models
from ._runtime import loadmat_retry, mixer, pause, savemat_retry, wait_for


class CFA_ge_process:
    def get_connectivity(self, ii_saved_local, neighbors, devices):
        """cfa_ge_2stage.py:14-32 (k-regular)."""
        return _tf1.kregular(ii_saved_local, neighbors, devices)

    def federated_weights_computing2(self, filename, filename2, ii, ii2, epoch, devices, neighbors,
                                     eps_t_control):
        """Single-neighbour stage-1 step (cfa_ge_2stage.py:42-100), kept for API compatibility."""
        wait_for(filename2)
        cur = _tf1.model_from_mat(loadmat_retry(filename2))
        wait_for(filename)
        nbr = _tf1.model_from_mat(loadmat_retry(filename))
        a = eps_t_control * _tf1.weight_factor(devices, ii, ii2, neighbors - 1)
        (W1, b1, W2, b2), _ = _tf1.gpu_mix(cur, [nbr], [a])
        savemat_retry("temp_datamat{}_{}.mat".format(ii, epoch),
                      {"weights1": W1, "biases1": b1, "weights2": W2, "biases2": b2})
        return W1, b1, W2, b2

    def __init__(self, federated, devices, ii_saved_local, neighbors, mewma):
        self.federated = federated
        self.devices = devices
        self.ii_saved_local = ii_saved_local
        self.neighbors = neighbors
        self.mewma = mewma  # MEWMA parameter rho
        self.neighbor_vec = self.get_connectivity(ii_saved_local, neighbors, devices)
        self.grad_fn = None  # optional override: f(x, y, W1, b1, W2, b2) -> [gW1, gb1, gW2, gb2]

    def setCNNparameters(self, filter, number, pooling, stride, multip, classes, input_data):
        self.filter = filter
        self.number = number
        self.pooling = pooling
        self.stride = stride
        self.multip = multip
        self.classes = classes
        self.input_data = input_data
        self.ML_model = 1

    def set2NNparameters(self, intermediate_nodes, classes, input_data):
        self.intermediate_nodes = intermediate_nodes
        self.classes = classes
        self.input_data = input_data
        self.ML_model = 2

    # -- helpers ----------------------------------------------------------------------------
    def _grad_shapes(self):
        D = self.devices
        if self.ML_model == 1:
            return ([self.filter, 1, self.number, D], [self.number, D],
                    [self.multip * self.number, self.classes, D], [self.classes, D])
        return ([self.input_data, self.intermediate_nodes, D], [self.intermediate_nodes, D],
                [self.intermediate_nodes, self.classes, D], [self.classes, D])

    def _gradients(self, x, y, model):
        W1, b1, W2, b2 = model
        if self.grad_fn is not None:
            return self.grad_fn(x, y, W1, b1, W2, b2)
        return _tf1_models.gradients(self.ML_model, x, y, W1, b1, W2, b2,
                                     stride=getattr(self, "stride", 1))

    def _stage1_mix(self, local4, nbr_vec, epoch, eps):
        models, _, _ = _tf1.load_neighbour_models(nbr_vec, epoch - 1)
        alphas = [eps * _tf1.weight_factor(self.devices, self.ii_saved_local, int(j), self.neighbors - 1)
                  for j in nbr_vec]
        if not models:
            return list(local4)
        (W1, b1, W2, b2), _ = _tf1.gpu_mix(local4, models, alphas)
        return [W1, b1, W2, b2]

    def _publish_gradients(self, x, y, nbr_vec, model_epoch, grad_epoch):
        """Gradients of the local cost at each neighbour's datamat{j}_{model_epoch} model, in slot j
        of [..., devices] buckets, published as datagrad{ii}_{grad_epoch}.mat (:480-547)."""
        gv = [np.zeros(s) for s in self._grad_shapes()]
        models = []
        for j in nbr_vec:  # the neighbours' models, loaded in the reference's order
            fname = "datamat{}_{}.mat".format(int(j), model_epoch)
            wait_for(fname)
            try:
                content = loadmat_retry(fname)
            except Exception:
                pause(5)
                content = loadmat_retry(fname)
            models.append([np.asarray(content["weights1"]), np.squeeze(np.asarray(content["biases1"])),
                           np.asarray(content["weights2"]), np.squeeze(np.asarray(content["biases2"]))])
        if self.grad_fn is not None:
            grads = [self._gradients(x, y, m) for m in models]
        else:  # every neighbour model in one batched forward/backward (f3)
            grads = _tf1_models.gradients_batched(self.ML_model, x, y, models,
                                                  stride=getattr(self, "stride", 1))
        for j, g in zip(nbr_vec, grads):
            for k in range(4):
                gv[k][..., int(j)] = np.asarray(g[k]).reshape(gv[k].shape[:-1])
        path = "datagrad{}_{}.mat".format(self.ii_saved_local, grad_epoch)
        savemat_retry(path, {"grad_weights1": gv[0], "grad_biases1": gv[1], "grad_weights2": gv[2],
                             "grad_biases2": gv[3], "epoch": grad_epoch})
        pause(5)

    def _neighbour_gradients(self, nbr_vec, grad_epoch):
        """Slot ii of each neighbour's datagrad{j}_{grad_epoch}.mat (:564-589)."""
        ii = self.ii_saved_local
        out = []
        for j in nbr_vec:
            fname = "datagrad{}_{}.mat".format(int(j), grad_epoch)
            wait_for(fname)
            c = loadmat_retry(fname)
            out.append([np.asarray(c["grad_weights1"])[..., ii], np.squeeze(np.asarray(c["grad_biases1"]))[..., ii],
                        np.asarray(c["grad_weights2"])[..., ii], np.squeeze(np.asarray(c["grad_biases2"]))[..., ii]])
        return out

    # hooks overridden by the mobile-network variant (cfa_ge_2stage_mobilenet.py)
    def _round_neighbors(self, epoch):
        return self.get_connectivity(self.ii_saved_local, self.neighbors, self.devices)

    def _states_for_update(self, states, n):
        return states

    def _update(self, W4, states, grads, lr1, lr2, init, use_filtered):
        W = mixer().mewma_tf1(W4, states, grads, self.mewma, (lr1, lr1, lr2, lr2), init, use_filtered)
        return _tf1.squeeze_out(*W)

    # -- 4-stage ------------------------------------------------------------------------------
    def getFederatedWeight_gradients(self, n_W_l1, n_W_l2, n_b_l1, n_b_l2, epoch, v_loss, eng,
                                     x_train2, y_train2, W_l1_saved, W_l2_saved, n_l1_saved,
                                     n_l2_saved, eps_t_control, learning_rate1, learning_rate2):
        """cfa_ge_2stage.py:129-385: (1) CFA mix with the epoch-1 models, published as
        datamat{ii}_{epoch}; (2) gradients of the local cost at the neighbours' epoch models ->
        datagrad{ii}_{epoch}; (3) W -= lr * g_j with the neighbours' gradients, the saved states
        set to g_j at epoch 1 and MEWMA-filtered afterwards (states do not enter W here)."""
        ii = self.ii_saved_local
        if not (self.federated and self.devices > 1):
            return n_W_l1, n_b_l1, n_W_l2, n_b_l2, W_l1_saved, W_l2_saved, n_l1_saved, n_l2_saved
        if epoch == 0:
            _tf1.publish(ii, epoch, n_W_l1, n_b_l1, n_W_l2, n_b_l2, epoch=epoch, loss_sample=v_loss)
            return n_W_l1, n_b_l1, n_W_l2, n_b_l2, W_l1_saved, W_l2_saved, n_l1_saved, n_l2_saved
        nbr_vec = self._round_neighbors(epoch)
        if len(nbr_vec) == 0:  # :203-211: the publish of the unassigned result fails, is retried once, raises
            print("Unable to save file .. retrying")
            pause(3)
            raise _tf1.no_neighbour_error()
        W = self._stage1_mix([n_W_l1, n_b_l1, n_W_l2, n_b_l2], nbr_vec, epoch, eps_t_control)
        _tf1.publish(ii, epoch, *W)  # the MIXED model (:203-211)
        wait_for("datamat{}_{}.mat".format(ii, epoch))
        pause(3)
        self._publish_gradients(x_train2, y_train2, nbr_vec, epoch, epoch)
        pause(5)
        grads = self._neighbour_gradients(nbr_vec, epoch)
        states = self._states_for_update([W_l1_saved, n_l1_saved, W_l2_saved, n_l2_saved], len(nbr_vec))
        W = self._update(W, states, grads, learning_rate1, learning_rate2, init=(epoch == 1),
                         use_filtered=False)
        return (*W, states[0], states[2], states[1], states[3])

    # -- 2-stage (fast) -----------------------------------------------------------------------
    def getFederatedWeight_gradients_fast(self, n_W_l1, n_W_l2, n_b_l1, n_b_l2, epoch, v_loss, eng,
                                          x_train2, y_train2, W_l1_saved, W_l2_saved, n_l1_saved,
                                          n_l2_saved, eps_t_control, learning_rate1, learning_rate2):
        """cfa_ge_2stage.py:388-635: (1) CFA mix with the epoch-1 models; publish the PRE-mix
        model as datamat{ii}_{epoch}; (2) gradients of the local cost at the neighbours' epoch-1
        models -> datagrad{ii}_{epoch}; (3) with the neighbours' epoch-1 gradients g_j (slot ii):
        s_j <- rho g_j + (1-rho) s_j, W <- W - lr * s_j (CNN) or W - lr * g_j (2NN)."""
        ii = self.ii_saved_local
        if not (self.federated and self.devices > 1):
            return n_W_l1, n_b_l1, n_W_l2, n_b_l2, W_l1_saved, W_l2_saved, n_l1_saved, n_l2_saved
        if epoch == 0:
            _tf1.publish(ii, epoch, n_W_l1, n_b_l1, n_W_l2, n_b_l2, epoch=epoch, loss_sample=v_loss)
            return n_W_l1, n_b_l1, n_W_l2, n_b_l2, W_l1_saved, W_l2_saved, n_l1_saved, n_l2_saved
        nbr_vec = self._round_neighbors(epoch)
        if len(nbr_vec) == 0:  # :463 reads the result the empty neighbour loop never assigned
            raise _tf1.no_neighbour_error()
        W = self._stage1_mix([n_W_l1, n_b_l1, n_W_l2, n_b_l2], nbr_vec, epoch, eps_t_control)
        pause(3)
        _tf1.publish(ii, epoch, n_W_l1, n_b_l1, n_W_l2, n_b_l2)  # PRE-mix model (:470-478)
        self._publish_gradients(x_train2, y_train2, nbr_vec, epoch - 1, epoch)
        if epoch >= 9:  # cache GC (:550-558)
            for path in glob.glob("datagrad{}_{}.mat".format(ii, epoch - 8), recursive=False):
                try:
                    os.remove(path)
                except OSError:
                    print("Error while deleting file")
        pause(5)
        grads = self._neighbour_gradients(nbr_vec, epoch - 1)
        states = self._states_for_update([W_l1_saved, n_l1_saved, W_l2_saved, n_l2_saved], len(nbr_vec))
        W = self._update(W, states, grads, learning_rate1, learning_rate2, init=False,
                         use_filtered=(self.ML_model == 1))
        return (*W, states[0], states[2], states[1], states[3])
