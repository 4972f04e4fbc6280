"""Generate the golden fixtures in tests/golden/*.npz by RUNNING THE REFERENCE CODE.

Runs only in the build container (needs /root/reference, read-only; nothing from it is copied
into the repo). The reference's consensus modules are imported from their files with stub
`tensorflow`/`keras` modules (TF is absent here and only feeds the TF graph/gradient code, which
is not on the reduction path), `pause` patched to a no-op, bytecode writing disabled, and a
temporary working directory (the modules exchange models through files relative to cwd).

Inputs are seeded synthetic models of the reference drivers' shapes; every fixture stores the
inputs and the reference's outputs. Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import importlib.util
import os
import random
import shutil
import sys
import tempfile
import types
import zlib

sys.dont_write_bytecode = True
os.environ.setdefault("MPLBACKEND", "Agg")

import numpy as np  # noqa: E402
import scipy.io as sio  # noqa: E402

REF = os.environ.get("CFA_REFERENCE", "/root/reference")
TF1 = os.path.join(REF, "tensorflow1_implementations")
TF2 = os.path.join(REF, "tensorflow2_implementations")
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------------------
# Stubs for the absent TF / Keras packages
# --------------------------------------------------------------------------------------
class _Any:
    """Absorbs any graph-building call (tf.placeholder, tf.nn.conv1d, operators, ...)."""

    def __getattr__(self, name):
        return _Any()

    def __call__(self, *a, **k):
        return _Any()

    def _op(self, *a):
        return _Any()

    __add__ = __radd__ = __sub__ = __rsub__ = __mul__ = __rmul__ = __neg__ = __truediv__ = _op


class _Session:
    def __init__(self, *a, **k):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def run(self, fetches, feed_dict=None):
        # Gradient sessions (cfa_ge_2stage.py:512-518) feed only the device's own outgoing
        # datagrad file; the pinned update reads the synthetic neighbour datagrad files.
        if isinstance(fetches, list):
            return [np.float64(0.0)] * len(fetches)
        return None


def install_stubs():
    tf = types.ModuleType("tensorflow")
    for name in ("placeholder", "expand_dims", "reshape", "matmul", "reduce_mean", "reduce_sum",
                 "log", "clip_by_value", "global_variables_initializer", "float32", "Variable",
                 "random_normal", "zeros"):
        setattr(tf, name, _Any())
    tf.nn = _Any()
    tf.layers = _Any()
    tf.gradients = lambda xs, ys: [_Any() for _ in xs]
    tf.Session = _Session
    tf.convert_to_tensor = np.asarray
    keras_tf = types.ModuleType("tensorflow.keras")
    keras_tf.layers = _Any()
    keras_tf.models = _Any()
    tf.keras = keras_tf
    sys.modules["tensorflow"] = tf
    sys.modules["tensorflow.keras"] = keras_tf
    sys.modules["tensorflow.keras.layers"] = keras_tf.layers
    sys.modules["tensorflow.keras.models"] = keras_tf.models
    keras = types.ModuleType("keras")
    kutils = types.ModuleType("keras.utils")
    kutils.to_categorical = lambda *a, **k: None
    keras.utils = kutils
    sys.modules["keras"] = keras
    sys.modules["keras.utils"] = kutils


def load_ref(path: str, name: str):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.pause = lambda *a, **k: None
    return mod


class Workdir:
    """Temporary cwd with the layout the reference expects (consensus/vGraph.mat, results/)."""

    def __enter__(self):
        self.old = os.getcwd()
        self.dir = tempfile.mkdtemp(prefix="cfa_golden_")
        os.makedirs(os.path.join(self.dir, "consensus"))
        os.makedirs(os.path.join(self.dir, "results"))
        shutil.copy(os.path.join(TF1, "consensus", "vGraph.mat"), os.path.join(self.dir, "consensus"))
        os.chdir(self.dir)
        return self.dir

    def __exit__(self, *a):
        os.chdir(self.old)
        shutil.rmtree(self.dir, ignore_errors=True)


def f32(rng, shape, scale=1.0):
    return (rng.standard_normal(shape) * scale).astype(np.float32)


def save(name: str, **arrays):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KiB)")


# --------------------------------------------------------------------------------------
# a1: TF1 cfa.py (static k-regular), 2NN shapes of federated_sample_2NN_CFA.py:35-36,68-71
# --------------------------------------------------------------------------------------
SHAPES_2NN = [(512, 32), (32,), (32, 8), (8,)]          # W1, b1, W2, b2  (P = 16 680)
SHAPES_CNN_GE = [(16, 1, 8), (8,), (168, 8), (8,)]       # federated_sample_CNN_CFA-GE.py:36-42
SHAPES_ONGRAPHS = [(3, 3, 1, 4), (4,), (4096, 6), (6,)]  # FL_CFA_CNN_tf2.py:56-65,113-121
SHAPES_ONGRAPHS_SMALL = [(3, 3, 1, 4), (4,), (512, 6), (6,)]  # same layers, shorter W2


def gen_model(rng, shapes, scale=1.0):
    return [f32(rng, s, scale) for s in shapes]


def case_tf1_cfa():
    cfa = load_ref(os.path.join(TF1, "consensus", "cfa.py"), "ref_tf1_cfa")
    out = {}
    specs = [  # (tag, shapes, devices, N, eps, devices under test)
        ("2nn_K5_N2_eps1", SHAPES_2NN, 5, 2, 1.0, (0, 2, 4)),
        ("2nn_K4_N2_eps1", SHAPES_2NN, 4, 2, 1.0, (0, 1, 2, 3)),  # config 1: federated_sample_2NN_CFA.py:107
        ("cnn_K5_N2_eps05", SHAPES_CNN_GE, 5, 2, 0.5, (2,)),
        ("cnn_K5_N3_eps1", SHAPES_CNN_GE, 5, 3, 1.0, (0, 2, 4)),
        ("cnn_K8_N4_eps07", SHAPES_CNN_GE, 8, 4, 0.7, (0, 1, 3, 7)),
    ]
    for tag, shapes, K, N, eps, under_test in specs:
        rng = np.random.default_rng(zlib.crc32(tag.encode()))
        models0 = [gen_model(rng, shapes) for _ in range(K)]   # published at epoch 0
        models1 = [gen_model(rng, shapes) for _ in range(K)]   # local models at epoch 1
        for t in range(4):
            out[f"{tag}/e0_{t}"] = np.stack([m[t] for m in models0])
            out[f"{tag}/e1_{t}"] = np.stack([m[t] for m in models1])
        out[f"{tag}/meta"] = np.array([K, N], dtype=np.int64)
        out[f"{tag}/eps"] = np.array(eps)
        out[f"{tag}/under_test"] = np.array(under_test, dtype=np.int64)
        with Workdir():
            procs = [cfa.CFA_process(True, K, j, N) for j in range(K)]
            for j in range(K):
                W1, b1, W2, b2 = models0[j]
                procs[j].getFederatedWeight(W1, W2, b1, b2, 0, np.zeros(3), eps)
            for ii in under_test:
                W1, b1, W2, b2 = models1[ii]
                res = procs[ii].getFederatedWeight(W1, W2, b1, b2, 1, np.zeros(3), eps)
                out[f"{tag}/nbr_{ii}"] = np.asarray(procs[ii].neighbor_vec, dtype=np.int64)
                for t in range(4):
                    out[f"{tag}/out_{ii}_{t}"] = np.asarray(res[t])
    save("tf1_cfa.npz", **out)


# --------------------------------------------------------------------------------------
# a2/a3: TF1 cfa_ongraphs.py, FL_CFA_CNN_tf2 shapes, modes 0/1, compression 0..4
# --------------------------------------------------------------------------------------
def ongraphs_models(rng, K, shapes):
    """Models in the regime the compression thresholds act on: W2 small, and neighbours close
    to each other (W2 starts at zero in FL_CFA_CNN_tf2.py:197-199)."""
    base_W2 = f32(rng, shapes[2], 0.01)
    models = []
    for _ in range(K):
        m = gen_model(rng, shapes)
        m[2] = (base_W2 + f32(rng, shapes[2], 3e-4)).astype(np.float32)
        models.append(m)
    return models


def case_tf1_ongraphs():
    og = load_ref(os.path.join(TF1, "consensus", "cfa_ongraphs.py"), "ref_tf1_ongraphs")
    out = {}
    K = 5
    cases = []
    # (tag, shape set, ii, graph, mode, neighbour list, compression, eps)
    for comp in range(5):
        cases.append((f"m1_c{comp}_ii2", "small", 2, 6, 1, [1, 3], comp, 1.0))
    for comp in (1, 3):
        cases.append((f"m1_c{comp}_ii0_n3", "small", 0, 6, 1, [4, 1, 2], comp, 0.8))
    for comp in (0, 2, 4):
        cases.append((f"m0_c{comp}_ii3", "small", 3, 6, 0, [2, 4, 0], comp, 1.0))
    cases.append(("m1_c2_ii2_full", "full", 2, 6, 1, [1, 3], 2, 1.0))
    cases.append(("m1_c0_ii4_n1", "small", 4, 6, 1, [3], 0, 1.0))
    cases.append(("g0_m1_c2_ii0", "small", 0, 0, 1, [], 2, 1.0))
    out["cases"] = np.array([c[0] for c in cases])
    stacks = {}
    for kind, shapes in (("small", SHAPES_ONGRAPHS_SMALL), ("full", SHAPES_ONGRAPHS)):
        rng = np.random.default_rng(zlib.crc32(kind.encode()))
        m0 = ongraphs_models(rng, K, shapes)
        m1 = ongraphs_models(rng, K, shapes)
        sgd = [ongraphs_models(rng, K, shapes) for _ in range(3)]  # post-"SGD" models, mode-0 steps
        stacks[kind] = (m0, m1, sgd)
        for t in range(4):
            out[f"{kind}/e0_{t}"] = np.stack([m[t] for m in m0])
            out[f"{kind}/e1_{t}"] = np.stack([m[t] for m in m1])
            for r in range(3 if kind == "small" else 1):  # the full-shape case is mode 1 only
                out[f"{kind}/sgd{r}_{t}"] = np.stack([m[t] for m in sgd[r]])
    for tag, kind, ii, graph, mode, nbrs, comp, eps in cases:
        models0, models1, sgd = stacks[kind]
        with Workdir():
            procs = [og.CFA_process(True, K, j, 2, graph, comp, mode) for j in range(K)]
            for j in range(K):
                W1, b1, W2, b2 = models0[j]
                procs[j].getFederatedWeight(W1, W2, b1, b2, 0, np.zeros(3), eps, [], False)
            p = procs[ii]
            calls = []  # (kind, neighbour arg, input source tag, inputs, result)
            if mode == 1:
                plan = [("mix", nbrs, "e1"), ("stop", [], "sgd0")]
            else:
                plan = [("mix", j, "e1" if s == 0 else f"sgd{s - 1}") for s, j in enumerate(nbrs)]
                plan.append(("stop", [], "sgd2"))
            for ck, nb, src in plan:
                srcm = models1 if src == "e1" else sgd[int(src[3:])]
                W1, b1, W2, b2 = [a.copy() for a in srcm[ii]]
                res = p.getFederatedWeight(W1, W2, b1, b2, 1, np.zeros(3), eps, nb, ck == "stop")
                calls.append((ck, nb, src, W2, res))
            published = sio.loadmat(f"datamat{ii}_1.mat")
        out[f"{tag}/meta"] = np.array([ii, graph, mode, comp, len(calls)], dtype=np.int64)
        out[f"{tag}/kind"] = np.array(kind)
        out[f"{tag}/eps"] = np.array(eps)
        for c, (ck, nb, src, W2_after, res) in enumerate(calls):
            out[f"{tag}/call{c}_nbrs"] = np.atleast_1d(np.asarray(nb, dtype=np.int64))
            out[f"{tag}/call{c}_stop"] = np.array(ck == "stop")
            out[f"{tag}/call{c}_src"] = np.array(src)
            # The caller's W2 after the call: the reference compresses it IN PLACE when no
            # neighbour is mixed (W_up_l2 aliases n_W_l2, cfa_ongraphs.py:219-271).
            out[f"{tag}/call{c}_in2_after"] = np.asarray(W2_after)
            for t in range(4):
                out[f"{tag}/call{c}_out_{t}"] = np.asarray(res[t])
            out[f"{tag}/call{c}_counter"] = np.array(res[4], dtype=np.int64)
        for key in ("weights1", "biases1", "weights2", "biases2", "counter_param"):
            out[f"{tag}/pub_{key}"] = np.asarray(published[key])
    save("tf1_ongraphs.npz", **out)


def case_mobile_network():
    og = load_ref(os.path.join(TF1, "consensus", "cfa_ongraphs.py"), "ref_tf1_ongraphs_mn")
    v3 = load_v3()
    out = {}
    with Workdir():
        graph = sio.loadmat("consensus/vGraph.mat")["graph"]
        out["graph"] = np.asarray(graph)
        p = og.CFA_process(True, 5, 0, 2, 1, 0, 0)
        rows = []
        for g in range(graph.shape[2]):
            for ii in range(5):
                for mx in (1, 2, 3, 4):
                    seed = g * 1000 + ii * 10 + mx
                    random.seed(seed)
                    nb = p.getMobileNetwork_connectivity(ii, mx, 5, g)
                    rows.append((g, ii, mx, seed, list(np.asarray(nb, dtype=np.int64))))
        q = v3.CFA_process(5, 0, 2, graph=1)
        rows_v3 = []
        for g in range(graph.shape[2]):
            for ii in range(5):
                nb = q.getMobileNetwork_connectivity(ii, 2, 5, g)
                rows_v3.append((g, ii, list(np.asarray(nb, dtype=np.int64))))
    out["mn_keys"] = np.array([r[:4] for r in rows], dtype=np.int64)
    out["mn_len"] = np.array([len(r[4]) for r in rows], dtype=np.int64)
    out["mn_vals"] = np.array(sum((r[4] for r in rows), []), dtype=np.int64)
    out["v3_keys"] = np.array([r[:2] for r in rows_v3], dtype=np.int64)
    out["v3_len"] = np.array([len(r[2]) for r in rows_v3], dtype=np.int64)
    out["v3_vals"] = np.array(sum((r[2] for r in rows_v3), []), dtype=np.int64)
    save("topology_mobile.npz", **out)


# --------------------------------------------------------------------------------------
# a4: TF1 CFA-GE (cfa_ge_2stage.py fast + 4-stage), CNN (config 3) and 2NN models
# --------------------------------------------------------------------------------------
def case_tf1_cfa_ge():
    ge = load_ref(os.path.join(TF1, "consensus", "cfa_ge_2stage.py"), "ref_tf1_cfa_ge")
    out = {}
    K, N, rho, eps, lr1, lr2 = 16, 2, 0.99, 1.0, 0.1, 0.05
    shapes_2nn_small = [(64, 16), (16,), (16, 8), (8,)]
    specs = [("cnn", 1, SHAPES_CNN_GE), ("2nn", 2, shapes_2nn_small)]
    for model_tag, ml, shapes in specs:
        for variant, epoch in (("fast", 5), ("4stage_e1", 1), ("4stage_e3", 3)):
            for ii in (0, 7):
                tag = f"{model_tag}_{variant}_ii{ii}"
                rng = np.random.default_rng(zlib.crc32(tag.encode()))
                models_prev = [gen_model(rng, shapes) for _ in range(K)]
                models_cur = [gen_model(rng, shapes) for _ in range(K)]
                grad_epoch = epoch - 1 if variant == "fast" else epoch
                grads = []
                for j in range(K):
                    grads.append([rng.standard_normal(tuple(s) + (K,)) for s in shapes])
                local = gen_model(rng, shapes)
                states = [rng.standard_normal(tuple(s) + (N,)) for s in shapes]
                with Workdir():
                    p = ge.CFA_ge_process(True, K, ii, N, rho)
                    if ml == 1:
                        p.setCNNparameters(16, 8, 5, 5, 21, 8, 512)
                    else:
                        p.set2NNparameters(16, 8, 64)
                    nbr = p.get_connectivity(ii, N, K)
                    for j in range(K):
                        W1, b1, W2, b2 = models_prev[j]
                        sio.savemat(f"datamat{j}_{epoch - 1}.mat",
                                    {"weights1": W1, "biases1": b1, "weights2": W2, "biases2": b2})
                        if variant != "fast" and j != ii:
                            W1, b1, W2, b2 = models_cur[j]
                            sio.savemat(f"datamat{j}_{epoch}.mat",
                                        {"weights1": W1, "biases1": b1, "weights2": W2, "biases2": b2})
                        g = grads[j]
                        sio.savemat(f"datagrad{j}_{grad_epoch}.mat",
                                    {"grad_weights1": g[0], "grad_biases1": g[1], "grad_weights2": g[2],
                                     "grad_biases2": g[3], "epoch": grad_epoch})
                    st = [s.copy() for s in states]
                    W1, b1, W2, b2 = local
                    fn = p.getFederatedWeight_gradients_fast if variant == "fast" else p.getFederatedWeight_gradients
                    res = fn(W1, W2, b1, b2, epoch, np.zeros(3), 0, None, None, st[0], st[2], st[1], st[3],
                             eps, lr1, lr2)
                out[f"{tag}/meta"] = np.array([K, N, ii, epoch, ml], dtype=np.int64)
                out[f"{tag}/hyper"] = np.array([rho, eps, lr1, lr2])
                out[f"{tag}/nbr"] = np.asarray(nbr, dtype=np.int64)
                for t in range(4):
                    out[f"{tag}/local_{t}"] = local[t]
                    out[f"{tag}/state_in_{t}"] = states[t]
                    for q, j in enumerate(nbr):
                        out[f"{tag}/prev{q}_{t}"] = models_prev[j][t]
                        out[f"{tag}/grad{q}_{t}"] = grads[j][t][..., ii]  # the slot read
                    out[f"{tag}/out_{t}"] = np.asarray(res[t])
                # res[4:8] = W_l1_saved, W_l2_saved, n_l1_saved, n_l2_saved
                for t, r in zip((0, 2, 1, 3), res[4:8]):
                    out[f"{tag}/state_out_{t}"] = np.asarray(r)
    save("tf1_cfa_ge.npz", **out)


# --------------------------------------------------------------------------------------
# a5/a6: TF2 consensus_v2/v3/v4 (weights + gradients), lenet-1 layer list
# --------------------------------------------------------------------------------------
SHAPES_LENET1 = [(5, 5, 1, 4), (4,), (5, 5, 4, 8), (8,), (128, 10), (10,)]  # P = 2202


def load_v3():
    return load_ref(os.path.join(TF2, "MNIST_dataset", "consensus", "consensus_v3.py"), "ref_tf2_v3")


def obj_array(layers):
    a = np.empty(len(layers), dtype=object)
    for i, l in enumerate(layers):
        a[i] = l
    return a


def publish_tf2(k, layers, epoch_count, training_end, grads=None):
    np.save(f"results/dump_train_model{k}.npy", obj_array(layers), allow_pickle=True)
    np.savez(f"results/dump_train_variables{k}.npz", frame_count=epoch_count, epoch_count=epoch_count,
             training_end=training_end, loss=0.5)
    if grads is not None:
        np.save(f"results/dump_train_grad{k}.npy", obj_array(grads), allow_pickle=True)


def case_tf2():
    mods = {
        "v2": load_ref(os.path.join(TF2, "MNIST_dataset", "consensus", "consensus_v2.py"), "ref_tf2_v2"),
        "v3": load_v3(),
        "v4": load_ref(os.path.join(TF2, "MNIST_dataset", "consensus", "consensus_v4.py"), "ref_tf2_v4"),
        "v3radar": load_ref(os.path.join(TF2, "FL_radar_dataset", "consensus", "consensus_v3.py"), "ref_tf2_v3r"),
        "v3cifar": load_ref(os.path.join(TF2, "CIFAR100_dataset", "consensus", "consensus_v3.py"), "ref_tf2_v3c"),
    }
    out = {}
    D = 8
    rng = np.random.default_rng(777)
    models = [gen_model(rng, SHAPES_LENET1) for _ in range(D)]
    grads = [gen_model(rng, SHAPES_LENET1, 0.1) for _ in range(D)]
    local = gen_model(rng, SHAPES_LENET1)
    local_g = gen_model(rng, SHAPES_LENET1, 0.1)
    for t in range(len(SHAPES_LENET1)):
        out[f"models_{t}"] = np.stack([m[t] for m in models])
        out[f"grads_{t}"] = np.stack([g[t] for g in grads])
        out[f"local_{t}"] = local[t]
        out[f"local_g_{t}"] = local_g[t]
    cases = [
        # (tag, module, kind, neighbour arg, neighbors arg, eps, training_end devices)
        ("v3_w_n2", "v3", "w", [1, 2], 2, 0.7, ()),
        ("v3_w_n3", "v3", "w", [5, 1, 6], 3, 0.2, ()),
        ("v3_w_end", "v3", "w", [1, 2, 3], 3, 0.5, (2,)),
        ("v2_w_n2", "v2", "w", [3, 4], 2, 0.5, ()),
        ("v3cifar_w_n4", "v3cifar", "w", [0, 2, 4, 6], 4, 0.2, ()),
        ("v3radar_w_n2", "v3radar", "w", [6, 7], 2, 0.5, ()),
        ("v4_w_n2", "v4", "w", [2, 4], 2, 0.5, ()),
        ("v4_w_ring", "v4", "w", 3, 1, 0.5, ()),
        ("v4_w_end", "v4", "w", [5, 6, 7], 3, 0.5, (6,)),
        ("v3_g_n2", "v3", "g", [1, 2], 2, 0.5, ()),
        ("v4_g_n2", "v4", "g", [3, 4], 2, 0.5, ()),
        ("v4_g_ring", "v4", "g", 5, 1, 0.3, ()),
    ]
    out["cases"] = np.array([c[0] for c in cases])
    for tag, modname, kind, nbr, nnb, eps, ended in cases:
        mod = mods[modname]
        with Workdir():
            for k in range(D):
                publish_tf2(k, models[k], 10, k in ended, grads[k])
            if modname in ("v2", "v3", "v3radar", "v3cifar"):
                p = mod.CFA_process(D, 0, 2)
            else:
                p = mod.CFA_process(D, 0, 2)
            np.random.seed(123)
            if kind == "w":
                loc = obj_array([a.copy() for a in local])
                p.update_local_model(loc)
                res = p.federated_weights_computing(nbr, nnb, 10, eps, 0, 30)
                inplace = [np.asarray(a) for a in loc]
            else:
                loc = obj_array([a.copy() for a in local])
                p.update_local_model(loc)
                gl = obj_array([a.copy() for a in local_g])
                p.update_local_gradient(gl)
                if modname == "v4":
                    res = p.federated_grads_computing(nbr, nnb, 10, eps, 1)
                else:
                    res = p.federated_grads_computing(nbr, nnb, 10, eps, 0, 30)
                inplace = [np.asarray(a) for a in gl]
            probe = np.random.random()
            status = bool(p.getTrainingStatusFromNeightbor())
        out[f"{tag}/nbr"] = np.atleast_1d(np.asarray(nbr, dtype=np.int64))
        out[f"{tag}/meta"] = np.array([nnb, int(status)], dtype=np.int64)
        out[f"{tag}/eps"] = np.array(eps)
        out[f"{tag}/rng_probe"] = np.array(probe)
        out[f"{tag}/ended"] = np.array(ended, dtype=np.int64)
        for t in range(len(SHAPES_LENET1)):
            out[f"{tag}/out_{t}"] = np.asarray(res[t])
            out[f"{tag}/inplace_{t}"] = inplace[t]
    save("tf2_consensus.npz", **out)


def case_variants():
    """Copies not covered above: TF1 cfa_mobilenet.py over several epochs of the vGraph mobile
    network; the CIFAR100 consensus_v3_threading.py (mixing under a caller lock); the
    FL_over_MQTT consensus_v3.py, whose constructor reads an undefined global `devices`
    (NameError as shipped; run here with that global injected to record its outputs)."""
    import threading
    out = {}
    # -- cfa_mobilenet: 5 devices (vGraph is 5 x 5 x 111), epochs 0..3, every device each epoch
    mn = load_ref(os.path.join(TF1, "consensus", "cfa_mobilenet.py"), "ref_tf1_cfa_mn")
    K, N, eps = 5, 2, 0.8
    rng = np.random.default_rng(4242)
    epochs = 4
    locals_ = [[gen_model(rng, SHAPES_CNN_GE) for _ in range(K)] for _ in range(epochs)]
    for e in range(epochs):
        for t in range(4):
            out[f"mobilenet/local_e{e}_{t}"] = np.stack([m[t] for m in locals_[e]])
    out["mobilenet/meta"] = np.array([K, N, epochs], dtype=np.int64)
    out["mobilenet/eps"] = np.array(eps)
    with Workdir():
        procs = [mn.CFA_process(True, K, j, N) for j in range(K)]
        for e in range(epochs):
            for j in range(K):
                W1, b1, W2, b2 = locals_[e][j]
                res = procs[j].getFederatedWeight(W1, W2, b1, b2, e, np.zeros(3), eps)
                if e > 0:
                    out[f"mobilenet/nbr_e{e}_{j}"] = np.asarray(procs[j].neighbor_vec, dtype=np.int64)
                for t in range(4):
                    out[f"mobilenet/out_e{e}_{j}_{t}"] = np.asarray(res[t])
    # -- TF2 copies: the same published population and local model as case_tf2's layer list
    D = 6
    rng = np.random.default_rng(5151)
    models = [gen_model(rng, SHAPES_LENET1) for _ in range(D)]
    local = gen_model(rng, SHAPES_LENET1)
    for t in range(len(SHAPES_LENET1)):
        out[f"tf2/models_{t}"] = np.stack([m[t] for m in models])
        out[f"tf2/local_{t}"] = local[t]
    thr = load_ref(os.path.join(TF2, "CIFAR100_dataset", "consensus", "consensus_v3_threading.py"), "ref_tf2_v3t")
    mq = load_ref(os.path.join(TF2, "FL_over_MQTT", "consensus", "consensus_v3.py"), "ref_tf2_v3mqtt")
    try:
        mq.CFA_process(0, 2)
        out["mqtt/ctor_raises_nameerror"] = np.array(False)
    except NameError:
        out["mqtt/ctor_raises_nameerror"] = np.array(True)
    mq.devices = D  # the global the shipped constructor expects
    rv4 = load_ref(os.path.join(TF2, "FL_radar_dataset", "consensus", "consensus_v4.py"), "ref_tf2_v4radar")
    cases = [("threading_n3", "thr", [1, 3, 5], 3, ()), ("threading_end", "thr", [2, 4], 2, (4,)),
             ("mqtt_n2", "mq", [4, 5], 2, ()), ("mqtt_end", "mq", [1, 2, 3], 3, (1,)),
             # FL_radar v4: one neighbour id, read `neighbors` times (consensus_v4.py:88-89)
             ("radar_v4_n1", "rv4", 3, 1, ()), ("radar_v4_n2", "rv4", 5, 2, ()),
             ("radar_v4_end", "rv4", 2, 2, (2,))]
    out["tf2/cases"] = np.array([c[0] for c in cases])
    for tag, which, nbr, nnb, ended in cases:
        with Workdir():
            for k in range(D):
                publish_tf2(k, models[k], 10, k in ended)
            if which == "thr":
                p = thr.CFA_process(threading.Lock(), D, 0, 2)
            elif which == "mq":
                p = mq.CFA_process(0, 2)
            else:
                p = rv4.CFA_process(D, 0, 1)
            np.random.seed(321)
            loc = obj_array([a.copy() for a in local])
            p.update_local_model(loc)
            res = p.federated_weights_computing(nbr, nnb, 10, 0.5, 0, 30)
            probe = np.random.random()
        out[f"tf2/{tag}/nbr"] = np.asarray(nbr, dtype=np.int64)
        out[f"tf2/{tag}/nnb"] = np.array(nnb, dtype=np.int64)
        out[f"tf2/{tag}/ended"] = np.array(ended, dtype=np.int64)
        out[f"tf2/{tag}/rng_probe"] = np.array(probe)
        for t in range(len(SHAPES_LENET1)):
            out[f"tf2/{tag}/out_{t}"] = np.asarray(res[t])
            out[f"tf2/{tag}/inplace_{t}"] = np.asarray(loc[t])
    save("variants.npz", **out)


def case_topology():
    cfa = load_ref(os.path.join(TF1, "consensus", "cfa.py"), "ref_tf1_cfa_topo")
    v3 = load_v3()
    v4 = load_ref(os.path.join(TF2, "MNIST_dataset", "consensus", "consensus_v4.py"), "ref_tf2_v4_topo")
    rows = {"tf1": [], "v3": [], "v4": [], "v4tx": []}
    for K in (4, 5, 8, 16, 32, 128):  # K = 4: config 1's population
        for N in (1, 2, 3, 4):
            p1 = cfa.CFA_process(True, K, 0, N)
            p3 = v3.CFA_process(K, 0, N)
            p4 = v4.CFA_process(K, 0, N)
            for ii in range(K):
                rows["tf1"].append((K, N, ii, np.atleast_1d(p1.get_connectivity(ii, N, K))))
                rows["v3"].append((K, N, ii, np.atleast_1d(p3.get_connectivity(ii, N, K))))
                rows["v4"].append((K, N, ii, np.atleast_1d(p4.get_connectivity(ii, N, K))))
                rows["v4tx"].append((K, N, ii, np.atleast_1d(p4.get_tx_connectivity(ii, N, K))))
    out = {}
    for name, r in rows.items():
        out[f"{name}_keys"] = np.array([x[:3] for x in r], dtype=np.int64)
        out[f"{name}_len"] = np.array([len(x[3]) for x in r], dtype=np.int64)
        out[f"{name}_vals"] = np.concatenate([np.asarray(x[3], dtype=np.int64) for x in r])
    save("topology_kregular.npz", **out)


def case_tf1_cfa_ge_mobilenet():
    ge = load_ref(os.path.join(TF1, "consensus", "cfa_ge_2stage_mobilenet.py"), "ref_tf1_cfa_ge_mn")
    out = {}
    K, N, rho, eps, lr1, lr2 = 5, 2, 0.99, 1.0, 0.1, 0.05
    for variant, epoch in (("fast", 5), ("4stage_e1", 1), ("4stage_e3", 3)):
        ii = 2
        tag = f"cnn_{variant}"
        rng = np.random.default_rng(zlib.crc32(("mn" + tag).encode()))
        with Workdir():
            graph = sio.loadmat("consensus/vGraph.mat")["graph"]
            nbr = [kk for kk in range(K) if graph[ii, kk, epoch] == 1]
            grad_epoch = epoch - 1 if variant == "fast" else epoch
            prev = {j: gen_model(rng, SHAPES_CNN_GE) for j in range(K)}
            grads = {j: [rng.standard_normal(tuple(s) + (K,)) for s in SHAPES_CNN_GE] for j in range(K)}
            for j in range(K):
                W1, b1, W2, b2 = prev[j]
                sio.savemat(f"datamat{j}_{epoch - 1}.mat", {"weights1": W1, "biases1": b1, "weights2": W2, "biases2": b2})
                if variant != "fast" and j != ii:
                    sio.savemat(f"datamat{j}_{epoch}.mat", {"weights1": W1, "biases1": b1, "weights2": W2, "biases2": b2})
                g = grads[j]
                sio.savemat(f"datagrad{j}_{grad_epoch}.mat", {"grad_weights1": g[0], "grad_biases1": g[1],
                                                             "grad_weights2": g[2], "grad_biases2": g[3]})
            local = gen_model(rng, SHAPES_CNN_GE)
            states = [np.zeros(tuple(s) + (N,)) for s in SHAPES_CNN_GE]
            p = ge.CFA_ge_process(True, K, ii, N, rho)
            p.setCNNparameters(16, 8, 5, 5, 21, 8, 512)
            fn = p.getFederatedWeight_gradients_fast if variant == "fast" else p.getFederatedWeight_gradients
            W1, b1, W2, b2 = local
            res = fn(W1, W2, b1, b2, epoch, np.zeros(3), 0, None, None, states[0], states[2], states[1], states[3],
                     eps, lr1, lr2)
        out[f"{tag}/meta"] = np.array([K, N, ii, epoch], dtype=np.int64)
        out[f"{tag}/hyper"] = np.array([rho, eps, lr1, lr2])
        out[f"{tag}/nbr"] = np.asarray(nbr, dtype=np.int64)
        for t in range(4):
            out[f"{tag}/local_{t}"] = local[t]
            for j in nbr:
                out[f"{tag}/prev{j}_{t}"] = prev[j][t]
                out[f"{tag}/grad{j}_{t}"] = grads[j][t][..., ii]
            out[f"{tag}/out_{t}"] = np.asarray(res[t])
        for t, r in zip((0, 2, 1, 3), res[4:8]):
            out[f"{tag}/state_out_{t}"] = np.asarray(r)
    save("tf1_cfa_ge_mobilenet.npz", **out)


# --------------------------------------------------------------------------------------
# f1: TF2 FedAvg parameter servers (parameter_server.py, parameter_server_v2.py)
# --------------------------------------------------------------------------------------
def case_parameter_server():
    ps1 = load_ref(os.path.join(TF2, "MNIST_dataset", "consensus", "parameter_server.py"), "ref_ps1")
    ps1c = load_ref(os.path.join(TF2, "CIFAR100_dataset", "consensus", "parameter_server.py"), "ref_ps1c")
    ps2 = load_ref(os.path.join(TF2, "MNIST_dataset", "consensus", "parameter_server_v2.py"), "ref_ps2")
    out = {}
    D = 7
    rng = np.random.default_rng(99)
    models = [gen_model(rng, SHAPES_LENET1) for _ in range(D)]
    grads = [gen_model(rng, SHAPES_LENET1, 0.1) for _ in range(D)]
    glob_ = gen_model(rng, SHAPES_LENET1)
    losses = rng.random(D)
    indexes_tx = np.stack([rng.permutation(D)[:4] for _ in range(5)], axis=1)  # [active, epochs]
    for t in range(len(SHAPES_LENET1)):
        out[f"models_{t}"] = np.stack([m[t] for m in models])
        out[f"grads_{t}"] = np.stack([g[t] for g in grads])
        out[f"global_{t}"] = glob_[t]
    out["losses"] = losses
    out["indexes_tx"] = indexes_tx
    cases = [  # (tag, module, method, aggregation_type, active, update_factor, epoch, ended)
        ("ps1_avg", "ps1", "w", 0, 3, 1, 0, ()),
        ("ps1_avg_u099", "ps1", "w", 0, 5, 0.99, 0, ()),
        ("ps1_best", "ps1", "w", 1, 4, 1, 0, ()),
        ("ps1_meta", "ps1", "meta", 0, 4, 1, 0, ()),
        ("ps1c_avg", "ps1c", "w", 0, 3, None, 0, ()),
        ("ps2_avg", "ps2", "w", 0, 4, None, 2, ()),
        ("ps2_avg_u1", "ps2", "w", 0, 4, 1, 3, ()),
        ("ps2_end", "ps2", "w", 0, 4, None, 1, (int(indexes_tx[2, 1]),)),
    ]
    out["cases"] = np.array([c[0] for c in cases])
    mods = {"ps1": ps1, "ps1c": ps1c, "ps2": ps2}
    for tag, modname, method, agg, active, u, epoch, ended in cases:
        with Workdir():
            for k in range(D):
                publish_tf2(k, models[k], 10, k in ended, grads[k])
                np.savez(f"results/dump_train_variables{k}.npz", epoch_count=10, training_end=k in ended,
                         loss=losses[k])
            params = obj_array([a.copy() for a in glob_])
            kw = {} if u is None else {"update_factor": u}
            if modname == "ps2":
                p = mods[modname].Parameter_Server(D, params, active, indexes_tx, **kw)
            else:
                p = mods[modname].Parameter_Server(D, params, active, **kw)
            random.seed(5)
            if method == "meta":
                res = p.federated_metalearning(epoch, agg)
            else:
                res = p.federated_target_weights_aggregation(epoch, agg)
            probe = random.random()
        out[f"{tag}/meta"] = np.array([agg, active, epoch], dtype=np.int64)
        out[f"{tag}/u"] = np.array(-1.0 if u is None else u)
        out[f"{tag}/ended"] = np.array(ended, dtype=np.int64)
        out[f"{tag}/rng_probe"] = np.array(probe)
        for t in range(len(SHAPES_LENET1)):
            out[f"{tag}/out_{t}"] = np.asarray(res[t])
    save("tf2_parameter_server.npz", **out)


# --------------------------------------------------------------------------------------
# f1: aggregation loops embedded in drivers (PS_server.py, learner_consensus.py,
# federated_sample_CNN_CFA_FA.py). The drivers cannot be imported (argparse at import, TF
# graphs, MQTT sockets), so the cited statements are read from the driver files and executed as
# they stand, in a namespace holding the variables they use.
# --------------------------------------------------------------------------------------
def driver_block(path: str, first: str, last: str, after: str = None):
    """Dedented source of the driver lines from the first line containing ``first`` (after the
    line containing ``after``) through the next line containing ``last``; returns (code, lines)."""
    import textwrap
    with open(path) as f:
        lines = f.read().splitlines()
    start = 0
    if after is not None:
        start = next(i for i, l in enumerate(lines) if after in l)
    i = next(k for k in range(start, len(lines)) if first in lines[k])
    j = next(k for k in range(i, len(lines)) if last in lines[k])
    return textwrap.dedent("\n".join(lines[i:j + 1])), (i + 1, j + 1)


def mat_roundtrip(model4):
    """What sio.loadmat returns for a datamat written by savemat (1-D biases come back [1, n])."""
    with Workdir():
        sio.savemat("m.mat", dict(zip(("weights1", "biases1", "weights2", "biases2"), model4)))
        c = sio.loadmat("m.mat")
    return {k: c[k] for k in ("weights1", "biases1", "weights2", "biases2")}


def case_driver_aggregations():
    out = {}
    rng = np.random.default_rng(4242)
    # ---- MQTT PS (PS_server.py:130-133) and device-side mix (learner_consensus.py:151-152)
    ps_path = os.path.join(TF2, "FL_over_MQTT", "PS_server.py")
    lc_path = os.path.join(TF2, "FL_over_MQTT", "learner_consensus.py")
    code_ps, span_ps = driver_block(ps_path, "for q in range(layers):", "/ active",
                                    after="active_device_indexes = indexes_tx[:, epoch_count]")
    code_lc, span_lc = driver_block(lc_path, "for q in range(layers):", "/ active", after="# apply consensus")
    out["ps_mqtt/src_lines"] = np.array(span_ps)
    out["learner/src_lines"] = np.array(span_lc)
    D, layers = 6, len(SHAPES_LENET1)
    glob_ = gen_model(rng, SHAPES_LENET1)  # model_global.get_weights(): fp32
    # payload layers: ndarray.tolist() on the learner, np.asarray(list) on the server -> fp64
    storage = [[np.asarray(a.tolist()) for a in gen_model(rng, SHAPES_LENET1)] for _ in range(D)]
    idx = rng.permutation(D)
    for t in range(layers):
        out[f"ps_mqtt/global_{t}"] = glob_[t]
        out[f"ps_mqtt/storage_{t}"] = np.stack([m[t] for m in storage])
    out["ps_mqtt/idx"] = idx
    for tag, active, u in (("a4_u1", 4, 1), ("a1_u05", 1, 0.5), ("a6_u1", 6, 1)):
        ns = {"layers": layers, "active": active, "update_factor": u, "local_models_storage": storage,
              "active_device_indexes": idx, "model_parameters": [a.copy() for a in glob_]}
        exec(code_ps, ns)
        for t in range(layers):
            out[f"ps_mqtt/{tag}/out_{t}"] = np.asarray(ns["model_parameters"][t])
        out[f"ps_mqtt/{tag}/meta"] = np.array([active, u], dtype=np.float64)
    ns = {"layers": layers, "active": 2, "update_factor": 1, "rx_global_model": storage[0],
          "model_parameters": [a.copy() for a in glob_]}
    exec(code_lc, ns)
    for t in range(layers):
        out[f"learner/out_{t}"] = np.asarray(ns["model_parameters"][t])

    # ---- TF1 CFA_FA server (federated_sample_CNN_CFA_FA.py:73-76 zeros, :86-89, :130-133) and
    #      client (:280-283), CNN shapes filter 16, number 8, multip 21
    fa_path = os.path.join(TF1, "federated_sample_CNN_CFA_FA.py")
    code_zero, span_zero = driver_block(fa_path, "server_w1 = np.zeros", "server_b2 = np.zeros")
    code_init, span_init = driver_block(fa_path, "server_w1 = server_w1 + balancing_vect[devices] * mathcontent",
                                        "server_b2 = server_b2 + balancing_vect[devices] * mathcontent")
    code_round, span_round = driver_block(fa_path, "server_w1 = server_w1 + eps_t_control * balancing_vect[devices] * (mathcontent",
                                          "server_b2 = server_b2 + eps_t_control * balancing_vect[devices] * (mathcontent")
    code_cli, span_cli = driver_block(fa_path, "W_val_l1 = W_val_l1 + eps_t_control2", "b_val_l2 = b_val_l2 + eps_t_control2")
    for k, sp in (("zeros", span_zero), ("init", span_init), ("round", span_round), ("client", span_cli)):
        out[f"cfa_fa/{k}_src_lines"] = np.array(sp)
    K = 5
    shapes = [(16, 1, 8), (8,), (168, 8), (8,)]
    contents0 = [mat_roundtrip(gen_model(rng, shapes)) for _ in range(K)]
    contents1 = [mat_roundtrip(gen_model(rng, shapes)) for _ in range(K)]
    for d in range(K):
        for key in ("weights1", "biases1", "weights2", "biases2"):
            out[f"cfa_fa/c0_{key}"] = np.stack([c[key] for c in contents0])
            out[f"cfa_fa/c1_{key}"] = np.stack([c[key] for c in contents1])
    ns = {"np": np, "filter": 16, "number": 8, "multip": 21, "balancing_vect": np.ones(K) * (1 / K)}
    exec(code_zero, ns)
    for d in range(K):
        ns["devices"], ns["mathcontent"] = d, contents0[d]
        exec(code_init, ns)
    for k, key in enumerate(("server_w1", "server_b1", "server_w2", "server_b2")):
        out[f"cfa_fa/init_{k}"] = np.asarray(ns[key])
    ns["eps_t_control"] = 0.7
    for d in range(K):
        ns["devices"], ns["mathcontent"] = d, contents1[d]
        exec(code_round, ns)
    for k, key in enumerate(("server_w1", "server_b1", "server_w2", "server_b2")):
        out[f"cfa_fa/round_{k}"] = np.asarray(ns[key])
    server_file = mat_roundtrip([ns["server_w1"], ns["server_b1"], ns["server_w2"], ns["server_b2"]])
    W_val = [a for a in gen_model(rng, shapes)]  # the device's fp32 model (TF values)
    for k, key in enumerate(("weights1", "biases1", "weights2", "biases2")):
        out[f"cfa_fa/server_file_{key}"] = server_file[key]
        out[f"cfa_fa/wval_{k}"] = W_val[k]
    ns2 = {"np": np, "W_val_l1": W_val[0], "b_val_l1": W_val[1], "W_val_l2": W_val[2], "b_val_l2": W_val[3],
           "eps_t_control2": 0.35, "mathcontent": server_file}
    exec(code_cli, ns2)
    for k, key in enumerate(("W_val_l1", "b_val_l1", "W_val_l2", "b_val_l2")):
        out[f"cfa_fa/client_{k}"] = np.asarray(ns2[key])
    save("f1_driver_aggregations.npz", **out)


def main():
    if not os.path.isdir(REF):
        sys.exit(f"reference tree not found at {REF}")
    install_stubs()
    case_topology()
    case_mobile_network()
    case_tf1_cfa()
    case_tf1_ongraphs()
    case_tf1_cfa_ge()
    case_tf1_cfa_ge_mobilenet()
    case_tf2()
    case_parameter_server()
    case_driver_aggregations()
    case_variants()


if __name__ == "__main__":
    main()
