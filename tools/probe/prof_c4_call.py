import cProfile, pstats, os, sys, tempfile
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tools", "probe"))
os.environ["FEDERATED_AMD_PAUSE_SCALE"] = "0"
import numpy as np
import tf2_calls as T
from federated_amd.consensus import consensus_v3
d = tempfile.mkdtemp(); os.chdir(d); os.makedirs("results")
rng = np.random.default_rng(0); K = 4
for k in range(K + 1):
    np.savez(f"results/dump_train_variables{k}.npz", epoch_count=5, training_end=False)
    np.save(f"results/dump_train_model{k}.npy", T.weights(T.VGG1, rng), allow_pickle=True)
p = consensus_v3.CFA_process(K + 1, 0, K); local = T.weights(T.VGG1, rng)
def call():
    p.update_local_model(local.copy()); p.federated_weights_computing(list(range(1, K + 1)), K, 5, 0.5)
for _ in range(5): call()
pr = cProfile.Profile(); pr.enable()
for _ in range(40): call()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(14)
