"""install_as_consensus() makes the reference's import lines resolve to the drop-in modules."""
import sys


def test_install_as_consensus_aliases_reference_imports():
    saved = {k: v for k, v in sys.modules.items() if k == "consensus" or k.startswith("consensus.")}
    try:
        from federated_amd.consensus import install_as_consensus
        install_as_consensus()
        from consensus.cfa_ongraphs import CFA_process as A  # noqa: E402  (FL_CFA_CNN_tf2.py:3)
        from consensus.consensus_v3 import CFA_process as B  # noqa: E402
        from federated_amd.consensus import cfa_ongraphs, consensus_v3
        assert A is cfa_ongraphs.CFA_process and B is consensus_v3.CFA_process
        install_as_consensus("fl_radar")
        from consensus.consensus_v3 import CFA_process as C  # noqa: E402
        from federated_amd.consensus.fl_radar import consensus_v3 as radar
        assert C is radar.CFA_process
    finally:
        for k in [k for k in sys.modules if k == "consensus" or k.startswith("consensus.")]:
            del sys.modules[k]
        sys.modules.update(saved)
