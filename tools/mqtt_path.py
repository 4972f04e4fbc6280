#!/usr/bin/env python3
"""(f2) End-to-end MQTT payload path: reference idiom vs the native codec + GPU fold.

One PS aggregation round of FL_over_MQTT (PS_server.py:90-149) for C active devices, and one
learner receive + publish (learner_consensus.py:136-153, 257-268), on the TF2 radar CNN shapes
(P = 3 745 446, a 33.7 MB payload) and the MQTT learner CNN shapes:

  reference: pickle.loads + np.asarray per layer; numpy fold; set_weights (fp32 cast);
             get_weights().tolist() + pickle.dumps
  native:    cfa_payload decode straight into pinned fp64 staging; one H2D, cfa_fold_f64, one
             D2H; fp32 cast; cfa_payload_encode (the same bytes)

The reference side is timed with the oracle's restatement of those driver lines (stdlib pickle
is the reference's codec). Writes one JSON line per case to stdout (and --out).
Usage: python tools/mqtt_path.py [--reps 5] [--out profiles/r01_mqtt_path.jsonl]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

RADAR = [(8, 8, 1, 32), (32,), (4, 4, 32, 64), (64,), (3, 3, 64, 64), (64,), (7168, 512), (512,), (512, 6), (6,)]
MQTT_CNN = [(5, 5, 1, 4), (4,), (5, 5, 4, 8), (8,), (7200, 6), (6,)]


def model(shapes, seed):
    rng = np.random.default_rng(seed)
    return [rng.standard_normal(s).astype(np.float32) for s in shapes]


def best(fn, reps):
    ts = []
    out = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--active", type=int, default=4)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from federated_amd import payload as pl, server
    from oracle import cfa_oracle as orc

    lines = []
    for name, shapes in (("radar_cnn", RADAR), ("mqtt_cnn", MQTT_CNN)):
        P = sum(int(np.prod(s)) for s in shapes)
        L = len(shapes)
        C = a.active
        gm = model(shapes, 0)
        payloads = [orc.mqtt_learner_payload(model(shapes, 1 + d), d, 10, 3, False) for d in range(C)]

        def ref_ps():
            storage = [orc.mqtt_decode_layers(p, L) for p in payloads]
            mp = orc.ps_mqtt_aggregate(gm, storage, list(range(C)), 1, C)
            return orc.mqtt_ps_payload([m.astype(np.float32) for m in mp], 4, False)

        def nat_ps():
            mp = server.ps_mqtt_aggregate_payloads(gm, payloads, 1, C)
            return server.ps_mqtt_publish([m.astype(np.float32) for m in mp], 4, False)

        nat_ps()  # warm (pinned staging, streams)
        t_ref, out_ref = best(ref_ps, max(1, a.reps // 2))
        t_nat, out_nat = best(nat_ps, a.reps)
        # native breakdown
        t_dec, _ = best(lambda: [pl.Payload(p).read_into(pl.layer_keys("model_layer", L), np.empty(P)) for p in payloads],
                        a.reps)
        mp = server.ps_mqtt_aggregate_payloads(gm, payloads, 1, C)
        w32 = [m.astype(np.float32) for m in mp]
        t_enc, _ = best(lambda: server.ps_mqtt_publish(w32, 4, False), a.reps)
        t_ref_dec, _ = best(lambda: [orc.mqtt_decode_layers(p, L) for p in payloads], 1)
        t_ref_enc, _ = best(lambda: orc.mqtt_ps_payload(w32, 4, False), 1)
        rec = {"case": f"ps_round_{name}", "params": P, "active": C, "payload_bytes": len(payloads[0]),
               "reference_ms": round(t_ref, 2), "native_ms": round(t_nat, 2), "speedup": round(t_ref / t_nat, 1),
               "identical_bytes": out_ref == out_nat,
               "native_decode_ms": round(t_dec, 2), "native_encode_ms": round(t_enc, 2),
               "reference_decode_ms": round(t_ref_dec, 2), "reference_encode_ms": round(t_ref_enc, 2),
               "decode_GBps_payload": round(C * len(payloads[0]) / t_dec / 1e6, 2),
               "encode_GBps_payload": round(len(out_nat) / t_enc / 1e6, 2)}
        lines.append(rec)

        lm = model(shapes, 50)

        def ref_learner():
            w, e, end = orc.mqtt_learner_receive(lm, payloads[0], L)
            return orc.mqtt_learner_payload([x.astype(np.float32) for x in w], 1, 11, e, end)

        def nat_learner():
            w, e, end = server.learner_consensus_receive(lm, payloads[0])
            return server.learner_publish([x.astype(np.float32) for x in w], 1, 11, e, end)

        nat_learner()
        t_ref, out_ref = best(ref_learner, max(1, a.reps // 2))
        t_nat, out_nat = best(nat_learner, a.reps)
        lines.append({"case": f"learner_round_{name}", "params": P, "payload_bytes": len(payloads[0]),
                      "reference_ms": round(t_ref, 2), "native_ms": round(t_nat, 2),
                      "speedup": round(t_ref / t_nat, 1), "identical_bytes": out_ref == out_nat})
    host = {"cpu": os.cpu_count()}
    for rec in lines:
        rec.update(host)
        print(json.dumps(rec), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            for rec in lines:
                fh.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
