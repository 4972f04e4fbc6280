"""The rank's stream budget: one stream per role and device, created once per process and reused.

A round at N > 1 runs on the compute stream (torch's current stream), one exchange stream
(``comm``: RCCL's groups, the link probe) and the host lane's two copy streams (``lane_out``:
D2H + its signals, ``lane_in``: H2D + its acks; hostlane.py). HIP maps a process's streams onto
``GPU_MAX_HW_QUEUES`` hardware queues (4 on this pool) and every stream drawn from torch's pool
may land on a queue another active stream holds, so no shard, lane or probe draws streams of its
own: they all take theirs from here. Nothing here waits on the GPU (the lane's waits are host
side, hostlane.py), so a shared queue costs concurrency, never a stall behind a parked wait.
"""
from __future__ import annotations

import threading
from typing import Dict, Tuple

ROLES = ("comm", "lane_out", "lane_in")

_lock = threading.Lock()
_streams: Dict[Tuple[int, str], object] = {}


def role_stream(role: str, device=None):
    """The process's stream for ``role`` on ``device`` (default: the current device)."""
    import torch
    if role not in ROLES:
        raise ValueError(f"unknown stream role {role!r} (roles: {', '.join(ROLES)})")
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if dev.type != "cuda":
        raise ValueError(f"stream roles are GPU streams, got device {dev}")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    with _lock:
        s = _streams.get((idx, role))
        if s is None:
            s = _streams[(idx, role)] = torch.cuda.Stream(torch.device("cuda", idx))
        return s


def budget() -> dict:
    """What the process has created: {device: [roles]} (the bench line reports it beside
    ``GPU_MAX_HW_QUEUES``)."""
    out: Dict[int, list] = {}
    with _lock:
        for (d, role) in sorted(_streams):
            out.setdefault(d, []).append(role)
    return out
