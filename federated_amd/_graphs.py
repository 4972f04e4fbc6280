"""hipGraph replay of whole consensus rounds.

A device-resident population round is a handful of small launches (population mix, gradient
evaluation, gradient step). At the reference's model sizes each launch runs for a few
microseconds, so a Python loop that launches round after round is bound by the host: ctypes
calls, argument checks and launch latency. The rounds of such a population cycle through a
closed period of buffer assignments (``PopulationRound``: models/out ping-pong, period 2;
``CfaGePopulation``: a 3-way rotation of (W, pub, mixed) times the (G, G_next) swap, period 6),
so one period's launches are captured once as a graph (torch.cuda.CUDAGraph = hipGraph on ROCm)
and replayed: the graph holds the same kernels with the same arguments, so the results are
the eager rounds' results bit for bit (tested in tests/test_gpu_graph_rounds.py).
"""
from __future__ import annotations

import gc
from typing import Callable, Dict, Tuple

import torch

BLOCK_PERIODS = 8  # periods per replay of the large graph
CAPTURE_MODE = "global"  # torch.cuda.graph capture_error_mode (hipStreamCaptureModeGlobal)


class RoundGraphs:
    """Replays ``step`` (one round launched on the current stream; it advances the caller's
    Python-side buffer assignment) through graphs of whole periods.

    ``phase()`` returns the caller's position in its period (hashable); a graph is captured per
    (phase, periods) the first time it is needed. Capturing launches nothing: the replays run
    the rounds."""

    def __init__(self, device: torch.device, step: Callable[[], None], period: int,
                 phase: Callable[[], object]):
        self.device, self.step, self.period, self.phase = device, step, int(period), phase
        self._graphs: Dict[Tuple[object, int], torch.cuda.CUDAGraph] = {}

    def _graph(self, periods: int) -> torch.cuda.CUDAGraph:
        key = (self.phase(), periods)
        g = self._graphs.get(key)
        if g is None:
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            # no garbage collection while capturing: collecting an unrelated dead graph, event or
            # stream would destroy a HIP object mid-capture and abort the process
            gc.collect()
            was_enabled = gc.isenabled()
            gc.disable()
            try:
                # strict ("global") capture: Engine construction ran cfa_device_prepare, so the
                # libcfa launch path queries, allocates and reconfigures nothing while capturing
                with torch.cuda.graph(g, stream=s, capture_error_mode=CAPTURE_MODE):
                    for _ in range(periods * self.period):
                        self.step()
            finally:
                if was_enabled:
                    gc.enable()
            if self.phase() != key[0]:
                raise RuntimeError("a period of rounds must return to its starting phase")
            self._graphs[key] = g
        return g

    def run(self, rounds: int) -> None:
        """``rounds`` rounds on the current stream: whole periods from graphs, the rest eager."""
        if rounds < 0:
            raise ValueError("rounds must be >= 0")
        full, rest = divmod(int(rounds), self.period)
        while full >= BLOCK_PERIODS:
            self._graph(BLOCK_PERIODS).replay()
            full -= BLOCK_PERIODS
        for _ in range(full):
            self._graph(1).replay()
        for _ in range(rest):
            self.step()
