"""Run-control callbacks of the reference (`src/simulation_callbacks.rs`) over an engine batch.

`KubernetriksSimulation::run_with_callbacks` (simulator.rs:355-372) loops `while on_step() { step() }`
and then calls `on_simulation_finish`.  The engine evaluates `on_step` on the device between events
(K10S_RUN_UNTIL_ALL_FINISHED), so a callbacks object here chooses the engine run mode and does the
finish hook on the host, for every replica of the batch:

* `RunUntilAllPodsAreFinishedCallbacks` (simulation_callbacks.rs:85-96): stop before the next step
  once `time % 1000 == 0` and every trace pod terminated; finish = `assert_and_print`.
* `RunUntilAllPodsAreFinishedAndLongRunningPodsExceedDeadlineCallbacks` (:98-129): as written, its
  `on_step` sets `all_short_pods_terminated` at the first qualifying `% 1000` check and returns
  `!all_short_pods_terminated`, i.e. false — the run stops at exactly the step the callbacks above
  stop at and the deadline branch is never reached (the reference marks this with "TODO: fix bug
  here which instantly terminates simulation", :114).  Reproduced as such; `deadline_time` is kept.
"""
from __future__ import annotations

from typing import List

from . import metrics
from .native import RUN_UNTIL_ALL_FINISHED


class SimulationCallbacks:
    """simulation_callbacks.rs:8-19."""

    def on_simulation_start(self, engine) -> None:
        pass

    def run(self, engine, max_time: float, max_events_per_launch: int) -> float:
        raise NotImplementedError

    def on_simulation_finish(self, engine) -> None:
        pass


class RunUntilAllPodsAreFinishedCallbacks(SimulationCallbacks):
    """simulation_callbacks.rs:21-96."""

    def __init__(self, printer_format: str = "json"):
        self.printer_format = printer_format
        self.printed: List[str] = []

    def run(self, engine, max_time: float, max_events_per_launch: int) -> float:
        return engine.run(RUN_UNTIL_ALL_FINISHED, 0.0, max_time, max_events_per_launch)

    def on_simulation_finish(self, engine) -> None:
        # assert_and_print (44-83) per replica; a replica stopped by a reference panic or by the
        # max_time guard did not reach the finish hook
        self.printed = [metrics.assert_and_print(r, self.printer_format) if r["status"] == "finished" else ""
                        for r in engine.results()]


class RunUntilAllPodsAreFinishedAndLongRunningPodsExceedDeadlineCallbacks(RunUntilAllPodsAreFinishedCallbacks):
    """simulation_callbacks.rs:98-129 (see the module docstring for why it stops where
    RunUntilAllPodsAreFinishedCallbacks stops)."""

    def __init__(self, deadline_time: float, printer_format: str = "json"):
        super().__init__(printer_format)
        self.deadline_time = deadline_time
        self.all_short_pods_terminated = False

    def on_simulation_finish(self, engine) -> None:
        self.all_short_pods_terminated = True
        super().on_simulation_finish(engine)


def run_with_callbacks(engine, callbacks: SimulationCallbacks, max_time: float = 1e12,
                       max_events_per_launch: int = 0) -> float:
    """KubernetriksSimulation::run_with_callbacks (simulator.rs:355-372) over every replica."""
    callbacks.on_simulation_start(engine)
    ms = callbacks.run(engine, max_time, max_events_per_launch)
    callbacks.on_simulation_finish(engine)
    return ms
