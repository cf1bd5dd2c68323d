"""Stage markers and a no-progress watchdog for multi-rank runs.

bench.py --gpus N (one rank per GPU) has never run on more than one GPU
before the driver's 8-GPU scaling run, so that run must explain itself if it
stops: every rank prints a flushed marker line on stderr at each stage
(communicator init, each warm-up batch, each timed step, the kernel-timing
pass, ...), and a watchdog thread watches for progress. After `budget_s`
seconds without a new marker it

  1. aborts the rank's collectives (`abort()`, e.g. vp_comm_abort: the RCCL
     communicator is aborted so its kernels stop spinning on a peer that
     never comes), in a helper thread it waits at most a few seconds for;
  2. prints a partial JSON line (rank 0 on stdout: the line the driver
     parses; every rank on stderr) naming the stage reached and the stages
     completed, with `"value": null` and an `"error"`;
  3. ends the process with exit status 3 (os._exit: the main thread may be
     blocked inside a collective, which nothing else can interrupt).

It never re-launches anything. The reference has no multi-GPU path
(/root/reference/nf.c:38,142: one core); this is readiness for the N > 1
runs of SURVEY.md §8(e).
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time

EXIT_STALLED = 3


class Watchdog:
    def __init__(self, rank: int, world: int, budget_s: float, partial: dict | None = None,
                 abort=None, tag: str = "bench", out=None, err=None):
        self.rank, self.world = rank, world
        self.budget_s = float(budget_s)
        self.partial = dict(partial or {})
        self.abort = abort
        self.tag = tag
        self.out = out or sys.stdout
        self.err = err or sys.stderr
        self.t0 = time.monotonic()
        self.last = self.t0
        self.stage_name = "start"
        self.done: list[str] = []
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread = None
        self.fired = False

    # ------------------------------------------------------------ markers --
    def stage(self, name: str):
        """Enter stage `name` (the previous one is complete): a flushed
        marker line on stderr, and the watchdog's clock restarts."""
        with self._lock:
            if self.stage_name != "start":
                self.done.append(self.stage_name)
            self.stage_name = name
            self.last = time.monotonic()
        self.err.write("[%s r%d/%d +%.2fs] %s\n" % (self.tag, self.rank, self.world,
                                                   self.last - self.t0, name))
        self.err.flush()

    def beat(self):
        """Progress without a new stage."""
        with self._lock:
            self.last = time.monotonic()

    # ----------------------------------------------------------- watchdog --
    def start(self, poll_s: float = 0.5):
        if self.budget_s <= 0 or self._thread is not None:
            return self
        self._thread = threading.Thread(target=self._run, args=(poll_s,), daemon=True,
                                        name="vigpath-watchdog")
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()

    def _run(self, poll_s):
        while not self._stop.wait(poll_s):
            with self._lock:
                idle = time.monotonic() - self.last
                stage = self.stage_name
            if idle > self.budget_s:
                self.fire(stage, idle)
                return

    def partial_line(self, stage: str, idle: float) -> dict:
        line = dict(self.partial)
        line.update({
            "value": None, "partial": True, "n_gpus": self.world,
            "error": "watchdog: rank %d made no progress for %.1f s in stage '%s'; "
                     "collectives aborted, run ended" % (self.rank, idle, stage),
            "stage_reached": stage, "stages_done": list(self.done),
            "rank": self.rank, "elapsed_s": round(time.monotonic() - self.t0, 2)})
        return line

    def fire(self, stage: str, idle: float):
        """Abort the collectives, print the partial line, exit 3."""
        self.fired = True
        if self.abort is not None:
            t = threading.Thread(target=self._abort_quietly, daemon=True)
            t.start()
            t.join(5.0)
        line = json.dumps(self.partial_line(stage, idle))
        try:
            self.err.write("[%s r%d/%d] WATCHDOG %s\n" % (self.tag, self.rank, self.world, line))
            self.err.flush()
            if self.rank == 0:
                self.out.write(line + "\n")
                self.out.flush()
        finally:
            os._exit(EXIT_STALLED)

    def _abort_quietly(self):
        try:
            self.abort()
        except Exception as e:  # noqa: BLE001 (best effort: the exit follows)
            self.err.write("[%s r%d] abort failed: %r\n" % (self.tag, self.rank, e))
            self.err.flush()
