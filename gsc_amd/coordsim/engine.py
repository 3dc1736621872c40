"""Discrete-event engine with SimPy-4 ordering semantics (scalar CPU oracle).

The reference simulator (coord-sim) runs on SimPy 4 (``coordsim/simulation/
flowsimulator.py``, ``siminterface/simulator.py:94``).  SimPy is not available
here, and the exact tie-breaking of simultaneous events decides which flows win
node/link capacity, so this module re-implements the small part of the SimPy
contract that coord-sim relies on:

* a heap ordered by ``(time, priority, event id)`` with ``URGENT=0`` for
  process initialisation / stop events and ``NORMAL=1`` for everything else;
* generator-based processes: ``env.process(gen)`` schedules an URGENT
  initialise event; a process that yields an event resumes when it fires; a
  process that returns schedules its own completion event (NORMAL, delay 0);
* ``run(until=t)`` schedules an URGENT stop event at ``t`` so NORMAL events at
  exactly ``t`` execute in the *next* ``run`` call (the run-window semantics
  described in SURVEY.md section 3.2);
* ``step()`` pops and fires exactly one event (used by the duration
  controller's ``get_init_state``).

The batched HIP simulator (``csrc/sim``) reproduces the same event ids, so
deterministic configurations agree bit-for-bit with this oracle.
"""
from __future__ import annotations

import heapq
from typing import Any, Callable, Generator, List, Optional

URGENT = 0
NORMAL = 1

_PENDING = object()


class StopSimulation(Exception):
    """Raised by the stop event scheduled by :meth:`Environment.run`."""


class EmptySchedule(Exception):
    """No further events are scheduled."""


class Event:
    """A one-shot event. ``callbacks`` is ``None`` once the event was processed."""

    __slots__ = ("env", "callbacks", "_value", "_ok")

    def __init__(self, env: "Environment"):
        self.env = env
        self.callbacks: Optional[List[Callable[["Event"], None]]] = []
        self._value: Any = _PENDING
        self._ok = True

    @property
    def triggered(self) -> bool:
        return self._value is not _PENDING

    @property
    def processed(self) -> bool:
        return self.callbacks is None

    @property
    def value(self) -> Any:
        if self._value is _PENDING:
            raise AttributeError("value of untriggered event")
        return self._value

    def succeed(self, value: Any = None) -> "Event":
        if self._value is not _PENDING:
            raise RuntimeError("event already triggered")
        self._ok = True
        self._value = value
        self.env.schedule(self, NORMAL)
        return self


class Timeout(Event):
    __slots__ = ("delay",)

    def __init__(self, env: "Environment", delay: float, value: Any = None):
        if delay < 0:
            raise ValueError(f"negative delay {delay}")
        super().__init__(env)
        self.delay = delay
        self._value = value
        env.schedule(self, NORMAL, delay)


class _Initialize(Event):
    __slots__ = ()

    def __init__(self, env: "Environment", process: "Process"):
        super().__init__(env)
        self.callbacks = [process._resume]
        self._value = None
        env.schedule(self, URGENT)


class Process(Event):
    """Wraps a generator; the process itself is an event that fires on return."""

    __slots__ = ("_generator", "_target")

    def __init__(self, env: "Environment", generator: Generator):
        if not hasattr(generator, "send"):
            raise ValueError(f"{generator!r} is not a generator")
        super().__init__(env)
        self._generator = generator
        self._target: Event = _Initialize(env, self)

    @property
    def is_alive(self) -> bool:
        return self._value is _PENDING

    def _resume(self, event: Event) -> None:
        env = self.env
        env.active_process = self
        while True:
            try:
                if event._ok:
                    event = self._generator.send(event._value)
                else:
                    event = self._generator.throw(event._value)
            except StopIteration as stop:
                event = None
                self._ok = True
                self._value = stop.args[0] if stop.args else None
                env.schedule(self, NORMAL)
                break
            if not isinstance(event, Event):
                raise RuntimeError(f"process yielded a non-event: {event!r}")
            if event.callbacks is not None:
                event.callbacks.append(self._resume)
                break
            # already processed: continue immediately with its value
        self._target = event
        env.active_process = None


class Environment:
    """Event loop with SimPy-compatible ordering."""

    def __init__(self, initial_time: float = 0):
        self._now = initial_time
        self._queue: list = []
        self._eid = 0
        self.active_process: Optional[Process] = None

    @property
    def now(self) -> float:
        return self._now

    @property
    def queue(self) -> list:
        return self._queue

    def schedule(self, event: Event, priority: int = NORMAL, delay: float = 0) -> None:
        heapq.heappush(self._queue, (self._now + delay, priority, self._eid, event))
        self._eid += 1

    def peek(self) -> float:
        return self._queue[0][0] if self._queue else float("inf")

    # factories -----------------------------------------------------------------
    def event(self) -> Event:
        return Event(self)

    def timeout(self, delay: float, value: Any = None) -> Timeout:
        return Timeout(self, delay, value)

    def process(self, generator: Generator) -> Process:
        return Process(self, generator)

    # loop ---------------------------------------------------------------------
    def step(self) -> None:
        try:
            self._now, _, _, event = heapq.heappop(self._queue)
        except IndexError:
            raise EmptySchedule() from None
        callbacks, event.callbacks = event.callbacks, None
        for cb in callbacks:
            cb(event)
        if not event._ok:
            raise event._value

    def run(self, until: Any = None) -> Any:
        if until is not None:
            if not isinstance(until, Event):
                at = float(until)
                if at <= self._now:
                    raise ValueError(f"until ({at}) must be > now ({self._now})")
                stop = Event(self)
                stop._ok = True
                stop._value = None
                self.schedule(stop, URGENT, at - self._now)
                until = stop
            elif until.callbacks is None:
                return until.value
            until.callbacks.append(_stop_callback)
        try:
            while True:
                self.step()
        except StopSimulation as exc:
            return exc.args[0]
        except EmptySchedule:
            if until is not None and not until.triggered:
                raise RuntimeError("no scheduled events left but until event was not triggered")
            return None


def _stop_callback(event: Event) -> None:
    if event._ok:
        raise StopSimulation(event._value)
    raise event._value
