"""The task side of snf4j's selector loop (InternalSelectorLoop.java: executenf queues a
task from any thread and wakes select(), :990-1011 and :1038-1046; handleTasks runs tasks
until the queue is empty, :641 and :751-758), the loop snf4j_amd.loop's batchers are
driven with by the bench and the tests.  Not part of the drop-in: in Java the loop is
snf4j's own."""
from __future__ import annotations

import collections
import threading


class SelectorLoop:
    """The task side of InternalSelectorLoop: executenf queues (any thread) and wakes
    the selector; handle_tasks runs tasks until the queue is empty."""

    def __init__(self):
        self._tasks = collections.deque()
        self._lock = threading.Lock()
        self._wake = threading.Event()
        self.iteration = 0

    def executenf(self, task):
        with self._lock:
            self._tasks.append(task)
        self._wake.set()

    def handle_tasks(self):
        while True:
            with self._lock:
                if not self._tasks:
                    return
                task = self._tasks.popleft()
            task()

    def select(self, timeout: float | None) -> bool:
        """Block until woken (executenf) or the timeout; True if woken."""
        woke = self._wake.wait(timeout)
        self._wake.clear()
        return woke

    def run_iteration(self, reads):
        """One loop iteration: the reads (callables, each a session's read -> decode),
        then the task phase."""
        self.iteration += 1
        for r in reads:
            r()
        self.handle_tasks()

    def has_tasks(self) -> bool:
        with self._lock:
            return bool(self._tasks)


def run_until_idle(loop: SelectorLoop, *batchers, timeout: float = 60.0):
    """Loop iterations without reads until every batcher's flushes are delivered
    (woken by the completion threads)."""
    import time
    end = time.monotonic() + timeout
    while any(b.inflight or b.flush_scheduled for b in batchers) or loop.has_tasks():
        if time.monotonic() > end:
            raise TimeoutError("flushes still in flight")
        loop.select(0.05)
        loop.run_iteration([])
