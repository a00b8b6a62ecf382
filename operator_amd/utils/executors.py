"""ThreadPoolExecutor that can wait until every submitted task (including
tasks submitted by tasks) has finished — used to drain the operator's
analysis and kube-write pools in tests and benchmarks."""
from __future__ import annotations

import threading
from concurrent.futures import ThreadPoolExecutor


class TrackedExecutor(ThreadPoolExecutor):
    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self._pending = 0
        self._cv = threading.Condition()

    def submit(self, fn, /, *args, **kwargs):
        with self._cv:
            self._pending += 1
        try:
            f = super().submit(fn, *args, **kwargs)
        except BaseException:
            self._done(None)
            raise
        f.add_done_callback(self._done)
        return f

    def _done(self, _f) -> None:
        with self._cv:
            self._pending -= 1
            if self._pending == 0:
                self._cv.notify_all()

    @property
    def pending(self) -> int:
        return self._pending

    def wait_idle(self, timeout: float | None = None) -> bool:
        with self._cv:
            return self._cv.wait_for(lambda: self._pending == 0, timeout)
