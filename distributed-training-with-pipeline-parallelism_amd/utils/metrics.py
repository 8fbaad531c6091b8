"""Per-step metrics and fail-fast watchdog.

* :class:`MetricsLogger` -- JSONL records (step, loss, lr, tokens/s, step time, grad
  norm, HBM peak, measured bubble), aggregated as max step time over ranks (the
  reference reports the last rank's wall clock only, helper:226-227; here every
  rank's clock counts).
* :class:`Watchdog` -- a heartbeat thread: if a step does not finish within
  ``timeout_s`` it prints every thread's stack plus the pipeline program grid of
  this rank and hard-exits, so the launcher tears the job down instead of hanging
  forever (the reference's ``join()`` has no timeout, nb:324-325).
"""
from __future__ import annotations

import faulthandler
import json
import os
import sys
import threading
import time
from typing import Callable, Optional

import torch
import torch.distributed as dist


class MetricsLogger:
    def __init__(self, path: Optional[str], rank: int = 0, device: Optional[torch.device] = None):
        self.path = path
        self.rank = rank
        self.device = device
        self._f = open(path, "a") if (path and rank == 0) else None

    def log(self, step: int, tokens: int, step_s: float, loss: Optional[float] = None, lr: Optional[float] = None,
            grad_norm: Optional[float] = None, bubble: Optional[float] = None, **extra) -> dict:
        t = torch.tensor([step_s], dtype=torch.float64, device=self.device or "cpu")
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        step_s = float(t.item())
        rec = {"step": step, "loss": loss, "lr": lr, "tokens_per_s": tokens / step_s if step_s > 0 else None,
               "step_ms": step_s * 1e3, "grad_norm": grad_norm, "bubble": bubble, "time": time.time()}
        if self.device is not None and self.device.type == "cuda":
            # reserved: what the device holds (HIP-graph pools keep freed blocks reserved;
            # the allocated counter drops when a capture frees them)
            rec["hbm_peak_gb"] = torch.cuda.max_memory_reserved(self.device) / 2 ** 30
            rec["hbm_allocated_peak_gb"] = torch.cuda.max_memory_allocated(self.device) / 2 ** 30
        rec.update(extra)
        if self._f is not None:
            self._f.write(json.dumps(rec) + "\n")
            self._f.flush()
        return rec

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None


class Watchdog:
    """``with wd.step(): trainer.train_step(...)`` -- aborts the process on a hang."""

    def __init__(self, timeout_s: float, describe: Optional[Callable[[], str]] = None, exit_code: int = 17):
        self.timeout_s = timeout_s
        self.describe = describe
        self.exit_code = exit_code
        self._deadline: Optional[float] = None
        self._limit = timeout_s
        self._lock = threading.Lock()
        self._stop = False
        self._thread = None
        if timeout_s and timeout_s > 0:
            self._thread = threading.Thread(target=self._run, name="mipipe-watchdog", daemon=True)
            self._thread.start()

    def _run(self):
        while not self._stop:
            time.sleep(min(1.0, max(0.05, self.timeout_s / 4)))
            with self._lock:
                dl = self._deadline
            if dl is not None and time.monotonic() > dl:
                rank = os.environ.get("RANK", "0")
                sys.stderr.write(f"[mipipe watchdog] rank {rank}: step exceeded {self._limit:.0f}s -- aborting\n")
                if self.describe is not None:
                    try:
                        sys.stderr.write(self.describe() + "\n")
                    except Exception as e:  # pragma: no cover - diagnostics only
                        sys.stderr.write(f"(describe failed: {e})\n")
                faulthandler.dump_traceback(all_threads=True)
                sys.stderr.flush()
                os._exit(self.exit_code)

    def step(self, timeout_s: Optional[float] = None):
        """Arm the watchdog for one phase (``timeout_s`` overrides the default limit)."""
        wd = self
        limit = wd.timeout_s if timeout_s is None else float(timeout_s)

        class _Ctx:
            def __enter__(self_):
                with wd._lock:
                    wd._deadline = time.monotonic() + limit if wd._thread else None
                    wd._limit = limit
                return self_

            def __exit__(self_, *exc):
                with wd._lock:
                    wd._deadline = None
                return False

        return _Ctx()

    def close(self):
        self._stop = True
