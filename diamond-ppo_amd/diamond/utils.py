"""Training utilities the agents construct (reference diamond/utils.py).

Only what the agents' constructors and train() touch is provided here: ``Checkpointer`` keeps the
reference's on-disk format (``{run_name}-step{step:06d}.pt`` holding ``{"step", "model_state",
"opt_state"}``, utils.py:584-619) so checkpoints are interchangeable; ``Ticker`` prints the same
progress columns (utils.py:20-215) without plotting; ``Logger`` / ``Timer`` keep their recording
methods (utils.py:270-543) and leave plotting (plotly) out of scope.
"""
from __future__ import annotations

import time
from collections import defaultdict, deque
from contextlib import contextmanager
from pathlib import Path

import numpy as np
import torch


class Checkpointer:
    def __init__(self, folder: str | Path = "models", run_name: str = "run", *,
                 keep_last: int | None = None) -> None:
        self.folder = Path(folder)
        self.run_name = run_name
        self.keep_last = keep_last

    def save(self, step: int, model: torch.nn.Module, optimizer=None) -> None:
        self.folder.mkdir(parents=True, exist_ok=True)
        path = self.folder / f"{self.run_name}-step{step:06d}.pt"
        payload = {"step": step, "model_state": model.state_dict()}
        if optimizer is not None:
            payload["opt_state"] = optimizer.state_dict()
        torch.save(payload, path)
        self._trim_old()

    def load(self, path: str | Path, model: torch.nn.Module, optimizer=None) -> None:
        chk = torch.load(path, map_location="cpu", weights_only=True)
        model.load_state_dict(chk["model_state"])
        if optimizer is not None and "opt_state" in chk:
            optimizer.load_state_dict(chk["opt_state"])

    def _trim_old(self) -> None:
        if self.keep_last is None:
            return
        ckpts = sorted(self.folder.glob(f"{self.run_name}-step*.pt"))
        for old in ckpts[:-self.keep_last]:
            old.unlink(missing_ok=True)


class Ticker:
    """Episode return/length tracking and a progress line per ~5% of training."""

    def __init__(self, total_steps: int, num_envs: int, rollout_steps: int, verbose: bool = True,
                 window: int = 100) -> None:
        self.total_steps, self.num_envs = total_steps, num_envs
        self.verbose = verbose
        self.ep_returns = np.zeros(num_envs)
        self.ep_lengths = np.zeros(num_envs, dtype=np.int64)
        self.recent_returns = deque(maxlen=window)
        self.recent_lengths = deque(maxlen=window)
        self.episodes = 0
        self.steps = 0
        self.start = time.time()
        self._next_print = 0.05

    def tick(self, rewards, dones) -> None:
        self.steps += self.num_envs
        self.ep_returns += np.asarray(rewards, dtype=np.float64)
        self.ep_lengths += 1
        d = np.asarray(dones, dtype=bool)
        for i in np.flatnonzero(d):
            self.recent_returns.append(self.ep_returns[i])
            self.recent_lengths.append(self.ep_lengths[i])
            self.episodes += 1
        self.ep_returns[d] = 0.0
        self.ep_lengths[d] = 0
        prog = self.steps / max(self.total_steps, 1)
        if self.verbose and prog >= self._next_print:
            self._next_print += 0.05
            el = time.time() - self.start
            mr = np.mean(self.recent_returns) if self.recent_returns else float("nan")
            ml = np.mean(self.recent_lengths) if self.recent_lengths else float("nan")
            print(f"{100 * prog:9.1f}%  | {self.steps:10,d}  | {self.episodes:9,d}  | {mr:9.2f}  |"
                  f" {ml:9.1f}  | {self.steps / max(el, 1e-9):7.0f}  | "
                  f"{time.strftime('%H:%M:%S', time.gmtime(el))}")


class Logger:
    def __init__(self) -> None:
        self.data = defaultdict(list)

    def log(self, key: str, step: int, value: float) -> None:
        self.data[key].append((step, float(value)))


class Timer:
    def __init__(self) -> None:
        self.timings = defaultdict(list)

    @contextmanager
    def time(self, name: str):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.timings[name].append(time.perf_counter() - t0)

    def mean(self, name: str) -> float:
        v = self.timings.get(name)
        return float(np.mean(v)) if v else float("nan")
