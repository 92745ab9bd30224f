"""Training utilities the agents construct (reference diamond/utils.py).

``Checkpointer`` keeps the reference's on-disk format (``{run_name}-step{step:06d}.pt`` holding
``{"step", "model_state", "opt_state"}``, utils.py:584-619) so checkpoints are interchangeable;
``Ticker`` prints the same progress table (utils.py:20-215); ``Logger`` / ``Timer`` record the
same series and timings and draw them with Plotly (utils.py:270-543; plotly imported on demand,
the built-in dark template instead of the reference's custom one).
"""
from __future__ import annotations

import time
from collections import deque
from contextlib import contextmanager
from pathlib import Path

import numpy as np
import torch


class Checkpointer:
    """``{run_name}-step{step:06d}.pt`` files holding ``{"step", "model_state", "opt_state"}`` --
    the reference's payload and naming (utils.py:584-619), so either side loads the other's files.
    Writes go to a temporary name first and are renamed into place (a crash mid-save never leaves a
    truncated checkpoint under the final name); loads are weights-only (no pickle code runs);
    ``keep_last`` trims by step number, not by file-name order."""

    def __init__(self, folder: str | Path = "models", run_name: str = "run", *,
                 keep_last: int | None = None) -> None:
        self.folder = Path(folder)
        self.run_name = run_name
        self.keep_last = keep_last

    def path_for(self, step: int) -> Path:
        return self.folder / f"{self.run_name}-step{step:06d}.pt"

    def save(self, step: int, model: torch.nn.Module, optimizer=None) -> None:
        payload = {"step": step, "model_state": model.state_dict()}
        if optimizer is not None:
            payload["opt_state"] = optimizer.state_dict()
        self.folder.mkdir(parents=True, exist_ok=True)
        final = self.path_for(step)
        tmp = final.with_name(final.name + ".partial")
        torch.save(payload, tmp)
        tmp.replace(final)
        if self.keep_last is not None:
            for _, old in self._saved()[:-self.keep_last]:
                old.unlink(missing_ok=True)

    def load(self, path: str | Path, model: torch.nn.Module, optimizer=None) -> None:
        state = torch.load(path, map_location="cpu", weights_only=True)
        model.load_state_dict(state["model_state"])
        if optimizer is not None and "opt_state" in state:
            optimizer.load_state_dict(state["opt_state"])

    def _saved(self) -> list:
        """(step, path) of this run's checkpoints, oldest step first."""
        prefix = f"{self.run_name}-step"
        found = []
        for f in self.folder.glob(prefix + "*.pt"):
            digits = f.stem[len(prefix):]
            if digits.isdigit():
                found.append((int(digits), f))
        return sorted(found)


class Ticker:
    """Console progress of a training run (the reference's table, utils.py:20-215): episode
    returns / lengths per env, the mean over the last ``window_size`` finished episodes, and a
    progress row every ``print_every`` vector steps, rewritten in place (``\r``) and left standing
    at ``num_checkpoints`` evenly spaced rollout boundaries.  FPS counts from the last standing
    row; keyword scalars given to :meth:`tick` are appended as columns."""

    # (header, width) of the fixed columns
    COLUMNS = (("Progress", 8), ("Step", 9), ("Episode", 8), ("Mean Rew", 8), ("Mean Len", 7),
               ("FPS", 6), ("Time", 8))

    def __init__(self, total_steps: int, num_envs: int, rollout_steps: int, *,
                 window_size: int = 100, print_every: int = 5, num_checkpoints: int = 20,
                 verbose: bool = True) -> None:
        self.total_steps = total_steps
        self.num_envs = num_envs
        self.rollout_steps = rollout_steps
        self.window_size = window_size
        self.print_every = print_every
        self.verbose = verbose
        per_rollout = rollout_steps * num_envs
        rollouts = total_steps // per_rollout
        # the standing rows: after rollouts k * rollouts // num_checkpoints, k = 1 .. num_checkpoints
        marks = np.arange(1, num_checkpoints + 1) * rollouts // num_checkpoints
        self.checkpoints = marks * per_rollout
        self._marks = set(int(x) for x in self.checkpoints)
        self.reset()

    def reset(self) -> None:
        """Clear the counters and clocks; keep the configuration."""
        self.current_step = 0
        self.current_episode = 1
        self.current_returns = np.zeros(self.num_envs, np.float32)
        self.current_lengths = np.zeros(self.num_envs, np.int64)
        self.recent_returns: deque = deque(maxlen=self.window_size)
        self.recent_lengths: deque = deque(maxlen=self.window_size)
        self.custom_logs: dict = {}
        self._header_printed = False
        self.start_time = time.time()
        self._mark_time, self._mark_step = self.start_time, 0

    def tick(self, rewards, dones, **custom_logs) -> None:
        """One vector-env step (and any extra scalars to show)."""
        done = np.asarray(dones, dtype=bool)
        self.current_step += self.num_envs
        self.current_returns += np.asarray(rewards, dtype=np.float32)
        self.current_lengths += 1
        if done.any():
            self.recent_returns.extend(float(x) for x in self.current_returns[done])
            self.recent_lengths.extend(int(x) for x in self.current_lengths[done])
            self.current_episode += int(done.sum())
            self.current_returns[done] = 0.0
            self.current_lengths[done] = 0
        self.custom_logs.update(custom_logs)
        if self.verbose:
            self.print_logs()

    def _row(self, now: float) -> list:
        fps = (self.current_step - self._mark_step) / (now - self._mark_time + 1e-6)
        h, rem = divmod(int(now - self.start_time), 3600)
        hms = f"{h:02}:{rem // 60:02}:{rem % 60:02}"
        cells = [f"{100 * self.current_step / self.total_steps:>7.1f}%",
                 f"{self.current_step:>9,}", f"{self.current_episode:>8,}",
                 f"{np.mean(self.recent_returns):>8.2f}", f"{np.mean(self.recent_lengths):>8.1f}",
                 f"{fps:>6.0f}", f"{hms:>8}"]
        return cells + [f"{v:.2f}" if isinstance(v, float) else str(v)
                        for v in self.custom_logs.values()]

    def print_logs(self) -> None:
        """Rewrite the progress row when one is due; leave it standing at a checkpoint."""
        now = time.time()
        if self.current_step in self._marks:
            if self._header_printed:
                print()
            self._mark_time, self._mark_step = now, self.current_step
        due = self.current_step % (self.num_envs * self.print_every) == 0
        if not due or not self.recent_returns:
            return
        if not self._header_printed:
            head = "  |  ".join(f"{name:>{w}}" for name, w in self.COLUMNS)
            print(head + "".join(f"  |  {k}" for k in self.custom_logs))
            self._header_printed = True
        print("\r" + "  |  ".join(self._row(now)), end="")

    @property
    def logs(self) -> dict:
        """Summary of the run so far."""
        elapsed = time.time() - self.start_time
        return {"total_steps": self.current_step, "total_episodes": self.current_episode - 1,
                "episode_returns": list(self.recent_returns),
                "episode_lengths": list(self.recent_lengths),
                "best_reward": max(self.recent_returns, default=None),
                "total_duration": elapsed, "mean_fps": self.current_step / (elapsed + 1e-6),
                "custom_logs": dict(self.custom_logs)}


def _figure_out(fig, show: bool):
    if show:
        fig.show()
    return fig


class Logger:
    """Named scalar series over steps (reference utils.py:270-458) and an interactive Plotly view:
    ``plot(name)`` draws the raw series faintly under a moving-average line whose window
    (1 .. 10,000 points) a slider selects, or a scatter; series longer than ``max_samples`` are
    drawn from a uniform random subset.  ``plot`` returns the figure (``show=False`` only builds
    it); plotly is imported when a plot is asked for."""

    SMOOTHING_WINDOWS = (1, 5, 20, 100, 500, 2000, 10_000)

    def __init__(self) -> None:
        self.logs: dict = {}
        self.theme = "plotly_dark"

    def log(self, log_name: str, step: int, value) -> None:
        series = self.logs.setdefault(log_name, {"steps": [], "values": []})
        series["steps"].append(step)
        series["values"].append(value)

    @staticmethod
    def _subsample(x: np.ndarray, y: np.ndarray, max_samples: int | None, mode: str = "uniform"):
        if max_samples is None or len(x) <= max_samples:
            return x, y
        if mode != "uniform":
            raise ValueError(f"Unknown subsample_mode: {mode}")
        keep = np.sort(np.random.choice(len(x), max_samples, replace=False))
        return x[keep], y[keep]

    def plot(self, log_name: str, mode: str = "line", scale: str = "linear",
             max_samples: int | None = 10_000, subsample_mode: str = "uniform", show: bool = True):
        assert log_name in self.logs, f"No log called {log_name!r}"
        import plotly.graph_objects as go
        x = np.asarray(self.logs[log_name]["steps"])
        y = np.asarray(self.logs[log_name]["values"])
        if mode not in ("line", "scatter"):
            raise ValueError(f"Unknown mode {mode!r}; use 'line' or 'scatter'.")
        if y.ndim != 1:
            raise ValueError(f"Log: {log_name} has data of shape: {y.shape} which is incompatible "
                             f"with mode={mode!r}.")
        fig = go.Figure()
        if mode == "scatter":
            xs, ys = self._subsample(x, y, max_samples, subsample_mode)
            fig.add_trace(go.Scatter(x=xs, y=ys, mode="markers", name=log_name,
                                     marker={"size": 4, "opacity": 0.7}))
        else:
            # moving averages over the full series, then one common subset of points
            smooth = [y if w == 1 else np.convolve(y, np.ones(w) / w, mode="same")
                      for w in self.SMOOTHING_WINDOWS]
            keep = (np.arange(len(x)) if max_samples is None or len(x) <= max_samples
                    else np.sort(np.random.choice(len(x), max_samples, replace=False)))
            fig.add_trace(go.Scatter(x=x[keep], y=y[keep], mode="lines", opacity=0.15,
                                     line={"width": 1, "color": "#c8c8c8"}, showlegend=False))
            for i, sm in enumerate(smooth):
                fig.add_trace(go.Scatter(x=x[keep], y=sm[keep], mode="lines", line={"width": 2},
                                         showlegend=False, visible=i == 0))
            n = len(self.SMOOTHING_WINDOWS)
            fig.update_layout(showlegend=False, sliders=[{
                "active": 0, "currentvalue": {"prefix": "Smoothing: "}, "x": 0.67, "y": 1.27,
                "len": 0.3, "steps": [{"method": "update", "label": str(w),
                                       "args": [{"visible": [True] + [j == i for j in range(n)]}]}
                                      for i, w in enumerate(self.SMOOTHING_WINDOWS)]}])
        fig.update_layout(template=self.theme, title=log_name, height=420, width=960,
                          yaxis={"type": scale}, xaxis_title="Step",
                          margin={"l": 40, "r": 20, "t": 60, "b": 40})
        return _figure_out(fig, show)


class Timer:
    """Named code-block timings (reference utils.py:461-543): ``with timer.time(name):`` keeps a
    running mean and a count per name; ``plot_timings`` draws the total time per block, largest
    first, as a Plotly bar chart (returned; ``show=False`` only builds it)."""

    def __init__(self) -> None:
        self.timings: dict = {}

    def reset(self) -> None:
        self.timings = {}

    @contextmanager
    def time(self, name: str):
        t0 = time.time()
        try:
            yield
        finally:
            dt = time.time() - t0
            rec = self.timings.setdefault(name, {"avg_time": 0.0, "count": 0})
            rec["count"] += 1
            rec["avg_time"] += (dt - rec["avg_time"]) / rec["count"]

    def mean(self, name: str) -> float:
        rec = self.timings.get(name)
        return float(rec["avg_time"]) if rec else float("nan")

    def plot_timings(self, show: bool = True):
        if not self.timings:
            print("No timings to plot.")
            return None
        import plotly.graph_objects as go
        totals = sorted(((r["avg_time"] * r["count"], k) for k, r in self.timings.items()),
                        reverse=True)
        fig = go.Figure(go.Bar(x=[k for _, k in totals], y=[t for t, _ in totals],
                               text=[f"{t:.4f}s" for t, _ in totals], textposition="outside",
                               showlegend=False, hovertemplate="%{y:.6f}s<extra></extra>"))
        fig.update_layout(template="plotly_dark", title="Code Timings", height=480, width=960,
                          yaxis_title="Total Time (seconds)", xaxis={"tickangle": -45},
                          margin={"l": 80, "r": 20, "t": 60, "b": 120})
        return _figure_out(fig, show)
