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
    """Live training progress (reference utils.py:20-215): per-env episode returns / lengths,
    a moving window of finished episodes, and one progress row per ``print_every`` vector steps,
    rewritten in place (``\r``) and kept as its own line at each of ``num_checkpoints`` evenly
    spaced rollout boundaries.  FPS is measured since the last checkpoint; extra keyword scalars
    passed to :meth:`tick` become extra columns."""

    def __init__(self, total_steps: int, num_envs: int, rollout_steps: int, *,
                 window_size: int = 100, print_every: int = 5, num_checkpoints: int = 20,
                 verbose: bool = True) -> None:
        self.total_steps = total_steps
        self.num_envs = num_envs
        self.rollout_steps = rollout_steps
        self.window_size = window_size
        self.print_every = print_every
        self.verbose = verbose
        # rollout-aligned steps at which a row is kept: i * (iterations // n) rollouts, i = 1..n
        per_rollout = rollout_steps * num_envs
        iters = total_steps // per_rollout
        self.checkpoints = (np.arange(1, num_checkpoints + 1) * iters // num_checkpoints) * per_rollout
        self._start_state()

    def _start_state(self) -> None:
        self.current_step = 0
        self.current_episode = 1
        self.current_returns = np.zeros(self.num_envs, np.float32)
        self.current_lengths = np.zeros(self.num_envs, np.int64)
        self.recent_returns: deque = deque(maxlen=self.window_size)
        self.recent_lengths: deque = deque(maxlen=self.window_size)
        self.custom_logs: dict = {}
        self._header_printed = False
        self.start_time = time.time()
        self.last_checkpoint_time = self.start_time
        self.last_checkpoint_step = 0

    def reset(self) -> None:
        """Clear the counters and clocks; keep the configuration."""
        self._start_state()

    def tick(self, rewards, dones, **custom_logs) -> None:
        """One vector-env step (and any extra scalars to show)."""
        done = np.asarray(dones, dtype=bool)
        self.current_step += self.num_envs
        self.current_returns += np.asarray(rewards, dtype=np.float32)
        self.current_lengths += 1
        for r, n in zip(self.current_returns[done], self.current_lengths[done]):
            self.recent_returns.append(float(r))
            self.recent_lengths.append(int(n))
            self.current_episode += 1
        self.current_returns[done] = 0.0
        self.current_lengths[done] = 0
        self.custom_logs.update(custom_logs)
        if self.verbose:
            self.print_logs()

    def print_logs(self) -> None:
        """Print (overwrite) the progress row when due; keep it at a checkpoint."""
        now = time.time()
        if self.current_step in self.checkpoints:
            if self._header_printed:
                print()
            self.last_checkpoint_time, self.last_checkpoint_step = now, self.current_step
        if self.current_step % (self.num_envs * self.print_every) or not self.recent_returns:
            return
        if not self._header_printed:
            cols = ["Progress", "Step", "Episode", "Mean Rew", "Mean Len", "FPS", "Time"]
            widths = [8, 9, 8, 8, 7, 6, 8]
            print("  |  ".join(f"{c:>{w}}" for c, w in zip(cols, widths)) +
                  "".join(f"  |  {k}" for k in self.custom_logs))
            self._header_printed = True
        fps = (self.current_step - self.last_checkpoint_step) / (now - self.last_checkpoint_time
                                                                  + 1e-6)
        cells = [f"{100 * self.current_step / self.total_steps:>7.1f}%",
                 f"{self.current_step:>9,}", f"{self.current_episode:>8,}",
                 f"{np.mean(self.recent_returns):>8.2f}", f"{np.mean(self.recent_lengths):>8.1f}",
                 f"{fps:>6.0f}", f"{self._hms(now - self.start_time):>8}"]
        cells += [f"{v:.2f}" if isinstance(v, float) else f"{v}" for v in self.custom_logs.values()]
        print("\r" + "  |  ".join(cells), end="")

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

    @staticmethod
    def _hms(seconds: float) -> str:
        h, rem = divmod(int(seconds), 3600)
        m, sec = divmod(rem, 60)
        return f"{h:02}:{m:02}:{sec:02}"


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
