"""Ticker / Logger / Timer behaviour (reference diamond/utils.py:20-543), host only."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-ppo_amd"))

from diamond.utils import Logger, Ticker, Timer  # noqa: E402


def test_ticker_episodes_checkpoints_and_table(capsys):
    t = Ticker(total_steps=4 * 2 * 10, num_envs=4, rollout_steps=2, print_every=1,
               num_checkpoints=5, verbose=True)
    # 10 rollouts of 2 steps x 4 envs: rows kept at rollouts 2, 4, 6, 8, 10
    assert list(t.checkpoints) == [16, 32, 48, 64, 80]
    rng = np.random.default_rng(0)
    ends = []
    for step in range(20):
        r = np.full(4, 1.0, np.float32)
        d = rng.random(4) < 0.3
        ends += [int(x) for x in np.flatnonzero(d)]
        t.tick(r, d, lr=0.5)
    out = capsys.readouterr().out
    assert out.startswith("Progress  |")
    assert "  |  lr" in out.splitlines()[0]
    assert out.count("\r") > 0 and "0.50" in out
    logs = t.logs
    assert logs["total_steps"] == 80 and logs["total_episodes"] == len(ends)
    # every finished episode's return equals its length (reward 1 per step)
    assert logs["episode_returns"] == [float(x) for x in logs["episode_lengths"]]
    assert logs["custom_logs"] == {"lr": 0.5}
    t.reset()
    assert t.current_step == 0 and t.logs["total_episodes"] == 0 and not t.recent_returns


def test_ticker_quiet_until_an_episode_ends(capsys):
    t = Ticker(total_steps=100, num_envs=2, rollout_steps=5, print_every=1)
    t.tick(np.ones(2), np.zeros(2, bool))
    assert capsys.readouterr().out == ""
    t.tick(np.ones(2), np.array([True, False]))
    assert "Progress" in capsys.readouterr().out


def test_logger_series_and_plots():
    lg = Logger()
    for s in range(300):
        lg.log("loss", s, 1.0 / (s + 1))
    assert lg.logs["loss"]["steps"][:3] == [0, 1, 2]
    fig = lg.plot("loss", show=False)
    assert len(fig.data) == 1 + len(Logger.SMOOTHING_WINDOWS)
    assert [tr.visible for tr in fig.data[1:]] == [True] + [False] * 6
    assert len(fig.layout.sliders[0].steps) == len(Logger.SMOOTHING_WINDOWS)
    fig = lg.plot("loss", mode="scatter", scale="log", max_samples=50, show=False)
    assert len(fig.data) == 1 and len(fig.data[0].x) == 50 and fig.layout.yaxis.type == "log"
    with pytest.raises(ValueError):
        lg.plot("loss", mode="bars", show=False)
    with pytest.raises(AssertionError):
        lg.plot("missing", show=False)
    x, y = Logger._subsample(np.arange(10), np.arange(10), None)
    assert len(x) == 10


def test_timer_running_mean_and_plot():
    tm = Timer()
    for _ in range(3):
        with tm.time("a"):
            pass
    with tm.time("b"):
        sum(range(20000))
    assert tm.timings["a"]["count"] == 3 and tm.timings["b"]["count"] == 1
    assert tm.mean("a") >= 0.0
    fig = tm.plot_timings(show=False)
    assert list(fig.data[0].x)[0] == "b"  # largest total first
    tm.reset()
    assert tm.timings == {} and tm.plot_timings(show=False) is None
