#!/usr/bin/env python3
"""Time the fused minibatch kernel of one or more libdppo builds (ablation variants), each in a
fresh subprocess, on the CartPole bench shape: median us per dppo_minibatch_grad_f32 launch
(HIP-event timing class 'grad').  Usage: python tools/ablate.py lib1.so lib2.so ..."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import ctypes, json, os, sys, numpy as np, torch
sys.path.insert(0, os.path.join(ROOT, "diamond-ppo_amd")); sys.path.insert(0, ROOT)
import bench, diamond
from diamond import _native as N
T, Nn, D, A = 128, int(os.environ.get("ABL_N", "4096")), 4, 2
cfg = diamond.PPOConfig(rollout_steps=T, num_envs=Nn, verbose=False)
agent = diamond.PPO(None, cfg, envs=bench.SpecEnvs(D, A, False))
dev = agent.device
ro, _ = bench.synth_rollout(T, Nn, D, A, False, 0.02, 0.005, 0, dev)
agent.learn_device(ro); torch.cuda.synchronize()
L = agent._learner; h = L.handle
hp = diamond.engine.hparams(cfg, cfg.lr, 0)
mb = T * Nn // 8
idx = torch.randperm(T * Nn, device=dev)[:mb].to(torch.int32)
g = torch.zeros(L.flat.total, device=dev)
s = torch.cuda.current_stream().cuda_stream
for _ in range(5):
    N.check(h.lib.dppo_minibatch_grad_f32(h.h, L.flat.flat.data_ptr(), idx.data_ptr(), mb, mb, ctypes.byref(hp), g.data_ptr(), None, s))
h.set_timing(True)
for _ in range(50):
    N.check(h.lib.dppo_minibatch_grad_f32(h.h, L.flat.flat.data_ptr(), idx.data_ptr(), mb, mb, ctypes.byref(hp), g.data_ptr(), None, s))
t = h.timing()
print(json.dumps({k: round(v[0] / max(v[1], 1) * 1e3, 2) for k, v in t.items() if v[1]}))
"""


def main():
    res = {}
    for lib in sys.argv[1:]:
        env = dict(os.environ, DPPO_LIB=os.path.abspath(lib))
        out = subprocess.run([sys.executable, "-c", "ROOT=%r\n" % ROOT + CHILD], env=env,
                             capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        res[os.path.basename(lib)] = json.loads(line[-1]) if line else out.stderr[-500:]
        print(os.path.basename(lib), res[os.path.basename(lib)], flush=True)


if __name__ == "__main__":
    main()
