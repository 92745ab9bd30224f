"""The learn() driver shared by PPO and ContinuousPPO.

Host side of the hot path (reference ``diamond/ppo.py:224-287``): it owns the flat parameter /
Adam buffers the gfx950 kernels update in place, keeps the reference's ``nn.Module`` and
``torch.optim.Adam`` objects as live views of those buffers (so ``state_dict()``, checkpoints and
``LinearLR`` behave exactly as in the reference), draws the minibatch permutations from the global
NumPy RNG bit-exactly, and issues ONE native call per learn().

Permutations (ppo.py:252-254) are produced off the critical path: the permutations for learn k+1
are drawn on a host thread while learn k is enqueued and runs, from the RNG state learn k leaves
behind (``dppo_perm_numpy``: one sequential MT19937 stream, each epoch's Fisher-Yates swaps on a
worker thread of their own).  Learn k+1 uses them only if the global NumPy RNG still holds
exactly that state (otherwise it draws afresh), so results and the RNG stream stay bit-identical
to the reference's.  For large batches (E*B >= 2^23 entries, or ``DPPO_PERM_DEVICE=1``) the host
only draws the swap targets and the GPU resolves the swaps (``shuffle.hip``,
``dppo_learn_targets_f32``): the host swap chain is cache-miss bound at those sizes.

Two paths, chosen once per agent:

* **fused** -- default network at supported sizes (hidden 64, obs_dim <= 32, actions <= 16):
  everything in ``dppo_learn_f32`` (old-policy eval, GAE, normalisation, E x M fused
  minibatch steps with clip + Adam, RCCL all-reduces when sharded).
* **generic** -- any other ``network_cls`` (reference readme.md:89-111): the network's own
  methods run forward/backward under torch autograd on the GPU; GAE, advantage statistics and
  normalisation, and clip + Adam run in the HIP kernels (SURVEY.md §7.2 hard part 7).
"""
from __future__ import annotations

import collections
import ctypes
import os
import socket
import threading
import warnings
import time
from dataclasses import dataclass

import numpy as np
import torch

from . import _native as N


def require_gpu(cfg_device_index: int = 0) -> torch.device:
    """The product path runs on the MI355X only; fail loudly otherwise (no CPU fallback)."""
    if not torch.cuda.is_available():
        raise RuntimeError("diamond (MI355X build) requires a HIP GPU; none is visible. "
                           "The reference's CPU path is not part of this package.")
    N.load()
    idx = cfg_device_index
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        import os
        idx = int(os.environ.get("LOCAL_RANK", idx))
    return torch.device("cuda", idx)


_SOLO = [False]


class solo:
    """``with engine.solo():`` agents built inside ignore an initialised torch.distributed group
    and run as one rank (bench.py measures its world-1 anchor on rank 0 inside an N-rank job)."""

    def __enter__(self):
        _SOLO[0] = True

    def __exit__(self, *exc):
        _SOLO[0] = False


def dist_world():
    d = torch.distributed
    if not _SOLO[0] and d.is_available() and d.is_initialized():
        return d.get_world_size(), d.get_rank()
    return 1, 0


# ---------------------------------------------------------------------------------------------
class FlatParams:
    """Re-home every parameter of ``module`` into one flat device buffer at the given offsets
    (tensors in ``named_parameters()`` order).  Parameters become views, so the module, its
    ``state_dict()`` and the optimizer all see the values the kernels write."""

    def __init__(self, module: torch.nn.Module, device, offsets=None, total=None):
        params = list(module.parameters())
        if offsets is None:
            offsets, off = [], 0
            for p in params:
                offsets.append(off)
                off = (off + p.numel() + 15) // 16 * 16
            total = off
        self.offsets = list(offsets)
        self.total = int(total)
        self.shapes = [tuple(p.shape) for p in params]
        self.numels = [p.numel() for p in params]
        self.flat = torch.zeros(self.total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.total + 8, dtype=torch.float32, device=device)
        with torch.no_grad():
            for p, o, n, s in zip(params, self.offsets, self.numels, self.shapes):
                self.flat[o:o + n].copy_(p.detach().reshape(-1).to(device))
                p.data = self.flat[o:o + n].view(s)
        self.params = params

    def views(self, buf):
        return [buf[o:o + n].view(s) for o, n, s in zip(self.offsets, self.numels, self.shapes)]

    def bind_grads(self):
        """Make p.grad views of the flat grad buffer (autograd accumulates into them in place)."""
        for p, g in zip(self.params, self.views(self.grad)):
            p.grad = g


def bind_adam_state(optimizer: torch.optim.Adam, flat: FlatParams):
    """Initialise torch Adam's per-parameter state as views of flat exp_avg / exp_avg_sq buffers
    (the layout torch would create lazily at the first step: optim/adam.py _init_group)."""
    m = torch.zeros_like(flat.flat)
    v = torch.zeros_like(flat.flat)
    for p, mv, vv in zip(flat.params, flat.views(m), flat.views(v)):
        optimizer.state[p] = {"step": torch.tensor(0.0, dtype=torch.float32),
                              "exp_avg": mv, "exp_avg_sq": vv}
    return m, v


def adam_step_count(optimizer, flat: FlatParams) -> int:
    st = optimizer.state.get(flat.params[0])
    return int(st["step"].item()) if st and "step" in st else 0


def advance_adam_steps(optimizer, flat: FlatParams, k: int):
    for p in flat.params:
        optimizer.state[p]["step"] += float(k)


def rebind_after_load(optimizer, flat: FlatParams, m, v):
    """After optimizer.load_state_dict (which replaces state tensors), copy values back into the
    flat buffers and restore the views."""
    with torch.no_grad():
        for p, mv, vv in zip(flat.params, flat.views(m), flat.views(v)):
            st = optimizer.state[p]
            if "exp_avg" in st and st["exp_avg"].data_ptr() != mv.data_ptr():
                mv.copy_(st["exp_avg"])
                vv.copy_(st["exp_avg_sq"])
                st["exp_avg"], st["exp_avg_sq"] = mv, vv
            if not isinstance(st.get("step"), torch.Tensor):
                st["step"] = torch.tensor(float(st.get("step", 0.0)), dtype=torch.float32)


# ---------------------------------------------------------------------------------------------
@dataclass
class DeviceRollout:
    """SoA rollout buffer resident in HBM (layouts in include/dppo.h)."""
    obs: torch.Tensor          # float32 [T, N, D]
    next_obs: torch.Tensor     # float32 [T, N, D]
    actions: torch.Tensor      # int32 [T, N] or float32 [T, N, A]
    rewards: torch.Tensor      # float32 [T, N]
    term: torch.Tensor         # uint8 [T, N]
    trunc: torch.Tensor        # uint8 [T, N]

    def check(self, T, N, D, A, continuous):
        def need(t, shape, dtype, name):
            if tuple(t.shape) != shape or t.dtype != dtype or not t.is_contiguous() or not t.is_cuda:
                raise ValueError(f"{name}: expected contiguous {dtype} {shape} on GPU, got "
                                 f"{t.dtype} {tuple(t.shape)} on {t.device}")
        need(self.obs, (T, N, D), torch.float32, "obs")
        need(self.next_obs, (T, N, D), torch.float32, "next_obs")
        if continuous:
            need(self.actions, (T, N, A), torch.float32, "actions")
        else:
            need(self.actions, (T, N), torch.int32, "actions")
        need(self.rewards, (T, N), torch.float32, "rewards")
        need(self.term, (T, N), torch.uint8, "term")
        need(self.trunc, (T, N), torch.uint8, "trunc")

    def as_struct(self) -> N.Rollout:
        return N.Rollout(self.obs.data_ptr(), self.next_obs.data_ptr(), self.actions.data_ptr(),
                         self.rewards.data_ptr(), self.term.data_ptr(), self.trunc.data_ptr())


def stage_experience(experience, device, continuous) -> DeviceRollout:
    """Stack the rollout lists (ppo.py:226-232) into SoA device tensors.  Host bytes go through
    pinned memory so the H2D copies are DMA transfers."""
    obs, next_obs, actions, rewards, terms, truncs = zip(*experience)

    def up(x, dtype):
        a = np.ascontiguousarray(np.asarray(x), dtype=dtype)
        return torch.from_numpy(a).pin_memory().to(device, non_blocking=True)

    act_dtype = np.float32 if continuous else np.int32
    return DeviceRollout(up(obs, np.float32), up(next_obs, np.float32), up(actions, act_dtype),
                         up(rewards, np.float32), up(terms, np.uint8), up(truncs, np.uint8))


class RolloutStager:
    """Per-step staging of a rollout into the SoA HBM buffer while the envs step.

    ``put(t, ...)`` copies step t's arrays into row t of a pinned host slot and enqueues that
    row's host->device copy on a side stream, so the PCIe transfer of a rollout overlaps the
    environment stepping instead of following it (``stage_experience`` stacks and uploads the
    whole rollout inside learn()).  Two slots alternate: a slot's pinned rows are rewritten only
    after its previous copies completed (``end`` marks them), and its device buffers only after
    the learn() that read them (``release``).  ``finish()`` returns the device rollout and makes
    the caller's stream wait for the copies."""

    def __init__(self, T: int, N: int, obs_shape, act_shape, continuous: bool, device):
        self.T, self.N, self.device = T, N, device
        self.continuous = bool(continuous)
        D = int(np.prod(obs_shape))
        A = int(np.prod(act_shape)) if continuous else 1
        self.D, self.A = D, A
        self.stream = torch.cuda.Stream(device=device)
        self.slots = []
        for _ in range(2):
            host = {
                "obs": torch.empty((T, N, D), dtype=torch.float32).pin_memory(),
                "next_obs": torch.empty((T, N, D), dtype=torch.float32).pin_memory(),
                "actions": (torch.empty((T, N, A), dtype=torch.float32) if continuous
                            else torch.empty((T, N), dtype=torch.int32)).pin_memory(),
                "rewards": torch.empty((T, N), dtype=torch.float32).pin_memory(),
                "term": torch.empty((T, N), dtype=torch.uint8).pin_memory(),
                "trunc": torch.empty((T, N), dtype=torch.uint8).pin_memory(),
            }
            dev = {k: torch.empty(v.shape, dtype=v.dtype, device=device) for k, v in host.items()}
            self.slots.append({"host": host, "dev": dev, "copied": None, "released": None,
                               "np": {k: v.numpy() for k, v in host.items()}})
        self.cur = 1
        self.rows = 0
        self.flushed = 0
        self.chunk = max(1, T // 8)  # rows per flush

    def begin(self) -> None:
        self.cur ^= 1
        sl = self.slots[self.cur]
        if sl["copied"] is not None:
            sl["copied"].synchronize()           # the pinned rows are free again
        if sl["released"] is not None:
            self.stream.wait_event(sl["released"])  # the learn() that read the device rows is done
        self.rows = 0
        self.flushed = 0

    def put(self, t: int, obs, next_obs, actions, rewards, term, trunc) -> None:
        sl = self.slots[self.cur]
        h = sl["np"]
        h["obs"][t] = np.reshape(obs, (self.N, self.D))
        h["next_obs"][t] = np.reshape(next_obs, (self.N, self.D))
        if self.continuous:
            h["actions"][t] = np.reshape(actions, (self.N, self.A))
        else:
            h["actions"][t] = actions
        h["rewards"][t] = rewards
        h["term"][t] = term
        h["trunc"][t] = trunc
        self.rows = t + 1
        if self.rows - self.flushed >= self.chunk:
            self._flush()

    def _flush(self) -> None:
        """Enqueue the host->device copies of the rows written since the last flush (one copy per
        array: the per-call cost, not the bytes, dominates at rollout-row sizes)."""
        sl = self.slots[self.cur]
        r0, r1 = self.flushed, self.rows
        if r1 > r0:
            with torch.cuda.stream(self.stream):
                for k, v in sl["host"].items():
                    sl["dev"][k][r0:r1].copy_(v[r0:r1], non_blocking=True)
        self.flushed = r1

    def end(self) -> None:
        """All rows written: flush the rest and mark the slot's copies (also when learn() never
        claims them)."""
        self._flush()
        ev = torch.cuda.Event()
        ev.record(self.stream)
        self.slots[self.cur]["copied"] = ev

    def finish(self) -> "DeviceRollout":
        if self.rows != self.T:
            raise ValueError(f"staged {self.rows} of {self.T} rollout steps")
        sl = self.slots[self.cur]
        torch.cuda.current_stream(self.device).wait_event(sl["copied"])
        d = sl["dev"]
        return DeviceRollout(d["obs"], d["next_obs"], d["actions"], d["rewards"], d["term"],
                             d["trunc"])

    def release(self) -> None:
        """Mark the current slot's device rows free once the work queued so far has run."""
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self.slots[self.cur]["released"] = ev


def hparams(cfg, lr: float, adam_step: int, betas=(0.9, 0.999)) -> N.HParams:
    return N.HParams(gamma=cfg.gamma, gae_lambda=cfg.gae_lambda, ppo_clip=cfg.ppo_clip,
                     value_loss_weight=cfg.value_loss_weight, entropy_beta=cfg.entropy_beta,
                     grad_norm_clip=cfg.grad_norm_clip, adam_beta1=betas[0], adam_beta2=betas[1],
                     adam_eps=cfg.adam_eps, advantage_norm=int(bool(cfg.advantage_norm)),
                     lr=float(lr), adam_step=int(adam_step))


# ---------------------------------------------------------------------------------------------
class _DraftWorker:
    """One long-lived host thread that runs the queued permutation drafts in order (a thread per
    learn cost ~0.7 ms of start-up on the launching thread).  ctypes releases the GIL during the
    draw."""

    def __init__(self):
        self._cv = threading.Condition()
        self._jobs = collections.deque()
        self._thread = threading.Thread(target=self._run, name="dppo-perm-draft", daemon=True)
        self._thread.start()

    def submit(self, fn, done: threading.Event):
        with self._cv:
            self._jobs.append((fn, done))
            self._cv.notify()

    def stop(self, timeout: float = 60.0):
        """Run what is queued, then end the thread (a None job is the stop mark)."""
        with self._cv:
            self._jobs.append((None, None))
            self._cv.notify()
        if threading.current_thread() is not self._thread:
            self._thread.join(timeout)

    def _run(self):
        while True:
            with self._cv:
                while not self._jobs:
                    self._cv.wait()
                fn, done = self._jobs.popleft()
            if fn is None:
                return
            try:
                fn()
            except Exception as e:  # the draft stays not-ok: its learn redraws on its own thread
                warnings.warn(f"permutation draft failed ({e!r}); the learn draws it itself")
            finally:
                done.set()
            # the finished job's closure must not outlive it: it holds the draft's buffers
            del fn, done


class NativeLearner:
    """Binds one agent (network + Adam) to a libdppo handle for its rollout shape."""

    PERM_DEVICE_MIN = 1 << 23  # E*B permutation entries above which the GPU resolves the swaps

    def __init__(self, network, optimizer, cfg, obs_dim, act_dim, continuous, device,
                 network_is_default: bool):
        self.cfg = cfg
        self.device = device
        self.continuous = bool(continuous)
        self.world, self.rank = dist_world()
        self.T, self.N = cfg.rollout_steps, cfg.num_envs
        self.D, self.A = obs_dim, act_dim
        # global minibatches (cfg.global_minibatches, world > 1): the permutations span the
        # global batch of T * N * world samples and libdppo keeps this rank's members of each
        self.global_mb = bool(getattr(cfg, "global_minibatches", False)) and self.world > 1
        self.dims = N.Dims(rollout_steps=self.T, num_envs=self.N, obs_dim=obs_dim,
                           act_dim=act_dim, continuous=int(continuous),
                           hidden=int(cfg.network_hidden_dim), num_epochs=cfg.num_epochs,
                           num_minibatches=cfg.num_minibatches, world_size=self.world,
                           rank=self.rank, global_minibatches=int(self.global_mb))
        self.perm_n = self.T * self.N * (self.world if self.global_mb else 1)
        self.handle = N.Handle(device.index or 0, self.dims)
        if not getattr(cfg, "gae_bitexact", True):
            self.handle.set_gae_mode(N.GAE_AFFINE)
        L = self.handle.layout
        names = [n for n, _ in network.named_parameters()]
        shapes_ok = network_is_default and L.count == len(names) and all(
            tuple(p.shape) in ((L.rows[i], L.cols[i]), (L.rows[i],)) for i, (_, p) in
            enumerate(network.named_parameters()))
        self.fused = bool(shapes_ok and cfg.network_hidden_dim == 64 and obs_dim <= 32
                          and act_dim <= 16)
        if self.fused:
            self.flat = FlatParams(network, device, [L.offset[i] for i in range(L.count)], L.total)
        else:
            self.flat = FlatParams(network, device)
            self.flat.bind_grads()
        self.m, self.v = bind_adam_state(optimizer, self.flat)
        self.optimizer = optimizer
        self.network = network
        # DPPO_FORCE_COMM=1: an RCCL communicator even for one rank, so learn() runs the
        # collective sequence (slab reduce -> ncclAllReduce -> clip + Adam) -- how the RCCL path
        # is exercised on a one-GPU box
        if self.world > 1 or os.environ.get("DPPO_FORCE_COMM") == "1":
            self._init_comm()
        self.last_trace = None
        # host-side seconds of learn(), reported by bench.py.  Launching thread: "perms" (waiting
        # for the look-ahead draft), "draft_start" (queueing the next drafts, including
        # "slot_wait": device back-pressure on a pinned slot) and "enqueue" (the native learn
        # call).  Draft thread: "draw" (the permutation draws: the host's own work per learn).
        self.host_seconds = {"perms": 0.0, "enqueue": 0.0, "draft_start": 0.0, "draw": 0.0,
                             "slot_wait": 0.0, "calls": 0, "lookahead_hits": 0}
        # host-load guard (round 6): draws that turn slow re-choose the swap pool's L3 domain
        self._draw_hist = collections.deque(maxlen=8)
        self._slow_draws = 0
        self._last_repin = 0.0
        self.repin_requests = 0
        self.lookahead = os.environ.get("DPPO_PERM_LOOKAHEAD", "1") != "0"
        # Where the Fisher-Yates swaps run.  The host's swap chain is cache-miss bound once the
        # [E][B] permutations outgrow the caches (C5 on one GPU, E*B = 33.5 M: ~46 ms of host
        # time per learn against ~32 ms of device time), so above PERM_DEVICE_MIN entries the
        # host only draws the MT19937 swap targets and the GPU resolves the swaps (shuffle.hip,
        # bit-identical).  DPPO_PERM_DEVICE=0/1 forces either side.
        env = os.environ.get("DPPO_PERM_DEVICE")
        self.device_shuffle = (env == "1") if env in ("0", "1") else (
            cfg.num_epochs * self.perm_n >= self.PERM_DEVICE_MIN)
        # look-ahead drafts in flight (FIFO), each chained on its predecessor's final RNG state;
        # DPPO_PERM_DEPTH (default 2) of them, in the handle's 3 pinned slots beside the one the
        # current learn uploads from -- two deep, a slow draw (host jitter) is absorbed instead
        # of stalling the next learn.  (Round 6 measured 3 deep in 4 slots: 286.4 against 287.7 M
        # env-steps/s at C3, 3 A/B pairs -- not kept.)
        self._drafts = collections.deque()
        self.draft_depth = max(1, min(N.PERM_SLOTS - 1,
                                      int(os.environ.get("DPPO_PERM_DEPTH", "2"))))
        self._slot = 0
        self._worker = None
        self._closed = False
        # global minibatches: the node's ranks share one draw per learn (drawshare.py;
        # DPPO_PERM_SHARE=0 keeps one draw per rank)
        self.share = None
        self._cur_share = None
        d = torch.distributed
        if not _SOLO[0] and d.is_available() and d.is_initialized():
            # setup() is a collective: enter it on every rank or on none (the enable inputs are
            # per-process environment and sizing, so the ranks agree on them first)
            want = (self.global_mb and self.device_shuffle and self.lookahead
                    and os.environ.get("DPPO_PERM_SHARE", "1") != "0")
            if self._all_ranks(d, want):
                from . import drawshare
                self.share = drawshare.setup(d, self)

    def _init_comm(self):
        """The rank exchange of the data-parallel learn.  DPPO_COMM: "auto" (default) = an RCCL
        communicator plus, for 2-8 ranks, the peer exchange (csrc/peer.hip: one-shot all-reduce
        over the ranks' xGMI-mapped buffers) when every rank maps every buffer and passes its
        self-test -- otherwise RCCL carries the exchange; "rccl" = RCCL only; "peer" = the peer
        exchange only (no communicator; also how two ranks share one GPU in the tests)."""
        d = torch.distributed
        self.peer = False
        mode = os.environ.get("DPPO_COMM", "auto")
        if mode not in ("auto", "rccl", "peer"):
            raise ValueError(f"DPPO_COMM={mode!r}: expected auto, rccl or peer")
        self.peer_status = "not run"
        if _SOLO[0] or not (d.is_available() and d.is_initialized()):   # one rank, no group
            if mode == "peer":   # (DPPO_FORCE_COMM=1: the 1-rank exchange, measurements)
                h = self.handle
                err = h.peer_open(1, 0, h.peer_export()) or h.peer_selftest(
                    torch.cuda.current_stream(self.device).cuda_stream)
                if err:
                    raise RuntimeError(f"peer exchange unavailable: {err}")
                self.peer = True
            else:
                self.handle.comm_init(1, 0, N.comm_unique_id())
            return
        if mode != "peer":
            obj = [N.comm_unique_id() if self.rank == 0 else None]
            d.broadcast_object_list(obj, src=0)
            self.handle.comm_init(self.world, self.rank, obj[0])
        if mode == "peer" or (mode == "auto" and 1 < self.world <= 8):
            self.peer = self._init_peer(d, required=mode == "peer")
        # replicate rank 0's initial parameters (identical seeds make this a no-op in practice)
        if d.get_backend() == "nccl":
            d.broadcast(self.flat.flat, src=0)
        else:
            cpu = self.flat.flat.cpu()
            d.broadcast(cpu, src=0)
            self.flat.flat.copy_(cpu)

    def _all_ranks(self, d, ok: bool) -> bool:
        dev = self.device if d.get_backend() == "nccl" else "cpu"
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        d.all_reduce(t, op=d.ReduceOp.MIN)
        return bool(t.item())

    def _gpu_identity(self):
        """(host, PCI domain, bus, device) of this rank's GPU: ranks with equal identities share
        one device."""
        pr = torch.cuda.get_device_properties(self.device)
        return (socket.gethostname(), pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id)

    def _init_peer(self, d, required: bool) -> bool:
        """Map every rank's exchange buffer and run one checked exchange; every rank keeps the
        peer exchange only if every rank succeeded (ranks must never disagree on the transport)."""
        h = self.handle
        # test hooks (DPPO_TEST_HOOKS=1, csrc/capi.cpp test_hook) must agree across ranks: a
        # sequence start that differs between ranks would stall every exchange
        hooks = ((os.environ.get("DPPO_PEER_XSEQ0"), os.environ.get("DPPO_PEER_SELFTEST_SKEW"))
                 if os.environ.get("DPPO_TEST_HOOKS") == "1" else None)
        me = (h.peer_export(), self._gpu_identity(), hooks)
        mine = [None] * self.world
        d.all_gather_object(mine, me)
        gpus = [m[1] for m in mine]
        if len({m[2][0] if m[2] else None for m in mine}) > 1:
            err = "DPPO_PEER_XSEQ0 differs across ranks"
        else:
            err = h.peer_open(self.world, self.rank, b"".join(m[0] for m in mine),
                              shared_device=len(set(gpus)) < len(gpus))
        if self._all_ranks(d, not err):
            err = h.peer_selftest(torch.cuda.current_stream(self.device).cuda_stream)
            if self._all_ranks(d, not err):
                self.peer_status = "passed"
                return True
            h.peer_close()
            self.peer_status = f"self-test failed: {err or 'on another rank'}"
        else:
            if not err:
                h.peer_close()
            self.peer_status = f"mapping failed: {err or 'on another rank'}"
        msg = f"peer exchange unavailable on rank {self.rank}: {err or 'another rank failed'}"
        if required:
            raise RuntimeError(msg)
        warnings.warn(msg + "; RCCL carries the exchange")
        return False

    # -----------------------------------------------------------------------------------------
    def act(self, observations: np.ndarray, seed: int, squash=None):
        """Sample actions for a batch of observations with the fused actor kernel
        (``dppo_act_f32``; default network only): pinned upload, one launch, pinned download.
        Discrete actions come back int64 like the reference's ``Categorical.sample().numpy()``;
        continuous ones float32 ``[n, A]``.

        ``squash`` (continuous only, the tanh-squash extension): ``True`` for tanh(u), or a
        ``(low, high)`` pair of A-float bounds; then the same kernel launch also emits the
        environment's actions (``dppo_act_squash_f32``) and ``(u, env_actions)`` is returned."""
        if not self.fused:
            raise RuntimeError("act() needs the default network (fused path)")
        if squash is not None and squash is not False:
            return self._act_squash(observations, seed, squash)
        obs = np.asarray(observations, dtype=np.float32).reshape(-1, self.D)
        n = obs.shape[0]
        b = getattr(self, "_act_bufs", None)
        if b is None or b["n"] != n:
            dt = torch.float32 if self.continuous else torch.int32
            shp = (n, self.A) if self.continuous else (n,)
            b = {"n": n, "obs_h": torch.empty((n, self.D), dtype=torch.float32).pin_memory(),
                 "obs_d": torch.empty((n, self.D), dtype=torch.float32, device=self.device),
                 "act_d": torch.empty(shp, dtype=dt, device=self.device),
                 "act_h": torch.empty(shp, dtype=dt).pin_memory()}
            self._act_bufs = b
        b["obs_h"].numpy()[:] = obs
        b["obs_d"].copy_(b["obs_h"], non_blocking=True)
        s = torch.cuda.current_stream(self.device)
        N.check(self.handle.lib.dppo_act_f32(self.handle.h, self.flat.flat.data_ptr(),
                                             b["obs_d"].data_ptr(), n, seed & (2 ** 64 - 1),
                                             self._next_act_counter(), b["act_d"].data_ptr(),
                                             s.cuda_stream), "dppo_act_f32")
        b["act_h"].copy_(b["act_d"], non_blocking=True)
        s.synchronize()
        out = b["act_h"].numpy()
        return out.copy() if self.continuous else out.astype(np.int64)

    def _next_act_counter(self) -> int:
        """The Philox call counter of the action samplers: ONE sequence shared by act() and the
        squashing sampler, so no two calls with the same seed reuse a noise draw."""
        c = self.__dict__.get("_act_counter", 0)
        self._act_counter = c + 1
        return c

    def _act_squash(self, observations, seed, squash):
        if not self.continuous:
            raise ValueError("tanh squash needs a continuous action space")
        obs = np.asarray(observations, dtype=np.float32).reshape(-1, self.D)
        n = obs.shape[0]
        b = getattr(self, "_sq_bufs", None)
        if b is None or b["n"] != n:
            b = {"n": n, "obs_h": torch.empty((n, self.D), dtype=torch.float32).pin_memory(),
                 "obs_d": torch.empty((n, self.D), dtype=torch.float32, device=self.device),
                 "out_d": torch.empty((2, n, self.A), dtype=torch.float32, device=self.device),
                 "out_h": torch.empty((2, n, self.A), dtype=torch.float32).pin_memory()}
            self._sq_bufs = b
        if squash is True:
            lo = hi = None
        else:
            lo = np.ascontiguousarray(np.broadcast_to(squash[0], (self.A,)), np.float32)
            hi = np.ascontiguousarray(np.broadcast_to(squash[1], (self.A,)), np.float32)
        b["obs_h"].numpy()[:] = obs
        b["obs_d"].copy_(b["obs_h"], non_blocking=True)
        s = torch.cuda.current_stream(self.device)
        N.check(self.handle.lib.dppo_act_squash_f32(
            self.handle.h, self.flat.flat.data_ptr(), b["obs_d"].data_ptr(), n,
            seed & (2 ** 64 - 1), self._next_act_counter(), N.ptr(lo), N.ptr(hi),
            b["out_d"][0].data_ptr(), b["out_d"][1].data_ptr(), s.cuda_stream),
            "dppo_act_squash_f32")
        b["out_h"].copy_(b["out_d"], non_blocking=True)
        s.synchronize()
        out = b["out_h"].numpy()
        return out[0].copy(), out[1].copy()

    def _start_draft(self, key: np.ndarray | None, pos: int | None):
        """Queue the draws of one more learn's permutations (or swap targets) on the draft worker
        thread, starting from (key, pos) -- or, when None, from the final state of the draft
        queued before it (the worker runs drafts in order, so it is known by then)."""
        busy = {self._slot} | {d["slot"] for d in self._drafts}
        slot = next(k for k in range(N.PERM_SLOTS) if k not in busy)
        prev = self._drafts[-1] if (key is None and self._drafts) else None
        d = {"slot": slot, "key_in": None if key is None else key.copy(), "pos_in": pos,
             "ok": False, "device": self.device_shuffle, "done": threading.Event()}
        draw = N.perm_targets_numpy if self.device_shuffle else N.perm_numpy
        # the job closes over plain values, not the learner: a queued or finished job never keeps
        # the learner (and its handle's pinned slots) alive
        device_shuffle, perm_n, epochs = self.device_shuffle, self.perm_n, self.cfg.num_epochs

        # The slot's previous upload must be done before the draws overwrite it: waited for here,
        # on the launching thread (device back-pressure), not on the draft thread -- a HIP wait
        # there slowed this thread's kernel enqueues ~2x (0.27 -> 0.55 ms per learn at C2).
        t0 = time.perf_counter()
        buf = d["buf"] = self.handle.perm_buffer(slot)
        self.host_seconds["slot_wait"] += time.perf_counter() - t0

        share = self.share

        def work():
            if prev is not None:
                if not prev["ok"]:
                    return
                d["key_in"], d["pos_in"] = prev["key_out"].copy(), prev["pos_out"]
            t1 = time.perf_counter()
            k = d["key_in"].copy()
            if device_shuffle and share is not None:
                # one draw per node: the leader draws into a shared slot, the others take it
                # when it is the draw of their own state (else draw it themselves)
                if share.leader:
                    sl, gen, d["pos_out"] = share.lead(
                        k, d["pos_in"], lambda kk, pp, view: draw(kk, pp, perm_n, epochs, view))
                    d["buf"], d["share"] = share.ptr(sl), (sl, gen)
                else:
                    r = share.follow(k, d["pos_in"])
                    if r is not None:
                        sl, gen, key_out, d["pos_out"] = r
                        k[:] = key_out
                        d["buf"], d["share"] = share.ptr(sl), (sl, gen)
                    else:
                        share.stats["own"] += 1
                        d["pos_out"] = draw(k, d["pos_in"], perm_n, epochs, buf)
            elif device_shuffle:
                d["pos_out"] = draw(k, d["pos_in"], perm_n, epochs, buf)
            else:
                # returns after the draws: the last epochs' swaps finish on the host pool while
                # the next draft's draws (chained on key_out) already run
                d["pos_out"], d["ticket"] = N.perm_numpy_async(k, d["pos_in"], perm_n, epochs,
                                                               buf)
            d["key_out"] = k
            d["t_draw"] = time.perf_counter() - t1
            d["ok"] = True

        if self._worker is None:
            self._worker = _DraftWorker()
        self._worker.submit(work, d["done"])
        self._drafts.append(d)

    @staticmethod
    def _finish(d):
        """Wait for a draft's draws and for the swaps still running on the host pool."""
        d["done"].wait()
        t = d.pop("ticket", None)
        if t is not None:
            N.perm_wait(t)

    def _drop(self, d):
        """A finished draft that will not be uploaded: give back the shared slot it holds."""
        if d.get("share") is not None and self.share is not None:
            self.share.drop(*d["share"])

    def _drain_drafts(self):
        """Wait for every queued draft (their slots are being written) and drop them."""
        while self._drafts:
            d = self._drafts.popleft()
            self._finish(d)
            self._drop(d)

    def close(self):
        """Release the handle safely: first every queued draft and the host-pool swaps still
        writing its pinned permutation slots, then the draft thread, then the device workspace
        (dppo_destroy frees the pinned slots).  Idempotent; also run when the learner is
        garbage-collected."""
        if getattr(self, "_closed", True):
            return
        self._closed = True
        try:
            self._drain_drafts()
        finally:
            if self._worker is not None:
                self._worker.stop()
                self._worker = None
            if self.share is not None:  # unregisters its slots from the handle first
                self.share.close()
                self.share = None
            self.handle.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _targets(self):
        """This learn's permutations (or, with device_shuffle, their swap targets) in a pinned
        slot; advances the global NumPy RNG exactly as num_epochs calls of
        np.random.permutation(B) would (ppo.py:254)."""
        key, pos, st = N.mt_state()
        if self._drafts:
            d = self._drafts.popleft()
            self._finish(d)
            if d["ok"]:
                self.host_seconds["draw"] += d["t_draw"]
                self._watch_draw(d["t_draw"])
            if (d["ok"] and d["device"] == self.device_shuffle and d["pos_in"] == pos
                    and np.array_equal(d["key_in"], key)):
                self._slot = d["slot"]
                self._cur_share = d.get("share")
                N.set_mt_state(st, d["key_out"], d["pos_out"])
                self.host_seconds["lookahead_hits"] += 1
                return d["buf"], d["key_out"], d["pos_out"]
            # the RNG moved between learns (or a draft failed): every later draft is chained
            # on the wrong state
            self._drop(d)
            self._drain_drafts()
        buf = self.handle.perm_buffer(self._slot)
        draw = N.perm_targets_numpy if self.device_shuffle else N.perm_numpy
        t0 = time.perf_counter()
        pos = draw(key, pos, self.perm_n, self.cfg.num_epochs, buf)
        self.host_seconds["draw"] += time.perf_counter() - t0
        N.set_mt_state(st, key, pos)
        return buf, key, pos

    # A draw is "slow" at > REPIN_FACTOR x the median of the last 8 and > REPIN_FLOOR_S.
    REPIN_FACTOR, REPIN_FLOOR_S, REPIN_EVERY_S = 2.5, 0.004, 5.0

    def _watch_draw(self, t: float):
        """Host-load guard.  The full-permutation draws (below PERM_DEVICE_MIN) run on the draft
        thread and the swap pool, pinned to one L3 domain (csrc/perm.cpp); on a shared host another
        tenant can saturate that domain -- one bench run on the box drew 6x slower for the whole
        run (13.2 ms per C3 learn instead of 2.2: host-bound at 75 M env-steps/s).  Two slow draws
        in a row queue a re-choice of the domain by load on the draft thread (the /proc/stat sample
        takes ~25 ms there, never on the launching thread), at most every REPIN_EVERY_S."""
        hist = self._draw_hist
        # (against the recent median; before there is one, against ~4x the measured healthy rate
        # of ~0.5 ns per drawn entry, so a domain that is busy from the first learn is left too).
        # The median of <= 8 floats in plain Python: the first np.median call of a process costs
        # 4-18 ms of lazy numpy set-up, and it fell on the first timed learn of bench.py -- one
        # stall that took C3's 20-learn line from 286 to 230 M env-steps/s (round 6 A/B)
        ref = (sorted(hist)[len(hist) // 2] * self.REPIN_FACTOR if len(hist) >= 4
               else 2e-9 * self.cfg.num_epochs * self.perm_n)
        slow = t > self.REPIN_FLOOR_S and t > ref
        hist.append(t)
        self._slow_draws = self._slow_draws + 1 if slow else 0
        now = time.monotonic()
        if (self._slow_draws >= 2 and not self.device_shuffle and self._worker is not None
                and now - self._last_repin > self.REPIN_EVERY_S):
            self._slow_draws = 0
            self._last_repin = now
            self.repin_requests += 1
            self._worker.submit(N.perm_repin, threading.Event())

    def learn(self, ro: DeviceRollout, lr: float, outputs: N.LearnOutputs | None = None):
        cfg = self.cfg
        B = self.perm_n
        if B % cfg.num_minibatches != 0:
            # reference: perms.reshape(E, M, B // M) raises (ppo.py:255)
            raise ValueError(f"cannot reshape array of size {B * cfg.num_epochs} into shape "
                             f"({cfg.num_epochs},{cfg.num_minibatches},{B // cfg.num_minibatches})")
        ro.check(self.T, self.N, self.D, self.A, self.continuous)
        step0 = adam_step_count(self.optimizer, self.flat)
        if self.fused:
            t0 = time.perf_counter()
            stream = torch.cuda.current_stream(self.device).cuda_stream
            if self.share is not None:
                self.share.pump()  # release the shared slots whose uploads are done
            self._cur_share = None
            pinned, key, pos = self._targets()
            t1 = time.perf_counter()
            # the next learns' draws overlap this learn's enqueue and device time
            if self.lookahead:
                if not self._drafts:
                    self._start_draft(key, pos)
                while len(self._drafts) < self.draft_depth:
                    self._start_draft(None, None)
            t2 = time.perf_counter()
            hp = hparams(cfg, lr, step0)
            fn = (self.handle.lib.dppo_learn_targets_f32 if self.device_shuffle
                  else self.handle.lib.dppo_learn_f32)
            try:
                N.check(fn(self.handle.h, ctypes.byref(ro.as_struct()),
                           self.flat.flat.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
                           ctypes.byref(hp), pinned,
                           ctypes.byref(outputs) if outputs is not None else None, stream),
                        "dppo_learn_f32")
            finally:
                # the upload from the shared slot is now enqueued (or the call failed): the slot
                # goes from held to pending, released once the upload's event has completed
                if self._cur_share is not None:
                    self.share.used(*self._cur_share)
                    self._cur_share = None
            t3 = time.perf_counter()
            hs = self.host_seconds
            hs["perms"] += t1 - t0
            hs["draft_start"] += t2 - t1
            hs["enqueue"] += t3 - t2
            hs["calls"] += 1
        else:
            self._learn_generic(ro, lr, step0)
        advance_adam_steps(self.optimizer, self.flat, cfg.num_epochs * cfg.num_minibatches)

    def trace(self) -> np.ndarray:
        """Per optimizer step {loss, loss_policy, loss_value, entropy, grad_norm} of the last
        fused learn() (synchronises)."""
        return self.handle.trace(self.cfg.num_epochs * self.cfg.num_minibatches)

    # -----------------------------------------------------------------------------------------
    def _learn_generic(self, ro: DeviceRollout, lr: float, step0: int):
        """Custom network_cls: torch autograd for the network, HIP kernels for GAE,
        normalisation and clip + Adam (reference ppo.py:224-287 step by step)."""
        cfg, lib, h = self.cfg, self.handle.lib, self.handle.h
        T, Nn = self.T, self.N
        B = T * Nn
        stream = torch.cuda.current_stream(self.device).cuda_stream
        net = self.network
        with torch.inference_mode():
            if self.continuous:
                means, log_stds, values = net.get_means_log_stds_and_values(ro.obs)
                from .continuous_ppo import JointNormal
                log_probs = JointNormal(loc=means, scale=log_stds.exp()).log_prob(ro.actions)
            else:
                logits, values = net.get_logits_and_values(ro.obs)
                log_probs = torch.distributions.Categorical(logits=logits).log_prob(
                    ro.actions.long())
            next_values = net.get_values(ro.next_obs)
        values = values.float().contiguous()
        next_values = next_values.float().contiguous()
        adv = torch.empty_like(values)
        ret = torch.empty_like(values)
        N.check(lib.dppo_gae_f32(h, ro.rewards.data_ptr(), ro.term.data_ptr(), ro.trunc.data_ptr(),
                                 values.data_ptr(), next_values.data_ptr(), adv.data_ptr(),
                                 ret.data_ptr(), cfg.gamma, cfg.gae_lambda, stream), "dppo_gae_f32")
        if cfg.advantage_norm:
            ms = torch.empty(4, dtype=torch.float32, device=self.device)
            N.check(lib.dppo_adv_stats(h, ms.data_ptr(), stream), "dppo_adv_stats")
            N.check(lib.dppo_adv_normalize_f32(adv.data_ptr(), ms.data_ptr(), B, stream),
                    "dppo_adv_normalize_f32")
        obs = ro.obs.reshape(B, *ro.obs.shape[2:])
        acts = ro.actions.reshape(B, *ro.actions.shape[2:])
        if not self.continuous:
            acts = acts.long()
        log_probs, adv, ret = log_probs.reshape(B), adv.reshape(B), ret.reshape(B)
        E, M = cfg.num_epochs, cfg.num_minibatches
        Bp = self.perm_n
        mbp = Bp // M
        perms = np.empty(E * Bp, np.int32)
        N.numpy_rng_permutations(Bp, E, perms)
        perms = perms.reshape(E, M, mbp)
        if self.global_mb:
            # this rank's members of each global minibatch (global flat index t * Ng + n)
            Ng, env0 = Nn * self.world, Nn * self.rank
            t_, n_ = np.divmod(perms.astype(np.int64), Ng)
            keep = (n_ >= env0) & (n_ < env0 + Nn)
            mb_lists = [[torch.from_numpy(t_[e, j][keep[e, j]] * Nn + n_[e, j][keep[e, j]] - env0)
                         .to(self.device) for j in range(M)] for e in range(E)]
        else:
            mb_lists = torch.from_numpy(perms.astype(np.int64)).to(self.device)
        step = step0
        for b_idx in mb_lists:
            for mb_idx in b_idx:
                self.flat.grad.zero_()
                # means over this rank's samples, weighted by their share of the global minibatch
                # (the all-reduce SUM below then yields the reference's global mean)
                share = (mb_idx.numel() / mbp) if self.global_mb else 1.0 / self.world
                if mb_idx.numel() == 0:
                    loss = sum(p.sum() for p in net.parameters()) * 0.0
                    loss.backward()
                    if self.world > 1:
                        torch.distributed.all_reduce(self.flat.grad)
                    step += 1
                    N.check(lib.dppo_clip_adam_f32(
                        self.flat.flat.data_ptr(), self.flat.grad.data_ptr(), self.m.data_ptr(),
                        self.v.data_ptr(), self.flat.total, cfg.grad_norm_clip, float(lr), 0.9,
                        0.999, cfg.adam_eps, step, None, stream), "dppo_clip_adam_f32")
                    continue
                if self.continuous:
                    from .continuous_ppo import JointNormal
                    m_, ls_, v_ = net.get_means_log_stds_and_values(obs[mb_idx])
                    dist = JointNormal(loc=m_, scale=ls_.exp())
                    new_v = v_
                else:
                    lg, new_v = net.get_logits_and_values(obs[mb_idx])
                    dist = torch.distributions.Categorical(logits=lg)
                new_lp = dist.log_prob(acts[mb_idx])
                ratio = (new_lp - log_probs[mb_idx]).exp()
                a_mb = adv[mb_idx]
                l_pi = torch.max(-a_mb * ratio,
                                 -a_mb * torch.clamp(ratio, 1.0 - cfg.ppo_clip, 1.0 + cfg.ppo_clip)).mean()
                l_v = 0.5 * torch.nn.functional.mse_loss(new_v, ret[mb_idx])
                ent = dist.entropy().mean()
                loss = l_pi + cfg.value_loss_weight * l_v + -cfg.entropy_beta * ent
                if self.world > 1:
                    loss = loss * share
                loss.backward()
                if self.world > 1:
                    torch.distributed.all_reduce(self.flat.grad)
                step += 1
                N.check(lib.dppo_clip_adam_f32(
                    self.flat.flat.data_ptr(), self.flat.grad.data_ptr(), self.m.data_ptr(),
                    self.v.data_ptr(), self.flat.total, cfg.grad_norm_clip, float(lr), 0.9, 0.999,
                    cfg.adam_eps, step, None, stream), "dppo_clip_adam_f32")
