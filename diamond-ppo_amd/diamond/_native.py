"""ctypes binding of libdppo (the gfx950 C ABI declared in include/dppo.h).

This is the product path: there is no CPU fallback.  If the shared library is missing or no
HIP device is present, the loaders raise instead of computing anything on the host.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DPPO_LIB") or os.path.join(_HERE, "libdppo.so")

DPPO_OK = 0
DPPO_EINVAL = -1
DPPO_EHIP = -2
DPPO_EUNSUPPORTED = -3
DPPO_ENOMEM = -4
DPPO_ECOMM = -5
MAX_TENSORS = 16
GAE_EXACT, GAE_AFFINE = 0, 1  # dppo_set_gae_mode
TRACE_FIELDS = 5
PERM_SLOTS = 3  # pinned permutation staging slots per handle (include/dppo.h DPPO_PERM_SLOTS)
PERM_EXT_SLOTS = 8  # external (caller-owned) staging slots per handle (DPPO_PERM_EXT_SLOTS)

EXPORTED = [
    "dppo_version", "dppo_last_error", "dppo_param_layout", "dppo_create", "dppo_destroy",
    "dppo_gae_f32", "dppo_gae_stream_probe", "dppo_set_gae_mode", "dppo_adv_stats", "dppo_adv_sums", "dppo_adv_stats_from_sums",
    "dppo_adv_normalize_f32", "dppo_old_policy_f32",
    "dppo_learn_f32", "dppo_minibatch_grad_f32", "dppo_prepare_f32", "dppo_clip_adam_f32",
    "dppo_perm_buffer", "dppo_perm_external", "dppo_perm_external_done", "dppo_get_trace", "dppo_perm_numpy", "dppo_comm_unique_id",
    "dppo_comm_init", "dppo_set_timing", "dppo_get_timing", "dppo_learn_targets_f32",
    "dppo_perm_targets_numpy", "dppo_perm_targets_numpy_par", "dppo_perm_par_stats", "dppo_perm_numpy_async", "dppo_perm_wait", "dppo_perm_stats", "dppo_perm_repin", "dppo_perm_domain", "dppo_perm_resolve", "dppo_perm_resolve_scratch", "dppo_perm_resolve_ex", "dppo_global_minibatch_lists", "dppo_act_f32", "dppo_act_squash_f32", "dppo_loopback_group",
    "dppo_status", "dppo_fanin_selftest", "dppo_actor_forward_f32",
    "dppo_peer_export", "dppo_peer_open", "dppo_peer_close", "dppo_peer_allreduce", "dppo_peer_info",
    "dppo_peer_selftest",
    "dppo_gru_param_layout", "dppo_gru_create", "dppo_gru_destroy", "dppo_gru_minibatch_grad_f32",
]
TIMING_CLASSES = ["eval", "gae", "adv_stats", "pack", "grad", "slab_reduce", "clip_adam",
                  "allreduce", "perm", "reduce_adam", "gae_probe"]


class Dims(ctypes.Structure):
    _fields_ = [("rollout_steps", ctypes.c_int32), ("num_envs", ctypes.c_int32),
                ("obs_dim", ctypes.c_int32), ("act_dim", ctypes.c_int32),
                ("continuous", ctypes.c_int32), ("hidden", ctypes.c_int32),
                ("num_epochs", ctypes.c_int32), ("num_minibatches", ctypes.c_int32),
                ("world_size", ctypes.c_int32), ("rank", ctypes.c_int32),
                ("global_minibatches", ctypes.c_int32)]


class HParams(ctypes.Structure):
    _fields_ = [("gamma", ctypes.c_float), ("gae_lambda", ctypes.c_float),
                ("ppo_clip", ctypes.c_float), ("value_loss_weight", ctypes.c_float),
                ("entropy_beta", ctypes.c_float), ("grad_norm_clip", ctypes.c_float),
                ("adam_beta1", ctypes.c_float), ("adam_beta2", ctypes.c_float),
                ("adam_eps", ctypes.c_float), ("advantage_norm", ctypes.c_int32),
                ("lr", ctypes.c_double), ("adam_step", ctypes.c_int64)]


class Layout(ctypes.Structure):
    _fields_ = [("total", ctypes.c_int64), ("n_real", ctypes.c_int64),
                ("count", ctypes.c_int32), ("pad_", ctypes.c_int32),
                ("offset", ctypes.c_int64 * MAX_TENSORS), ("numel", ctypes.c_int64 * MAX_TENSORS),
                ("rows", ctypes.c_int32 * MAX_TENSORS), ("cols", ctypes.c_int32 * MAX_TENSORS)]


class GruDims(ctypes.Structure):
    _fields_ = [("rollout_steps", ctypes.c_int32), ("num_envs", ctypes.c_int32),
                ("obs_dim", ctypes.c_int32), ("act_dim", ctypes.c_int32),
                ("hidden", ctypes.c_int32), ("gru_hidden", ctypes.c_int32)]


class GruBatch(ctypes.Structure):
    _fields_ = [("obs", ctypes.c_void_p), ("actions", ctypes.c_void_p),
                ("old_log_probs", ctypes.c_void_p), ("advantages", ctypes.c_void_p),
                ("returns", ctypes.c_void_p), ("prev_dones", ctypes.c_void_p),
                ("hx0", ctypes.c_void_p)]


class Rollout(ctypes.Structure):
    _fields_ = [("obs", ctypes.c_void_p), ("next_obs", ctypes.c_void_p),
                ("actions", ctypes.c_void_p), ("rewards", ctypes.c_void_p),
                ("term", ctypes.c_void_p), ("trunc", ctypes.c_void_p)]


class LearnOutputs(ctypes.Structure):
    _fields_ = [("log_probs", ctypes.c_void_p), ("values", ctypes.c_void_p),
                ("next_values", ctypes.c_void_p), ("advantages", ctypes.c_void_p),
                ("returns", ctypes.c_void_p)]


_lib = None


def load():
    """Load libdppo.so (raises ImportError if it was not built: run __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libdppo.so not found at {LIB_PATH}; build it with "
                          f"`make -C diamond-ppo_amd` (hipcc --offload-arch=gfx950)")
    lib = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, f32, f64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_double
    P = ctypes.POINTER
    sig = {
        "dppo_version": (ctypes.c_char_p, []),
        "dppo_last_error": (ctypes.c_char_p, []),
        "dppo_param_layout": (ctypes.c_int, [P(Dims), P(Layout)]),
        "dppo_create": (ctypes.c_int, [ctypes.c_int, P(Dims), P(vp)]),
        "dppo_destroy": (None, [vp]),
        "dppo_gae_f32": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, f32, f32, vp]),
        "dppo_adv_stats": (ctypes.c_int, [vp, vp, vp]),
        "dppo_gae_stream_probe": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "dppo_set_gae_mode": (ctypes.c_int, [vp, i32]),
        "dppo_adv_normalize_f32": (ctypes.c_int, [vp, vp, i64, vp]),
        "dppo_adv_sums": (ctypes.c_int, [vp, vp, vp]),
        "dppo_adv_stats_from_sums": (ctypes.c_int, [vp, f64, vp, vp]),
        "dppo_old_policy_f32": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, i64, vp]),
        "dppo_act_f32": (ctypes.c_int, [vp, vp, vp, i64, ctypes.c_uint64, ctypes.c_uint64, vp, vp]),
        "dppo_act_squash_f32": (ctypes.c_int, [vp, vp, vp, i64, ctypes.c_uint64, ctypes.c_uint64,
                                               vp, vp, vp, vp, vp]),
        "dppo_learn_f32": (ctypes.c_int, [vp, P(Rollout), vp, vp, vp, P(HParams), vp,
                                          P(LearnOutputs), vp]),
        "dppo_learn_targets_f32": (ctypes.c_int, [vp, P(Rollout), vp, vp, vp, P(HParams), vp,
                                                  P(LearnOutputs), vp]),
        "dppo_minibatch_grad_f32": (ctypes.c_int, [vp, vp, vp, i32, i32, P(HParams), vp, vp, vp]),
        "dppo_prepare_f32": (ctypes.c_int, [vp, P(Rollout), vp, P(HParams), P(LearnOutputs), vp]),
        "dppo_clip_adam_f32": (ctypes.c_int, [vp, vp, vp, vp, i64, f32, f64, f32, f32, f32, i64,
                                              vp, vp]),
        "dppo_perm_buffer": (ctypes.c_int, [vp, i32, P(vp)]),
        "dppo_perm_external": (ctypes.c_int, [vp, i32, vp, i64]),
        "dppo_perm_external_done": (ctypes.c_int, [vp, i32, P(i32)]),
        "dppo_get_trace": (ctypes.c_int, [vp, vp, i32]),
        "dppo_perm_numpy": (ctypes.c_int, [vp, P(i32), i64, i32, vp]),
        "dppo_perm_targets_numpy": (ctypes.c_int, [vp, P(i32), i64, i32, vp]),
        "dppo_perm_targets_numpy_par": (ctypes.c_int, [vp, P(i32), i64, i32, vp, i32, vp, vp]),
        "dppo_perm_par_stats": (ctypes.c_int, [P(i64)]),
        "dppo_perm_repin": (ctypes.c_int, [vp]),
        "dppo_perm_domain": (ctypes.c_int, [P(i64)]),
        "dppo_perm_numpy_async": (ctypes.c_int, [vp, P(i32), i64, i32, vp, P(vp)]),
        "dppo_perm_wait": (ctypes.c_int, [vp]),
        "dppo_perm_stats": (ctypes.c_int, [P(i64)]),
        "dppo_perm_resolve": (ctypes.c_int, [vp, vp, i64, i32, vp, vp]),
        "dppo_perm_resolve_scratch": (i64, [i64, i32]),
        "dppo_perm_resolve_ex": (ctypes.c_int, [vp, vp, i64, i32, vp, i64, vp]),
        "dppo_global_minibatch_lists": (ctypes.c_int, [vp, vp, vp, vp, vp]),
        "dppo_comm_unique_id": (ctypes.c_int, [vp]),
        "dppo_comm_init": (ctypes.c_int, [vp, i32, i32, vp]),
        "dppo_loopback_group": (ctypes.c_int, [P(vp), i32]),
        "dppo_peer_export": (ctypes.c_int, [vp, vp]),
        "dppo_peer_open": (ctypes.c_int, [vp, i32, i32, vp, i32]),
        "dppo_peer_close": (ctypes.c_int, [vp]),
        "dppo_peer_info": (ctypes.c_int, [vp, P(i64)]),
        "dppo_peer_allreduce": (ctypes.c_int, [vp, vp, i64, i32, vp]),
        "dppo_peer_selftest": (ctypes.c_int, [vp, vp]),
        "dppo_status": (ctypes.c_int, [vp]),
        "dppo_actor_forward_f32": (ctypes.c_int, [vp, vp, vp, i64, vp, vp]),
        "dppo_fanin_selftest": (ctypes.c_int, [vp, i32, i32, i64, vp]),
        "dppo_gru_param_layout": (ctypes.c_int, [P(GruDims), P(Layout)]),
        "dppo_gru_create": (ctypes.c_int, [ctypes.c_int, P(GruDims), P(vp)]),
        "dppo_gru_destroy": (None, [vp]),
        "dppo_gru_minibatch_grad_f32": (ctypes.c_int, [vp, vp, P(GruBatch), vp, i32, i32,
                                                       P(HParams), vp, vp]),
        "dppo_set_timing": (ctypes.c_int, [vp, i32]),
        "dppo_get_timing": (ctypes.c_int, [vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            # an older library under DPPO_LIB (A/B timing against a previous build) may lack the
            # newest entry points; the shipped library exports all of EXPORTED (test_native_cpu)
            if os.environ.get("DPPO_LIB"):
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class NativeError(RuntimeError):
    pass


def check(rc: int, what: str = ""):
    """Map libdppo status codes onto the exception types the reference raises."""
    if rc == DPPO_OK:
        return
    msg = load().dppo_last_error().decode(errors="replace")
    text = f"{what}: {msg}" if what else msg
    if rc == DPPO_EINVAL:
        raise ValueError(text)
    if rc == DPPO_EUNSUPPORTED:
        raise NotImplementedError(text)
    if rc == DPPO_ENOMEM:
        raise MemoryError(text)
    raise NativeError(f"libdppo error {rc}: {text}")


def ptr(t) -> int:
    """Raw device/host address of a torch tensor or numpy array (None -> 0)."""
    if t is None:
        return None
    if isinstance(t, np.ndarray):
        return t.ctypes.data
    return t.data_ptr()


def param_layout(dims: Dims) -> Layout:
    L = Layout()
    check(load().dppo_param_layout(ctypes.byref(dims), ctypes.byref(L)), "dppo_param_layout")
    return L


def _mt_call(fn: str, key: np.ndarray, pos: int, n: int, count: int, out) -> int:
    assert key.dtype == np.uint32 and key.size == 624 and key.flags.c_contiguous
    p = ctypes.c_int32(int(pos))
    dst = out if isinstance(out, int) else out.ctypes.data
    if not isinstance(out, int):
        assert out.dtype == np.int32 and out.size >= n * count and out.flags.c_contiguous
    check(getattr(load(), fn)(key.ctypes.data, ctypes.byref(p), int(n), int(count), dst), fn)
    return int(p.value)


def perm_numpy(key: np.ndarray, pos: int, n: int, count: int, out: np.ndarray | int) -> int:
    """NumPy-legacy-exact permutations (host C++).  ``key`` (uint32[624]) is advanced in place;
    returns the new ``pos``.  ``out`` is an int32 array of count*n or a raw host address."""
    return _mt_call("dppo_perm_numpy", key, pos, n, count, out)


def perm_numpy_async(key: np.ndarray, pos: int, n: int, count: int, out: int):
    """:func:`perm_numpy` whose swaps may still be running on the host pool when it returns:
    (new pos, ticket); ``perm_wait(ticket)`` before ``out`` is read."""
    assert key.dtype == np.uint32 and key.size == 624 and key.flags.c_contiguous
    p = ctypes.c_int32(int(pos))
    t = ctypes.c_void_p()
    check(load().dppo_perm_numpy_async(key.ctypes.data, ctypes.byref(p), int(n), int(count),
                                       out, ctypes.byref(t)), "dppo_perm_numpy_async")
    return int(p.value), t.value


def perm_wait(ticket) -> None:
    check(load().dppo_perm_wait(ticket), "dppo_perm_wait")


def perm_stats() -> dict:
    """{calls, pooled, ring}: host permutation draws so far, on the swap pool, with the ring."""
    out = (ctypes.c_int64 * 3)()
    check(load().dppo_perm_stats(out), "dppo_perm_stats")
    return {"calls": out[0], "pooled": out[1], "ring": out[2]}


def perm_targets_numpy(key: np.ndarray, pos: int, n: int, count: int,
                       out: np.ndarray | int) -> int:
    """The MT19937 half of :func:`perm_numpy`: Fisher-Yates swap targets ``out[c][i] = j_i``
    (the device resolves the swaps).  Advances ``key``/``pos`` exactly like perm_numpy."""
    return _mt_call("dppo_perm_targets_numpy", key, pos, n, count, out)


PAR_STATS = ["path", "chunks", "records", "zone_words", "replayed_words", "max_offset", "W", "Wb",
             "scan_us", "stitch_us", "assembly_us", "slowest_chunk_us", "words", "fail", "total_us",
             "jump_us", "scalar_words", "triggers", "stitch_work_us"]


def perm_targets_numpy_par(key: np.ndarray, pos: int, n: int, count: int, out: np.ndarray,
                           threads: int, chunks: int = 0, w: int = 0, w_mult: float = 0.0):
    """:func:`perm_targets_numpy` split over ``threads`` threads (csrc/permpar.cpp), identical
    results; returns (new pos, stats dict).  chunks / w / w_mult: the split and near-miss band
    (tests force small ones to exercise every stitch path)."""
    assert key.dtype == np.uint32 and key.size == 624 and key.flags.c_contiguous
    assert out.dtype == np.int32 and out.size >= n * count and out.flags.c_contiguous
    p = ctypes.c_int32(int(pos))
    opts = np.array([chunks, w, int(round(w_mult * 100))], np.int64)
    st = np.zeros(24, np.int64)
    check(load().dppo_perm_targets_numpy_par(key.ctypes.data, ctypes.byref(p), int(n), int(count),
                                             out.ctypes.data, int(threads), opts.ctypes.data,
                                             st.ctypes.data), "dppo_perm_targets_numpy_par")
    return int(p.value), {k: int(st[i]) for i, k in enumerate(PAR_STATS)}


def perm_repin() -> dict:
    """Choose the permutation pool's L3 domain again by load (csrc/perm.cpp; blocks ~25 ms)."""
    out = (ctypes.c_int64 * 4)()
    check(load().dppo_perm_repin(out), "dppo_perm_repin")
    return {"moved": bool(out[0]), "first_cpu": out[1], "busy_pct": out[2], "repins": out[3]}


def perm_domain() -> dict:
    """{first_cpu, busy_pct, repins} of the permutation pool's L3 domain (-1: not pinned)."""
    out = (ctypes.c_int64 * 3)()
    if not hasattr(load(), "dppo_perm_domain"):  # (an older A/B library)
        return {"first_cpu": -1, "busy_pct": -1, "repins": 0}
    check(load().dppo_perm_domain(out), "dppo_perm_domain")
    return {"first_cpu": out[0], "busy_pct": out[1], "repins": out[2]}


def perm_par_stats() -> dict:
    """{attempts, parallel, fallback}: large draws through dppo_perm_targets_numpy so far."""
    out = (ctypes.c_int64 * 3)()
    check(load().dppo_perm_par_stats(out), "dppo_perm_par_stats")
    return {"attempts": out[0], "parallel": out[1], "fallback": out[2]}


def mt_state(rng=None):
    """(key copy, pos, full state tuple) of the global legacy NumPy RNG (or ``rng``)."""
    st = (np.random.get_state() if rng is None else rng.get_state())
    if st[0] != "MT19937":
        raise ValueError("only the legacy MT19937 RandomState is supported")
    return np.array(st[1], dtype=np.uint32, copy=True), int(st[2]), st


def set_mt_state(st, key: np.ndarray, pos: int, rng=None):
    new = (st[0], key, pos, st[3], st[4])
    if rng is None:
        np.random.set_state(new)
    else:
        rng.set_state(new)


def numpy_rng_permutations(n: int, count: int, out, rng=None):
    """Draw ``count`` permutations of range(n) exactly as ``count`` calls of
    ``rng.permutation(n)`` would (rng = the global legacy NumPy RNG by default, reference
    ppo.py:254), leaving the RNG in the same final state."""
    key, pos, st = mt_state(rng)
    pos = perm_numpy(key, pos, n, count, out)
    set_mt_state(st, key, pos, rng)


def perm_resolve(targets_dev: int, perms_dev: int, n: int, count: int, scratch_dev: int,
                 stream: int):
    """Device Fisher-Yates resolution (dppo_perm_resolve): perms[c] = arange(n) shuffled by
    targets[c]; scratch holds 3*count*n int32."""
    check(load().dppo_perm_resolve(targets_dev, perms_dev, int(n), int(count), scratch_dev,
                                   stream), "dppo_perm_resolve")


def perm_resolve_scratch(n: int, count: int) -> int:
    """int32 scratch elements at which dppo_perm_resolve_ex runs its packed, fused form."""
    return int(load().dppo_perm_resolve_scratch(int(n), int(count)))


def perm_resolve_ex(targets_dev: int, perms_dev: int, n: int, count: int, scratch_dev: int,
                    scratch_ints: int, stream: int):
    """dppo_perm_resolve with an explicit scratch size (>= 3*count*n int32)."""
    check(load().dppo_perm_resolve_ex(targets_dev, perms_dev, int(n), int(count), scratch_dev,
                                      int(scratch_ints), stream), "dppo_perm_resolve_ex")


class Handle:
    """Owns one dppo_handle (device workspace sized for one rollout shape)."""

    def __init__(self, device_index: int, dims: Dims):
        self.lib = load()
        self.dims = dims
        h = ctypes.c_void_p()
        check(self.lib.dppo_create(int(device_index), ctypes.byref(dims), ctypes.byref(h)),
              "dppo_create")
        self.h = h
        self.layout = param_layout(dims)

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            self.lib.dppo_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def perm_buffer(self, slot: int = 0) -> int:
        """Pinned [E][B] int32 staging slot ``slot`` (0 .. PERM_SLOTS-1); waits, on the calling
        thread, for the slot's previous upload."""
        p = ctypes.c_void_p()
        check(self.lib.dppo_perm_buffer(self.h, int(slot), ctypes.byref(p)), "dppo_perm_buffer")
        return p.value

    def perm_external(self, k: int, ptr: int | None, nbytes: int = 0):
        """Register caller-owned host memory as external staging slot ``k`` (page-locked by the
        handle, uploaded from directly); ``ptr=None`` unregisters it."""
        check(self.lib.dppo_perm_external(self.h, int(k), ptr, int(nbytes)), "dppo_perm_external")

    def perm_external_done(self, k: int) -> bool:
        """True once the last upload from external slot ``k`` has completed (non-blocking)."""
        d = ctypes.c_int32()
        check(self.lib.dppo_perm_external_done(self.h, int(k), ctypes.byref(d)),
              "dppo_perm_external_done")
        return bool(d.value)

    def trace(self, rows: int) -> np.ndarray:
        out = np.zeros((rows, TRACE_FIELDS), np.float32)
        check(self.lib.dppo_get_trace(self.h, out.ctypes.data, int(rows)), "dppo_get_trace")
        return out

    def set_gae_mode(self, mode: int):
        check(self.lib.dppo_set_gae_mode(self.h, int(mode)), "dppo_set_gae_mode")

    def set_timing(self, enable: bool):
        check(self.lib.dppo_set_timing(self.h, int(bool(enable))), "dppo_set_timing")

    def timing(self) -> dict:
        """{class: (total_ms, launches)} since set_timing(True) (synchronises)."""
        ms = np.zeros(len(TIMING_CLASSES), np.float64)
        cnt = np.zeros(len(TIMING_CLASSES), np.int64)
        check(self.lib.dppo_get_timing(self.h, ms.ctypes.data, cnt.ctypes.data), "dppo_get_timing")
        return {k: (float(ms[i]), int(cnt[i])) for i, k in enumerate(TIMING_CLASSES)}

    def comm_init(self, nranks: int, rank: int, uid: bytes):
        buf = ctypes.create_string_buffer(uid, 128)
        check(self.lib.dppo_comm_init(self.h, int(nranks), int(rank), buf), "dppo_comm_init")

    # peer exchange (csrc/peer.hip): one-shot all-reduce over the ranks' mapped buffers
    def peer_export(self) -> bytes:
        buf = ctypes.create_string_buffer(64)
        check(self.lib.dppo_peer_export(self.h, buf), "dppo_peer_export")
        return buf.raw

    def peer_open(self, nranks: int, rank: int, handles: bytes, shared_device=False) -> str:
        """Map every rank's exchange buffer; returns "" or the error text (no exception: the
        ranks must agree on the outcome before any of them exchanges).  shared_device: some
        ranks run on the same GPU (DPPO_PEER_SHARED_DEVICE)."""
        buf = ctypes.create_string_buffer(bytes(handles), 64 * int(nranks))
        rc = self.lib.dppo_peer_open(self.h, int(nranks), int(rank), buf,
                                     1 if shared_device else 0)
        return "" if rc == 0 else (self.lib.dppo_last_error().decode() or f"rc {rc}")

    def peer_selftest(self, stream) -> str:
        rc = self.lib.dppo_peer_selftest(self.h, stream)
        return "" if rc == 0 else (self.lib.dppo_last_error().decode() or f"rc {rc}")

    def peer_close(self):
        check(self.lib.dppo_peer_close(self.h), "dppo_peer_close")

    def peer_info(self) -> dict:
        """{ranks, fused, memory, exchanges} of this handle's peer exchange (dppo_peer_info)."""
        out = (ctypes.c_int64 * 4)()
        check(self.lib.dppo_peer_info(self.h, out), "dppo_peer_info")
        mem = {0: "coarse-grained", 1: "fine-grained", 2: "uncached", -1: None}[out[2]]
        return {"ranks": out[0], "fused": bool(out[1]), "memory": mem, "exchanges": out[3]}

    def peer_allreduce(self, ptr: int, n: int, f64: bool, stream):
        check(self.lib.dppo_peer_allreduce(self.h, ptr, int(n), int(bool(f64)), stream),
              "dppo_peer_allreduce")


class GruHandle:
    """Owns one dppo_gru_handle (RecurrentPPO's fused minibatch-gradient workspace)."""

    def __init__(self, device_index: int, dims: GruDims):
        self.lib = load()
        self.dims = dims
        h = ctypes.c_void_p()
        check(self.lib.dppo_gru_create(int(device_index), ctypes.byref(dims), ctypes.byref(h)),
              "dppo_gru_create")
        self.h = h
        self.layout = Layout()
        check(self.lib.dppo_gru_param_layout(ctypes.byref(dims), ctypes.byref(self.layout)),
              "dppo_gru_param_layout")

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            self.lib.dppo_gru_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def loopback_group(handles) -> None:
    """Join handles (rank r = handles[r], one device) into a loopback group: their concurrent
    dppo_learn_f32 calls exchange what RCCL would carry, summed on the device (parity tests of
    the data-parallel path on one GPU)."""
    arr = (ctypes.c_void_p * len(handles))(*[h.h.value for h in handles])
    check(load().dppo_loopback_group(arr, len(handles)), "dppo_loopback_group")


def comm_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    check(load().dppo_comm_unique_id(buf), "dppo_comm_unique_id")
    return buf.raw
