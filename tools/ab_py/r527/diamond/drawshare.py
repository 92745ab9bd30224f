"""One reference-exact permutation draw per node, shared by the node's ranks.

With ``cfg.global_minibatches`` every rank needs the same E permutations of the GLOBAL batch
(``ppo.py:252-255``: ``np.random.permutation`` E times from the same NumPy state on every rank),
so the ranks of one node would each run the same draw -- at configs[4] 33.5 M Fisher-Yates
targets per learn, ~400 MB of host memory traffic per draw, eight times over on an 8-GPU node.
Here the node's first rank (the leader) draws into slots of POSIX shared memory and the other
ranks (followers) upload from those slots: every rank page-locks the slots with its handle
(``dppo_perm_external``, hipHostRegister), so each GPU's upload is still a direct DMA.

Protocol (``SLOTS`` slots; draft ``j`` of a learner -- its j-th look-ahead draw -- uses slot
``j % SLOTS``):

* leader: waits until every active follower has released the slot's current content and its own
  upload from the slot is done; draws into it; writes the slot header (draft index, a fingerprint
  of the NumPy state the draw started from, the final MT19937 key and pos); then bumps the slot's
  generation -- the release store that makes the header and data visible (x86 stores are not
  reordered with one another, and every field is written before it);
* follower: waits for the slot's generation to move past what it has released with the header's
  draft index equal to its own ``j``; takes the slot only if the fingerprint equals that of its
  OWN state (otherwise, or after ``DPPO_PERM_SHARE_TIMEOUT_S``, it draws itself: the result is
  always the draw of its own state).  A slot it took is HELD from ``follow()`` until its learn
  has enqueued the upload (``used()``: held -> pending) or the draft is dropped unused
  (``drop()``, a look-ahead miss); a pending slot is released once its upload is done
  (``dppo_perm_external_done``, polled at every learn).  Only a slot holding a draft index it has
  passed and never took (skipped: mismatch or timeout) is released on sight.

The leader holds its own drafts the same way, so it never draws over a draft of its own that is
still waiting for its learn.

Every wait is bounded.  A leader that cannot get a slot back raises (a follower that stopped
releasing is a follower that stopped learning).  Design notes: DESIGN.md §6.
"""
from __future__ import annotations

import hashlib
import os
import socket
import threading
import time

import numpy as np

SLOTS = 4
MAX_LOCAL = 16
_MAGIC = 0x53505044  # "DPPS"
_GLOBAL = 4096       # bytes: magic, slot bytes, active flags
_SLOT_HDR = 4096     # bytes per slot header
_ALIGN = 2 << 20     # slot data aligned to 2 MiB


def fingerprint(key: np.ndarray, pos: int) -> int:
    """64-bit digest of a NumPy MT19937 state (key words + pos)."""
    h = hashlib.blake2b(np.ascontiguousarray(key, np.uint32).tobytes(), digest_size=8)
    h.update(int(pos).to_bytes(8, "little", signed=True))
    return int.from_bytes(h.digest(), "little") & 0x7FFFFFFFFFFFFFFF


class NodeDrawShare:
    """The shared slots of one node (see the module docstring).  ``handle`` needs
    ``perm_external(k, ptr, nbytes)`` and ``perm_external_done(k)`` (diamond._native.Handle)."""

    def __init__(self, name: str, create: bool, local_index: int, local_world: int,
                 slot_bytes: int, handle):
        from multiprocessing import shared_memory
        if not (0 <= local_index < local_world <= MAX_LOCAL):
            raise ValueError("local rank out of range")
        self.name = name
        self.leader = local_index == 0
        self.me = local_index
        self.nloc = local_world
        self.slot_bytes = int(slot_bytes)
        self.stride = (self.slot_bytes + _ALIGN - 1) // _ALIGN * _ALIGN
        self.data0 = (_GLOBAL + SLOTS * _SLOT_HDR + _ALIGN - 1) // _ALIGN * _ALIGN
        size = self.data0 + SLOTS * self.stride
        if create:
            self.shm = shared_memory.SharedMemory(name=name, create=True, size=size)
        else:
            self.shm = shared_memory.SharedMemory(name=name, create=False)
            try:  # the creator owns the segment: an attaching process must not unlink it at exit
                from multiprocessing import resource_tracker
                resource_tracker.unregister(self.shm._name, "shared_memory")
            except Exception:
                pass
        buf = self.shm.buf
        self.g = np.ndarray((_GLOBAL // 8,), np.int64, buf, 0)
        self.hdr = [np.ndarray((_SLOT_HDR // 8,), np.int64, buf, _GLOBAL + s * _SLOT_HDR)
                    for s in range(SLOTS)]
        self.keys = [np.ndarray((624,), np.uint32, buf, _GLOBAL + s * _SLOT_HDR + 64)
                     for s in range(SLOTS)]
        # per slot: [0] generation, [1] draft index, [2] fingerprint, [3] pos out,
        # [8 .. 8+624/2) key (as uint32 view above), [400 + r] released generation of local rank r
        self.views = [np.ndarray((self.slot_bytes // 4,), np.int32, buf,
                                 self.data0 + s * self.stride) for s in range(SLOTS)]
        if create:
            self.g[:] = 0
            for h in self.hdr:
                h[:] = 0
                h[1] = -1
            self.g[1] = self.slot_bytes
            self.g[0] = _MAGIC
        elif int(self.g[0]) != _MAGIC or int(self.g[1]) != self.slot_bytes:
            raise RuntimeError(f"shared draw segment {name}: layout mismatch")
        self.handle = handle
        self._registered = []
        for s in range(SLOTS):
            handle.perm_external(s, self.ptr(s), self.slot_bytes)
            self._registered.append(s)
        self.g[16 + self.me] = 1  # active
        self.pending = []         # (slot, generation) uploads in flight
        self.held = {}            # slot -> generation: taken, upload not yet enqueued
        self._mu = threading.Lock()  # pump() runs on the launching and the draft thread
        self.j = 0                # this rank's next draft index
        self.live = 0             # the lowest draft index this rank may still take
        self.timeout = float(os.environ.get("DPPO_PERM_SHARE_TIMEOUT_S", "60"))
        self.stats = {"shared": 0, "own": 0, "mismatch": 0, "timeout": 0}

    # -- layout -----------------------------------------------------------------------------
    def ptr(self, s: int) -> int:
        return self.views[s].ctypes.data

    def _released(self, s: int, r: int) -> int:
        return int(self.hdr[s][400 + r])

    # -- both sides -------------------------------------------------------------------------
    def pump(self):
        """Release every slot whose upload by this rank is done, and (followers) every slot
        holding a draft index this rank has passed.  Called at every learn and while waiting."""
        with self._mu:
            still = []
            for s, gen in self.pending:
                if self.handle.perm_external_done(s):
                    if not self.leader:
                        self.hdr[s][400 + self.me] = gen
                else:
                    still.append((s, gen))
            self.pending = still
            if self.leader:
                return
            # under the lock: follow() marks a slot held and moves `live` past it atomically
            busy = {s for s, _ in self.pending} | set(self.held)
            for s in range(SLOTS):
                h = self.hdr[s]
                if (s not in busy and int(h[0]) > int(h[400 + self.me])
                        and 0 <= int(h[1]) < self.live):
                    h[400 + self.me] = int(h[0])

    def used(self, s: int, gen: int):
        """The learn just enqueued uploads from slot ``s`` (content ``gen``): held -> pending."""
        with self._mu:
            self.held.pop(s, None)
            self.pending.append((s, gen))

    def drop(self, s: int, gen: int):
        """A draft taken from slot ``s`` (content ``gen``) will not be uploaded (look-ahead miss,
        failed learn, shutdown): give the slot back at once."""
        with self._mu:
            if self.held.get(s) != gen:
                return
            del self.held[s]
            if not self.leader:
                self.hdr[s][400 + self.me] = max(gen, int(self.hdr[s][400 + self.me]))

    # -- leader -----------------------------------------------------------------------------
    def lead(self, key: np.ndarray, pos: int, draw) -> tuple[int, int, int]:
        """Draw this rank's next draft into its slot: ``draw(key, pos, out_view) -> pos_out``
        (key updated in place).  Returns (slot, generation, pos_out)."""
        j = self.j
        self.j += 1
        s = j % SLOTS
        h = self.hdr[s]
        gen = int(h[0])
        t0 = time.monotonic()
        while True:
            self.pump()
            with self._mu:
                own_done = s not in self.held and all(ps != s for ps, _ in self.pending)
            free = all(self._released(s, r) >= gen for r in range(1, self.nloc)
                       if int(self.g[16 + r]) == 1)
            if own_done and free:
                break
            if time.monotonic() - t0 > self.timeout:
                raise RuntimeError(f"shared draw: slot {s} not released by every rank within "
                                   f"{self.timeout:.0f} s (DPPO_PERM_SHARE_TIMEOUT_S)")
            time.sleep(50e-6)
        fp = fingerprint(key, pos)
        pos_out = draw(key, pos, self.views[s])
        self.keys[s][:] = key
        h[3] = pos_out
        h[2] = fp
        h[1] = j
        with self._mu:
            self.held[s] = gen + 1
        h[0] = gen + 1  # publish: every field above is already stored
        self.stats["shared"] += 1
        return s, gen + 1, pos_out

    # -- follower ---------------------------------------------------------------------------
    def follow(self, key: np.ndarray, pos: int):
        """The leader's draw of this rank's next draft, if it is the draw of (key, pos):
        (slot, generation, key_out, pos_out); None -> draw it yourself."""
        j = self.j
        self.j += 1
        with self._mu:
            self.live = j
        try:
            return self._follow(j, key, pos)
        finally:
            with self._mu:
                self.live = j + 1

    def _follow(self, j: int, key: np.ndarray, pos: int):
        s = j % SLOTS
        h = self.hdr[s]
        want = fingerprint(key, pos)
        t0 = time.monotonic()
        while True:
            gen = int(h[0])
            if gen > self._released(s, self.me) and int(h[1]) == j:
                fp, pos_out = int(h[2]), int(h[3])
                key_out = self.keys[s].copy()
                if int(h[0]) != gen:  # rewritten while being read: the leader moved on
                    continue
                if fp != want:
                    h[400 + self.me] = gen
                    self.stats["mismatch"] += 1
                    return None
                with self._mu:  # held until used() or drop(): pump() must not release it
                    self.held[s] = gen
                self.stats["shared"] += 1
                return s, gen, key_out, pos_out
            if int(h[1]) > j:  # the leader is past this draft: not for us
                self.stats["mismatch"] += 1
                return None
            if time.monotonic() - t0 > self.timeout:
                self.stats["timeout"] += 1
                return None
            self.pump()
            time.sleep(50e-6)

    def close(self):
        try:
            self.g[16 + self.me] = 0
            for s in range(SLOTS):  # nothing of ours may hold the leader back any more
                self.hdr[s][400 + self.me] = 1 << 62
        except Exception:
            pass
        for s in self._registered:
            try:
                self.handle.perm_external(s, None)
            except Exception:
                pass
        self._registered = []
        for v in ("views", "keys", "hdr", "g"):
            setattr(self, v, None)
        try:
            self.shm.close()
            if self.leader:
                self.shm.unlink()
        except Exception:
            pass


def setup(d, learner):
    """Collective over the process group: group the ranks by host, let each host's first rank
    create the segment and the others attach, agree on the outcome (every rank shares, or none).
    Returns a NodeDrawShare or None."""
    host = socket.gethostname()
    peers = [None] * learner.world
    d.all_gather_object(peers, (host, learner.rank))
    local = sorted(r for h, r in peers if h == host)
    me, nloc = local.index(learner.rank), len(local)
    if nloc < 2 or nloc > MAX_LOCAL:
        return None
    token = [os.urandom(6).hex() if learner.rank == 0 else None]
    d.broadcast_object_list(token, src=0)
    name = f"dppo_draw_{token[0]}_{local[0]}"
    slot_bytes = learner.cfg.num_epochs * learner.perm_n * 4
    share, err = None, ""
    if me == 0:
        try:
            share = NodeDrawShare(name, True, 0, nloc, slot_bytes, learner.handle)
        except Exception as e:  # no room in /dev/shm, registration refused, ...
            err = str(e)
    ok = learner._all_ranks(d, not err)
    if ok and me != 0:
        try:
            share = NodeDrawShare(name, False, me, nloc, slot_bytes, learner.handle)
        except Exception as e:
            err = str(e)
    if not learner._all_ranks(d, not err):
        if share is not None:
            share.close()
        return None
    return share
