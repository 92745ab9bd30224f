"""The node-shared draw (diamond/drawshare.py) across real processes, on the CPU: a leader draws
the learner's chain of look-ahead drafts (NumPy-exact Fisher-Yates swap targets, the
``dppo_perm_targets_numpy`` path of a global-minibatch learn) into shared-memory slots; a
follower with the same NumPy state takes every draft and gets bit for bit its own draw (targets,
MT19937 key and pos); a follower whose state differs never takes one, draws itself, and never
holds the leader back.  The handle is a stand-in whose uploads complete at once."""
import multiprocessing as mp
import os
import time
import uuid

import numpy as np
import pytest

from conftest import PKG  # noqa: F401  (puts diamond-ppo_amd on sys.path)

N_SAMPLES, EPOCHS, DRAFTS = 4096, 3, 9


class _Handle:
    def perm_external(self, k, ptr, nbytes=0):
        pass

    def perm_external_done(self, k):
        return True


def _run(name, create, me, nloc, seed, q, bar):
    from diamond import _native as N
    from diamond import drawshare as S
    try:
        share = S.NodeDrawShare(name, create, me, nloc, EPOCHS * N_SAMPLES * 4, _Handle())
        bar.wait(60)  # every rank attached (engine: setup()'s agreement collective)
        key, pos, _ = N.mt_state(np.random.RandomState(seed))
        taken, ok = 0, True
        for _ in range(DRAFTS):
            mine_key = key.copy()
            mine = np.empty(EPOCHS * N_SAMPLES, np.int32)
            mine_pos = N.perm_targets_numpy(mine_key, pos, N_SAMPLES, EPOCHS, mine)
            if share.leader:
                sl, gen, pos = share.lead(
                    key, pos, lambda kk, pp, view: N.perm_targets_numpy(kk, pp, N_SAMPLES,
                                                                         EPOCHS, view))
                got = share.views[sl][:EPOCHS * N_SAMPLES]
                ok &= bool(np.array_equal(got, mine)) and pos == mine_pos
                share.used(sl, gen)
            else:
                r = share.follow(key, pos)
                if r is not None:
                    sl, gen, key_out, pos_out = r
                    ok &= bool(np.array_equal(share.views[sl][:EPOCHS * N_SAMPLES], mine))
                    ok &= bool(np.array_equal(key_out, mine_key)) and pos_out == mine_pos
                    share.used(sl, gen)
                    taken += 1
                key, pos = mine_key, mine_pos
            if share.leader:
                ok &= bool(np.array_equal(key, mine_key))
            share.pump()
        stats = dict(share.stats)
        bar.wait(60)  # nobody closes (the leader unlinks) while another rank still reads
        share.close()
        q.put((me, ok, taken, stats))
    except Exception as e:  # reported to the parent
        q.put((me, False, -1, repr(e)))


def _spawn(seeds):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    bar = ctx.Barrier(len(seeds))
    name = f"dppo_test_{os.getpid()}_{uuid.uuid4().hex[:8]}"
    nloc = len(seeds)
    # the leader creates the segment before the followers attach
    lead = ctx.Process(target=_run, args=(name, True, 0, nloc, seeds[0], q, bar))
    lead.start()
    import time
    for _ in range(200):
        if os.path.exists(f"/dev/shm/{name}"):
            break
        time.sleep(0.05)
    rest = [ctx.Process(target=_run, args=(name, False, r, nloc, seeds[r], q, bar))
            for r in range(1, nloc)]
    for p in rest:
        p.start()
    out = {}
    for _ in range(nloc):
        me, ok, taken, stats = q.get(timeout=120)
        out[me] = (ok, taken, stats)
    for p in [lead] + rest:
        p.join(30)
    assert all(p.exitcode == 0 for p in [lead] + rest)
    return out


@pytest.mark.timeout(180)
def test_followers_take_the_leaders_draws_bit_exact():
    out = _spawn([11, 11, 11])
    for r, (ok, taken, stats) in out.items():
        assert ok, (r, stats)
        if r:
            assert taken == DRAFTS and stats["shared"] == DRAFTS, stats


@pytest.mark.timeout(180)
def test_a_follower_with_another_state_draws_itself_and_never_blocks_the_leader():
    os.environ["DPPO_PERM_SHARE_TIMEOUT_S"] = "20"
    try:
        out = _spawn([11, 11, 12])
    finally:
        del os.environ["DPPO_PERM_SHARE_TIMEOUT_S"]
    assert out[0][0] and out[1][0] and out[2][0]
    assert out[1][1] == DRAFTS            # the matching follower took every draft
    assert out[2][1] == 0 and out[2][2]["mismatch"] + out[2][2]["timeout"] == DRAFTS


def test_a_failing_draft_does_not_stop_the_draft_worker():
    """A draft whose job raises (e.g. the shared draw's bounded wait) leaves the worker running:
    later drafts still run and signal completion (before, the worker thread died with the
    exception and the next learn waited forever)."""
    import threading
    import warnings
    from diamond.engine import _DraftWorker
    w = _DraftWorker()
    ran = []
    d1, d2 = threading.Event(), threading.Event()

    def bad():
        raise RuntimeError("slot not released")

    with warnings.catch_warnings(record=True):
        warnings.simplefilter("always")
        w.submit(bad, d1)
        w.submit(lambda: ran.append(1), d2)
        assert d1.wait(10) and d2.wait(10) and ran == [1]
    w.stop()


class _SlowHandle(_Handle):
    """Uploads complete only when the test says so (``finish``)."""

    def __init__(self):
        self.done = {}

    def perm_external_done(self, k):
        return self.done.get(k, True)


def _race_follower(name, ready, took, upload_done, q):
    from diamond import drawshare as S
    try:
        ready.wait(30)
        h = _SlowHandle()
        share = S.NodeDrawShare(name, False, 1, 2, 64, h)
        key = np.zeros(624, np.uint32)
        r0 = share.follow(key, 0)      # takes draft 0 (slot 0): its learn has not run yet
        r1 = share.follow(key, 0)      # the look-ahead follows draft 1 meanwhile
        share.pump()                   # the next learn starts: pump() before its _targets()
        assert r0 is not None and r1 is not None, (r0, r1)
        took.set()
        time.sleep(1.0)                # the leader, two learns ahead, wants slot 0 back
        h.done[r0[0]] = False
        share.used(r0[0], r0[1])       # the learn enqueues its upload from slot 0 ...
        share.pump()
        time.sleep(0.5)
        upload_done.set()              # ... which completes only now
        h.done[r0[0]] = True
        deadline = time.monotonic() + 20
        while time.monotonic() < deadline and q.empty():
            share.pump()
            time.sleep(0.01)
        share.used(r1[0], r1[1])
        share.pump()
        q.put(("follower", 0, None))
        share.close()
    except Exception as e:
        q.put(("follower", -1, repr(e)))


@pytest.mark.timeout(120)
def test_leader_never_reuses_a_slot_whose_follower_upload_is_not_done():
    """A follower that took draft j holds its slot through its look-ahead's next follow() and
    pump() until the learn's upload from the slot has completed: the leader's draft j+SLOTS
    (same slot) must wait for that upload.  Before the fix the slot was released as soon as
    the follower moved on to draft j+1, and the leader drew over it mid-upload."""
    from diamond import drawshare as S
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    took, upload_done, ready = ctx.Event(), ctx.Event(), ctx.Event()
    name = f"dppo_race_{os.getpid()}_{uuid.uuid4().hex[:8]}"
    # the leader pre-draws drafts 0..SLOTS-1 into every slot before the follower attaches
    pre = S.NodeDrawShare(name, True, 0, 2, 64, _Handle())
    try:
        for _ in range(S.SLOTS):
            sl, gen, _ = pre.lead(np.zeros(624, np.uint32), 0, lambda kk, pp, v: pp)
            pre.used(sl, gen)
        pre.g[16 + 1] = 1  # the follower counts as active from the start
        f = ctx.Process(target=_race_follower, args=(name, ready, took, upload_done, q))
        f.start()
        ready.set()
        assert took.wait(60)
        fill = lambda kk, pp, view: pp  # noqa: E731
        sl, gen, _ = pre.lead(np.zeros(624, np.uint32), 0, fill)  # draft SLOTS -> slot 0
        early = not upload_done.is_set()
        pre.used(sl, gen)
        q.put(("leader", sl, early))
        who = {}
        for _ in range(2):
            tag, a, b = q.get(timeout=60)
            who[tag] = (a, b)
        f.join(30)
        assert f.exitcode == 0, who
        assert who["follower"][0] == 0, who
        assert who["leader"] == (0, False), "leader reused slot 0 before the follower's upload"
    finally:
        pre.close()


def _drop_follower(name, ready, took, q):
    from diamond import drawshare as S
    try:
        ready.wait(30)
        h = _SlowHandle()
        share = S.NodeDrawShare(name, False, 1, 2, 64, h)
        key = np.zeros(624, np.uint32)
        r0 = share.follow(key, 0)      # takes draft 0 (slot 0) ...
        share.pump()
        assert r0 is not None and r0[0] in share.held, (r0, share.held)
        took.set()
        time.sleep(0.5)
        share.drop(r0[0], r0[1])       # ... and drops it unused (a look-ahead miss)
        assert r0[0] not in share.held
        deadline = time.monotonic() + 20
        while time.monotonic() < deadline and q.empty():
            share.pump()
            time.sleep(0.01)
        q.put(("follower", 0, None))
        share.close()
    except Exception as e:
        q.put(("follower", -1, repr(e)))


@pytest.mark.timeout(120)
def test_a_dropped_draft_gives_its_slot_back_without_an_upload():
    """drop() (engine: a look-ahead miss or a failed learn) releases a held slot at once: the
    leader's next draft into that slot proceeds although no upload from it was ever enqueued."""
    from diamond import drawshare as S
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    took, ready = ctx.Event(), ctx.Event()
    name = f"dppo_drop_{os.getpid()}_{uuid.uuid4().hex[:8]}"
    pre = S.NodeDrawShare(name, True, 0, 2, 64, _Handle())
    try:
        for _ in range(S.SLOTS):
            sl, gen, _ = pre.lead(np.zeros(624, np.uint32), 0, lambda kk, pp, v: pp)
            pre.used(sl, gen)
        pre.g[16 + 1] = 1
        f = ctx.Process(target=_drop_follower, args=(name, ready, took, q))
        f.start()
        ready.set()
        assert took.wait(60)
        t0 = time.monotonic()
        sl, gen, _ = pre.lead(np.zeros(624, np.uint32), 0, lambda kk, pp, v: pp)
        waited = time.monotonic() - t0
        pre.used(sl, gen)
        q.put(("leader", sl, waited))
        who = {}
        for _ in range(2):
            tag, a, b = q.get(timeout=60)
            who[tag] = (a, b)
        f.join(30)
        assert f.exitcode == 0 and who["follower"][0] == 0, who
        assert who["leader"][0] == 0 and 0.3 < who["leader"][1] < 15, who  # waited for drop()
    finally:
        pre.close()
