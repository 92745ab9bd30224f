"""Restatement of NumPy's legacy ``RandomState.permutation(n)``.  TEST INFRASTRUCTURE ONLY.

The reference draws its minibatch order from the legacy global NumPy RNG
(``diamond/ppo.py:120-122`` seeds it, ``ppo.py:254`` calls ``np.random.permutation``).
NumPy is a third-party dependency (reference ``pyproject.toml:40`` pins ``numpy>=2.0.0``;
this image ships 2.2.6).  Its published algorithm, restated here:

* ``RandomState.permutation(int n)`` = ``arr = arange(n); shuffle(arr)``   (numpy/random/mtrand.pyx)
* ``shuffle`` on a 1-D array = ``_shuffle_raw``: for i = n-1 down to 1:
  ``j = random_interval(bitgen, i)``; swap arr[i], arr[j]                   (mtrand.pyx)
* ``random_interval(max)``: mask = smallest 2^k - 1 >= max; for max <= 0xffffffff draw
  ``next_uint32 & mask`` until <= max                  (numpy/random/src/distributions/distributions.c)
* ``next_uint32`` of the legacy MT19937 bit generator = classic ``genrand_int32``
  (twist of 624 words + tempering)                           (numpy/random/src/mt19937/mt19937.c)

Pinned against NumPy itself and against ``tests/golden/perm_seed42.npz`` (captured from the
reference environment: first 8 of ``permutation(1024)`` after ``seed(42)`` are
``[525 357 444 31 618 587 447 734]``).  Pure Python: small n only.
"""
from __future__ import annotations

import numpy as np

N_, M_ = 624, 397
MATRIX_A, UPPER, LOWER = 0x9908B0DF, 0x80000000, 0x7FFFFFFF


class MT19937:
    def __init__(self, key, pos):
        self.mt = [int(k) & 0xFFFFFFFF for k in key]
        self.pos = int(pos)

    @classmethod
    def from_numpy_state(cls, state):
        name, key, pos = state[0], state[1], state[2]
        assert name == "MT19937"
        return cls(key, pos)

    def _twist(self):
        mt = self.mt
        for i in range(N_):
            y = (mt[i] & UPPER) | (mt[(i + 1) % N_] & LOWER)
            mt[i] = mt[(i + M_) % N_] ^ (y >> 1) ^ (MATRIX_A if y & 1 else 0)
        self.pos = 0

    def next32(self):
        if self.pos >= N_:
            self._twist()
        y = self.mt[self.pos]
        self.pos += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF

    def random_interval(self, mx):
        if mx == 0:
            return 0
        mask = mx
        for s in (1, 2, 4, 8, 16, 32):
            mask |= mask >> s
        assert mx <= 0xFFFFFFFF
        while True:
            v = self.next32() & mask
            if v <= mx:
                return v

    def permutation(self, n):
        arr = list(range(n))
        for i in range(n - 1, 0, -1):
            j = self.random_interval(i)
            arr[i], arr[j] = arr[j], arr[i]
        return np.array(arr, dtype=np.int64)

    def numpy_state(self, template):
        return (template[0], np.array(self.mt, dtype=np.uint32), self.pos) + tuple(template[3:])
