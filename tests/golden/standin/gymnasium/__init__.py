"""Minimal local stand-in for the `gymnasium` API surface the reference env
modules touch (gymnasium is not installed and there is no network).

Only used by tests/golden/gen_goldens.py, in the build container, to import
the reference modules and record golden vectors.  Seeding follows
gymnasium.utils.seeding.np_random exactly: SeedSequence(seed) -> PCG64 ->
Generator, re-seeded only when `seed is not None`.
"""
from . import spaces, utils  # noqa: F401
from .utils import seeding


class Env:
    metadata = {"render_modes": []}
    _np_random = None

    @property
    def np_random(self):
        if self._np_random is None:
            self._np_random, _ = seeding.np_random()
        return self._np_random

    @np_random.setter
    def np_random(self, value):
        self._np_random = value

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self._np_random, _ = seeding.np_random(seed)

    def render(self, mode="human"):
        return None

    def close(self):
        pass
