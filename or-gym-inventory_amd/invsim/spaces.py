"""Box spaces with the gymnasium.spaces.Box surface the reference uses
(``low``, ``high``, ``shape``, ``dtype``, ``sample()``, ``contains()``).

gymnasium is an optional dependency: when it is importable its ``Box`` is
used, so ``isinstance(space, gymnasium.spaces.Box)`` holds for SB3/RLlib.
"""
import numpy as np

try:  # pragma: no cover - gymnasium is absent in the build image
    from gymnasium.spaces import Box as _GymBox
except Exception:  # noqa: BLE001
    _GymBox = None


class _Box:
    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        self.dtype = np.dtype(dtype)
        if shape is None:
            shape = np.shape(low) if np.ndim(low) else np.shape(high)
        self.shape = tuple(int(s) for s in shape)
        self.low = np.broadcast_to(np.asarray(low, dtype=self.dtype), self.shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype=self.dtype), self.shape).copy()
        self.np_random = np.random.default_rng(seed)

    def seed(self, seed=None):
        self.np_random = np.random.default_rng(seed)
        return [seed]

    def sample(self):
        if np.issubdtype(self.dtype, np.integer):
            return self.np_random.integers(self.low, self.high, endpoint=True).astype(self.dtype)
        return self.np_random.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    def __eq__(self, other):
        return (isinstance(other, _Box) and self.shape == other.shape and self.dtype == other.dtype
                and np.array_equal(self.low, other.low) and np.array_equal(self.high, other.high))


def Box(low, high, shape=None, dtype=np.float32, seed=None):
    if _GymBox is not None:  # pragma: no cover
        return _GymBox(low=low, high=high, shape=shape, dtype=dtype, seed=seed)
    return _Box(low, high, shape=shape, dtype=dtype, seed=seed)


def batch_box(single, n):
    """gymnasium.vector.utils.batch_space for a Box."""
    low = np.broadcast_to(single.low, (n,) + tuple(single.shape))
    high = np.broadcast_to(single.high, (n,) + tuple(single.shape))
    return Box(low, high, shape=(n,) + tuple(single.shape), dtype=single.dtype)
