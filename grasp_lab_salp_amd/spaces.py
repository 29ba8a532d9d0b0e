"""``Box`` spaces: gymnasium's when it is installed, else a minimal stand-in
with the attributes SB3 and the reference read (low, high, shape, dtype,
sample, contains).  gymnasium is not part of this image."""
import numpy as np

try:  # pragma: no cover - depends on the environment
    from gymnasium import Env as GymEnv
    from gymnasium.spaces import Box
except ImportError:  # pragma: no cover
    GymEnv = object

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
            self.dtype = np.dtype(dtype)
            if shape is not None:
                low = np.full(shape, low, dtype=self.dtype)
                high = np.full(shape, high, dtype=self.dtype)
            self.low = np.asarray(low, dtype=self.dtype)
            self.high = np.asarray(high, dtype=self.dtype)
            self.shape = self.low.shape
            self._rng = np.random.default_rng(seed)

        def seed(self, seed=None):
            self._rng = np.random.default_rng(seed)
            return [seed]

        def sample(self):
            lo = np.where(np.isfinite(self.low), self.low, -1e6)
            hi = np.where(np.isfinite(self.high), self.high, 1e6)
            return self._rng.uniform(lo, hi).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low}, {self.high}, {self.shape}, {self.dtype})"

__all__ = ["Box", "GymEnv"]
