"""Observation/action spaces: gymnasium.spaces.Box when gymnasium is importable, else a
minimal Box with the same attributes (low, high, shape, dtype, contains, sample)."""
import numpy as np

try:  # pragma: no cover - gymnasium is absent in this image
    from gymnasium.spaces import Box  # noqa: F401
except ImportError:
    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            if shape is not None:
                low = np.full(shape, low, dtype=self.dtype) if np.isscalar(low) else np.asarray(low)
                high = np.full(shape, high, dtype=self.dtype) if np.isscalar(high) else np.asarray(high)
            self.low = np.asarray(low, dtype=self.dtype)
            self.high = np.asarray(high, dtype=self.dtype)
            self.shape = self.low.shape

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def sample(self, rng=None):
            rng = rng or np.random.default_rng()
            lo = np.where(np.isfinite(self.low), self.low, -1.0)
            hi = np.where(np.isfinite(self.high), self.high, 1.0)
            return rng.uniform(lo, hi).astype(self.dtype)

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"
