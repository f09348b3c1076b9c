"""Batched GPU environments (HoverAviary, MultiRaceAviary)."""
from .hover import HoverAviary  # noqa: F401
from .race import MultiRaceAviary  # noqa: F401
