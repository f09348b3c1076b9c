"""gym_pybullet_adrp_amd — MI355X-native batched quadrotor step for gym-pybullet-adrp.

The hot path (HoverAviary / MultiRaceAviary env.step: PYB physics sub-steps, force
models, Mellinger controller, collision, obs/reward/termination) runs as one fused HIP
kernel per env.step inside libadrp.so (csrc/), called through the C-ABI in
include/adrp.h.  This package holds the ctypes loader and the gymnasium/SB3-style
vectorised env classes that mirror the reference's surface.
"""
__version__ = "0.1.0"
