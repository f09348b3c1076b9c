"""ctypes loader of libadrp.so (the C-ABI in include/adrp.h).

torch is imported first on purpose: libadrp.so is linked against libamdhip64.so.7 and
the dynamic loader then binds it to the HIP runtime torch already loaded, so torch's
hipStream_t handles and device pointers are valid inside libadrp.

There is no CPU fallback: if the library or a HIP device is missing, loading or
creating a handle raises.
"""
import ctypes
import os

import torch  # noqa: F401  (binds the shared HIP runtime before libadrp loads)

from .utils import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ADRP_LIB", os.path.join(HERE, "libadrp.so"))   # override: build experiments

_lib = None


class AdrpError(RuntimeError):
    pass


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise AdrpError(f"{LIB_PATH} is missing: build it with `make -C gym_pybullet_adrp_amd/csrc` "
                        "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    P, I = ctypes.c_void_p, ctypes.c_int
    lib.adrp_abi_version.restype = I
    lib.adrp_default_config.argtypes = [I, P]
    lib.adrp_default_config.restype = I
    lib.adrp_create.argtypes = [P, I, ctypes.POINTER(P)]
    lib.adrp_create.restype = I
    lib.adrp_destroy.argtypes = [P]
    lib.adrp_destroy.restype = None
    lib.adrp_last_error.argtypes = [P]
    lib.adrp_last_error.restype = ctypes.c_char_p
    lib.adrp_obs_dim.argtypes = [P]
    lib.adrp_act_dim.argtypes = [P]
    lib.adrp_reset.argtypes = [P, P, P, P]
    lib.adrp_reset.restype = I
    lib.adrp_step.argtypes = [P, P, P, P, P, P, P, P]
    lib.adrp_step.restype = I
    lib.adrp_state_layout.argtypes = [P, ctypes.POINTER(I), ctypes.POINTER(I)]
    lib.adrp_state_field.argtypes = [P, I, I]
    lib.adrp_state_field.restype = ctypes.c_char_p
    lib.adrp_get_state.argtypes = [P, P, P, P]
    lib.adrp_set_state.argtypes = [P, P, P, P]
    lib.adrp_kernel_name.argtypes = [P]
    lib.adrp_kernel_name.restype = ctypes.c_char_p
    if hasattr(lib, "adrp_handle_kernel_name"):   # (A/B runs may load an older build without it)
        lib.adrp_handle_kernel_name.argtypes = [P]
        lib.adrp_handle_kernel_name.restype = ctypes.c_char_p
    lib.adrp_step_bytes.argtypes = [P]
    lib.adrp_step_bytes.restype = ctypes.c_int64
    lib.adrp_profile_begin.argtypes = [P, I]
    lib.adrp_profile_begin.restype = I
    lib.adrp_profile_end.argtypes = [P, P, I]
    lib.adrp_profile_end.restype = I
    lib.adrp_reseed.argtypes = [P, ctypes.c_uint64, P]
    lib.adrp_reseed.restype = I
    if hasattr(lib, "adrp_set_noise"):       # (older experiment builds lack it)
        lib.adrp_set_noise.argtypes = [P, P, P]
        lib.adrp_set_noise.restype = I
    lib.adrp_set_wrappers.argtypes = [P, I, I]
    lib.adrp_set_wrappers.restype = I
    lib.adrp_enable_commands.argtypes = [P]
    lib.adrp_race_command.argtypes = [P, P, P, P]
    lib.adrp_get_command_state.argtypes = [P, P, P, P]
    lib.adrp_set_command_state.argtypes = [P, P, P, P]
    lib.adrp_set_diagnostics.argtypes = [P, I]
    lib.adrp_set_diagnostics.restype = I
    lib.adrp_diagnostic_contact_count.argtypes = [P, I]
    lib.adrp_diagnostic_contact_count.restype = I
    lib.adrp_persistent_begin.argtypes = [P] + [ctypes.POINTER(P)] * 6
    lib.adrp_persistent_begin.restype = I
    lib.adrp_persistent_step.argtypes = [P]
    lib.adrp_persistent_step.restype = I
    lib.adrp_persistent_end.argtypes = [P]
    lib.adrp_persistent_end.restype = I
    lib.adrp_race_moment_hash.argtypes = [P, P, ctypes.c_size_t]
    lib.adrp_race_moment_hash.restype = I
    lib.adrp_race_moment_log.argtypes = [P, P, P, ctypes.c_size_t, I]
    lib.adrp_race_moment_log.restype = I
    lib.adrp_race_reset_counts.argtypes = [P, P, I]
    lib.adrp_race_reset_counts.restype = I
    lib.adrp_policy_create.argtypes = [I, I, I, I, I, P, P, P, P, P, P, ctypes.POINTER(P)]
    lib.adrp_policy_create.restype = I
    lib.adrp_policy_act.argtypes = [P, P, I, I, I, P, P]
    lib.adrp_policy_act.restype = I
    lib.adrp_policy_destroy.argtypes = [P]
    lib.adrp_policy_destroy.restype = None
    # (every entry point include/adrp.h declares is bound: a library without one fails here, loudly)
    lib.adrp_policy_create2.argtypes = [I, I, I, I, I, I, P, P, P, P, P, P, ctypes.POINTER(P)]
    lib.adrp_policy_create2.restype = I
    lib.adrp_policy_set_critic.argtypes = [P] + [P] * 7
    lib.adrp_policy_set_critic.restype = I
    lib.adrp_policy_sample.argtypes = [P, P, I, I, I, ctypes.c_uint64, ctypes.c_uint32, P, P, P, P, P, P]
    lib.adrp_policy_sample.restype = I
    lib.adrp_gae.argtypes = [P, P, P, P, P, I, I, ctypes.c_double, ctypes.c_double, P, P, P]
    lib.adrp_gae.restype = I
    lib.adrp_compact_rows.argtypes = [P, P, P, I, I, I, P, P, P, P]
    lib.adrp_compact_rows.restype = I
    lib.adrp_memcpy_async.argtypes = [P, P, ctypes.c_size_t, I, P]
    lib.adrp_memcpy_async.restype = I
    lib.adrp_stream_synchronize.argtypes = [P]
    lib.adrp_stream_synchronize.restype = I
    lib.adrp_vec_bind.argtypes = [P, I, ctypes.POINTER(abi.AdrpVecIO)]
    lib.adrp_vec_bind.restype = I
    lib.adrp_vec_step.argtypes = [P, I, P]
    lib.adrp_vec_step.restype = I
    if hasattr(lib, "adrp_math_probe"):      # (A/B runs may load an older build without it)
        lib.adrp_math_probe.argtypes = [I, P, P, I, P]
        lib.adrp_math_probe.restype = I
    if lib.adrp_abi_version() != abi.ABI_VERSION:
        raise AdrpError(f"libadrp ABI {lib.adrp_abi_version()} != python mirror {abi.ABI_VERSION}")
    _lib = lib
    return lib


def default_config(task):
    cfg = abi.AdrpConfig()
    rc = load().adrp_default_config(task, ctypes.byref(cfg))
    if rc != 0:
        raise AdrpError(load().adrp_last_error(None).decode())
    return cfg


def kernel_name(cfg):
    """step-kernel instantiation this config selects (see include/adrp.h)"""
    return load().adrp_kernel_name(ctypes.byref(cfg)).decode()


if hasattr(torch._C, "_cuda_getCurrentRawStream"):
    _raw_stream = torch._C._cuda_getCurrentRawStream      # device index -> hipStream_t as an int
else:  # pragma: no cover
    def _raw_stream(index):
        return torch.cuda.current_stream(index).cuda_stream


def _p(t):
    """device pointer of a tensor (or None)"""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class Handle:
    """Owns one adrp_t: E envs x N drones resident in the HBM of one GPU."""

    def __init__(self, cfg, device):
        self.lib = load()
        if not torch.cuda.is_available():
            raise AdrpError("no HIP device visible: libadrp has no CPU fallback")
        self.device = torch.device("cuda", device)
        h = ctypes.c_void_p()
        rc = self.lib.adrp_create(ctypes.byref(cfg), device, ctypes.byref(h))
        if rc != 0:
            msg = self.lib.adrp_last_error(None).decode()
            raise (ValueError if rc == abi.ERR_INVALID else AdrpError)(f"adrp_create: {msg}")
        self.h = h
        self.cfg = cfg
        self.E, self.N = cfg.num_envs, cfg.num_drones
        self.S = cfg.pyb_freq // cfg.ctrl_freq     # sub-steps per env.step
        self.D = self.lib.adrp_obs_dim(h)
        self.A = self.lib.adrp_act_dim(h)
        nf, ni = ctypes.c_int(), ctypes.c_int()
        self.lib.adrp_state_layout(h, ctypes.byref(nf), ctypes.byref(ni))
        self.nf, self.ni = nf.value, ni.value
        self.real = torch.float64 if cfg.precision else torch.float32
        self._step = self.lib.adrp_step
        self._dev_index = self.device.index

    def close(self):
        if getattr(self, "h", None):
            self.lib.adrp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            raise AdrpError(f"{what}: {self.lib.adrp_last_error(self.h).decode()}")

    def _stream(self):
        """the caller's current HIP stream on this handle's device (a raw handle: no Stream object)"""
        return _raw_stream(self._dev_index)

    def field_names(self):
        return ([self.lib.adrp_state_field(self.h, 0, k).decode() for k in range(self.nf)],
                [self.lib.adrp_state_field(self.h, 1, k).decode() for k in range(self.ni)])

    def reset(self, obs, mask=None):
        self._check(self.lib.adrp_reset(self.h, _p(mask), _p(obs), self._stream()), "adrp_reset")

    def bind(self, obs, rew, term, trunc, tobs=None):
        """cache the device addresses of an env's persistent output buffers for step_ptr"""
        self._outs = (obs.data_ptr(), rew.data_ptr(), term.data_ptr(), trunc.data_ptr(),
                      None if tobs is None else tobs.data_ptr())

    def step_ptr(self, act_ptr):
        """adrp_step on the buffers of the last bind() (the hot call of a Python-driven loop: one
        ctypes call, no tensor introspection)"""
        rc = self._step(self.h, act_ptr, *self._outs, _raw_stream(self._dev_index))
        if rc != 0:
            self._check(rc, "adrp_step")

    def step(self, act, obs, rew, term, trunc, tobs=None):
        """act None: command mode, the setpoints the last command() left"""
        rc = self._step(self.h, None if act is None else act.data_ptr(), obs.data_ptr(), rew.data_ptr(), term.data_ptr(),
                        trunc.data_ptr(), None if tobs is None else tobs.data_ptr(), _raw_stream(self._dev_index))
        if rc != 0:
            self._check(rc, "adrp_step")

    def get_state(self):
        f = torch.empty((self.nf, self.E * self.N), dtype=self.real, device=self.device)
        i = torch.empty((self.ni, self.E * self.N), dtype=torch.int32, device=self.device)
        self._check(self.lib.adrp_get_state(self.h, _p(f), _p(i), self._stream()), "adrp_get_state")
        return f, i

    def set_state(self, f, i):
        f = f.to(device=self.device, dtype=self.real).contiguous()
        i = i.to(device=self.device, dtype=torch.int32).contiguous()
        assert f.shape == (self.nf, self.E * self.N) and i.shape == (self.ni, self.E * self.N)
        self._check(self.lib.adrp_set_state(self.h, _p(f), _p(i), self._stream()), "adrp_set_state")

    def step_bytes(self):
        return self.lib.adrp_step_bytes(self.h)

    def kernel_name(self):
        """the step-kernel instantiation this handle launches now"""
        if not hasattr(self.lib, "adrp_handle_kernel_name"):
            return kernel_name(self.cfg)
        return self.lib.adrp_handle_kernel_name(self.h).decode()

    # ---- high-level command mode (include/adrp.h adrp_enable_commands) ----
    CMD_NF, CMD_NI, CMD_ARGS = 63, 3, 14

    def enable_commands(self):
        self._check(self.lib.adrp_enable_commands(self.h), "adrp_enable_commands")
        self.commands = True

    def command(self, cmd, args):
        """cmd int32 [E, N] (ADRP_CMD_*), args float64 [E, N, 14], device tensors"""
        cmd = cmd.to(device=self.device, dtype=torch.int32).contiguous()
        args = args.to(device=self.device, dtype=torch.float64).contiguous()
        assert cmd.numel() == self.E * self.N and args.numel() == self.E * self.N * self.CMD_ARGS
        self._check(self.lib.adrp_race_command(self.h, _p(cmd), _p(args), self._stream()), "adrp_race_command")

    def get_command_state(self):
        f = torch.empty((self.CMD_NF, self.E * self.N), dtype=torch.float32, device=self.device)
        i = torch.empty((self.CMD_NI, self.E * self.N), dtype=torch.int32, device=self.device)
        self._check(self.lib.adrp_get_command_state(self.h, _p(f), _p(i), self._stream()), "adrp_get_command_state")
        return f, i

    def set_command_state(self, f, i):
        f = f.to(device=self.device, dtype=torch.float32).contiguous()
        i = i.to(device=self.device, dtype=torch.int32).contiguous()
        assert f.shape == (self.CMD_NF, self.E * self.N) and i.shape == (self.CMD_NI, self.E * self.N)
        self._check(self.lib.adrp_set_command_state(self.h, _p(f), _p(i), self._stream()), "adrp_set_command_state")

    def reseed(self, seed):
        """re-key the random streams as a handle created with `seed` (episode counters zeroed)"""
        seed = int(seed) & (2 ** 64 - 1)
        self._check(self.lib.adrp_reseed(self.h, seed, self._stream()), "adrp_reseed")
        self.cfg.seed = seed

    def set_noise(self, act_noise, force):
        """parity mode (include/adrp.h adrp_set_noise): float64 device tensors [E*N, S, 4] / [E*N, S, 3]
        (kept referenced here: the library keeps the pointers), or None, None"""
        self._noise = (act_noise, force)
        self._check(self.lib.adrp_set_noise(self.h, _p(act_noise), _p(force)), "adrp_set_noise")

    def set_wrappers(self, reward_wrapper, obs_wrapper):
        self._check(self.lib.adrp_set_wrappers(self.h, int(bool(reward_wrapper)), int(obs_wrapper)), "adrp_set_wrappers")
        self.cfg.track.reward_wrapper = int(bool(reward_wrapper))
        self.cfg.track.obs_wrapper = int(obs_wrapper)

    def set_diagnostics(self, enable=True):
        """True / 1: contact counter, race moment hash; 2: also the race firmware moment log (the
        step then runs the one-lane race kernel)"""
        level = int(enable) if not isinstance(enable, bool) else (1 if enable else 0)
        self._check(self.lib.adrp_set_diagnostics(self.h, level), "adrp_set_diagnostics")

    def contact_count(self, reset=True):
        """env-steps that touched the plane contact model since the last reset (diagnostics on)"""
        return self.lib.adrp_diagnostic_contact_count(self.h, 1 if reset else 0)

    def moment_hash(self):
        """race, diagnostics on: [E*N] uint32 per drone slot, the hash of the int16 (roll, pitch, yaw)
        moments of every firmware call of the last env.step (the parity tests compare it with the CPU
        restatement's)"""
        import numpy as np
        out = np.zeros(self.E * self.N, np.uint32)
        self._check(self.lib.adrp_race_moment_hash(self.h, out.ctypes.data_as(ctypes.c_void_p), out.size),
                    "adrp_race_moment_hash")
        return out

    def moment_log(self):
        """race, diagnostics level 2: (moments int16 [E*N][S][3], calls int32 [E*N]) of the last
        env.step, the int16 (roll, pitch, yaw) of every firmware call in call order"""
        import numpy as np
        n = self.E * self.N
        out = np.zeros((n, self.S, 3), np.int16)
        cnt = np.zeros(n, np.int32)
        self._check(self.lib.adrp_race_moment_log(self.h, out.ctypes.data_as(ctypes.c_void_p),
                                                  cnt.ctypes.data_as(ctypes.c_void_p), n, self.S), "adrp_race_moment_log")
        return out, cnt

    def reset_counts(self, reset=True):
        """race, diagnostics on: (auto-resets copied from a next-reset image, auto-resets computed
        inline) by the four-lane kernel since the last read"""
        import numpy as np
        out = np.zeros(2, np.int32)
        self._check(self.lib.adrp_race_reset_counts(self.h, out.ctypes.data_as(ctypes.c_void_p), 1 if reset else 0),
                    "adrp_race_reset_counts")
        return int(out[0]), int(out[1])

    def profile_begin(self, n):
        self._check(self.lib.adrp_profile_begin(self.h, n), "adrp_profile_begin")

    def profile_end(self, n):
        import numpy as np
        out = np.zeros(n, np.float32)
        got = self.lib.adrp_profile_end(self.h, out.ctypes.data_as(ctypes.c_void_p), n)
        if got < 0:
            self._check(got, "adrp_profile_end")
        return out[:got]
