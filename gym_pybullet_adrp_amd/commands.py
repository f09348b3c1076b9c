"""High-level command actions for MultiRaceAviary.

The reference accepts, besides an ndarray of FULLSTATE targets, a list with one ``(Command, args)``
tuple per drone (envs/MultiRaceAviary.py:190-210), which each drone's MellingerControl process
dispatches to send*Cmd and then process_command_queue(args[-1]) (control/MellingerControl.py:17-61,
292-303).  Here those tuples are packed into two arrays, one command code per drone and
ADRP_CMD_ARGS float64 slots (include/adrp.h): the command's own arguments flattened in the
reference's order in slots 0..12, and the reference's ``args[-1]`` (the commander clock the
controller hands to crtpCommanderHighLevelUpdateTime) in slot 13.  The kernel side is
csrc/commander.h.
"""
import numpy as np

from .utils.enums import Command

CMD_ARGS = 14
TIME_SLOT = 13

# include/adrp.h ADRP_CMD_*
COMMAND_CODE = {Command.NONE: 0, Command.FULLSTATE: 1, Command.TAKEOFF: 2, Command.TAKEOFFYAW: 3,
                Command.TAKEOFFVEL: 4, Command.LAND: 5, Command.LANDYAW: 6, Command.LANDVEL: 7,
                Command.STOP: 8, Command.GOTO: 9, Command.NOTIFY: 10}

# (number of positional args, their flattened widths) of send*Cmd (MellingerControl.py:491-699);
# STOP / NOTIFY take none, but process_command_queue still reads args[-1]
_SIGNATURE = {
    Command.FULLSTATE: (3, 3, 3, 1, 3, 1),   # pos, vel, acc, yaw, rpy_rate, timestep
    Command.TAKEOFF: (1, 1),                 # height, duration
    Command.TAKEOFFYAW: (1, 1, 1),           # height, duration, yaw
    Command.TAKEOFFVEL: (1, 1, 1),           # height, vel, relative
    Command.LAND: (1, 1),
    Command.LANDYAW: (1, 1, 1),
    Command.LANDVEL: (1, 1, 1),
    Command.GOTO: (3, 1, 1, 1),              # pos, yaw, duration_s, relative
}


def _as_command(c):
    if isinstance(c, Command):
        return c
    if isinstance(c, str):
        try:
            return Command[c]
        except KeyError:
            return Command(c)
    raise TypeError(f"not a Command: {c!r}")


def encode_one(cmd, args):
    """One drone's (Command, args) -> (code, float64[CMD_ARGS])."""
    cmd = _as_command(cmd)
    out = np.zeros(CMD_ARGS, np.float64)
    args = list(args) if args is not None else []
    if cmd == Command.NONE:
        return 0, out
    if not args:   # process_command_queue(args[-1]) (MellingerControl.py:57)
        raise IndexError(f"{cmd}: process_command_queue reads args[-1], but args is empty")
    sig = _SIGNATURE.get(cmd)
    if sig is not None:
        if len(args) != len(sig):
            raise TypeError(f"{cmd}: expected {len(sig)} positional arguments, got {len(args)}")
        k = 0
        for a, w in zip(args, sig):
            v = np.asarray(a, np.float64).reshape(-1)
            if v.size != w:
                raise ValueError(f"{cmd}: argument of width {v.size}, expected {w}")
            out[k:k + w] = v
            k += w
    out[TIME_SLOT] = float(np.asarray(args[-1], np.float64).reshape(-1)[-1])
    return COMMAND_CODE[cmd], out


def encode_commands(actions, num_envs, num_drones):
    """Per-env lists of per-drone (Command, args) tuples -> (codes int32 [E, N], args float64 [E, N, 14]).

    With num_envs == 1 the reference's own format (a list of N tuples) is accepted as well.  A
    drone's entry may also be an array [x, y, z, yaw]: FULLSTATE (target, 0, 0, yaw, 0, t) as the
    ndarray path sends it (MultiRaceAviary.py:190-194); its t only sets the commander clock, which
    FULLSTATE never reads (every _update_setpoint sets it again), so it is left 0."""
    E, N = int(num_envs), int(num_drones)
    if E == 1 and len(actions) == N and (len(actions) == 0 or _is_drone_entry(actions[0])):
        actions = [actions]
    if len(actions) != E:
        raise ValueError(f"expected {E} per-env command lists, got {len(actions)}")
    codes = np.zeros((E, N), np.int32)
    args = np.zeros((E, N, CMD_ARGS), np.float64)
    for e, per_env in enumerate(actions):
        if len(per_env) != N:
            raise ValueError(f"env {e}: expected {N} per-drone commands, got {len(per_env)}")
        for n, item in enumerate(per_env):
            if isinstance(item, (tuple, list)) and len(item) == 2 and isinstance(item[0], (Command, str)):
                codes[e, n], args[e, n] = encode_one(*item)
            else:
                v = np.asarray(item, np.float64).reshape(-1)
                if v.size != 4:
                    raise ValueError(f"env {e} drone {n}: neither a (Command, args) tuple nor [x, y, z, yaw]")
                codes[e, n] = COMMAND_CODE[Command.FULLSTATE]
                args[e, n, 0:3] = v[0:3]
                args[e, n, 9] = v[3]
    return codes, args


def _is_drone_entry(x):
    """a (Command, args) tuple or a 4-vector (not a per-env list of those)"""
    if isinstance(x, (tuple, list)) and len(x) == 2 and isinstance(x[0], (Command, str)):
        return True
    if isinstance(x, np.ndarray) and x.ndim == 1:
        return True
    return False
