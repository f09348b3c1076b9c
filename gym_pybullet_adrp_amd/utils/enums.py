"""Enums with the reference's names and values (gym_pybullet_adrp/utils/enums.py:8-87)."""
from enum import Enum


class DroneModel(Enum):
    CF2X = "cf2x_IROS"   # cf2x_IROS.urdf constants (enums.py:12)
    CF2P = "cf2p"
    RACE = "racer"


class Physics(Enum):
    PYB = "pyb"
    DYN = "dyn"
    PYB_GND = "pyb_gnd"
    PYB_DRAG = "pyb_drag"
    PYB_DW = "pyb_dw"
    PYB_GND_DRAG_DW = "pyb_gnd_drag_dw"


class ActionType(Enum):
    MEL = "mel"
    RPM = "rpm"
    PID = "pid"
    VEL = "vel"
    ONE_D_RPM = "one_d_rpm"
    ONE_D_PID = "one_d_pid"


class ObservationType(Enum):
    KIN = "kin"
    RGB = "rgb"


class Command(Enum):
    FULLSTATE = "fst"
    TAKEOFF = "tko"
    TAKEOFFYAW = "toy"
    TAKEOFFVEL = "tov"
    LAND = "lnd"
    LANDYAW = "ldy"
    LANDVEL = "ldv"
    STOP = "stp"
    GOTO = "gto"
    NOTIFY = "ntf"
    NONE = "non"


class RaceMode(Enum):
    COMPARE = 0
    COMPETE = 1


# enum -> C-ABI codes (include/adrp.h)
PHYSICS_CODE = {Physics.PYB: 0, Physics.DYN: 1, Physics.PYB_GND: 2, Physics.PYB_DRAG: 3,
                Physics.PYB_DW: 4, Physics.PYB_GND_DRAG_DW: 5}
