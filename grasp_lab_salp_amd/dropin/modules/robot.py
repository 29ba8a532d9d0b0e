"""Import-path stand-in for the reference's ``robot`` module (src/robot.py): the
HIP-backed classes of :mod:`grasp_lab_salp_amd.robot` under the reference's
module name (see :mod:`grasp_lab_salp_amd.dropin`)."""
from grasp_lab_salp_amd.robot import *          # noqa: F401,F403
from grasp_lab_salp_amd.robot import __all__     # noqa: F401

__salp_dropin__ = True
