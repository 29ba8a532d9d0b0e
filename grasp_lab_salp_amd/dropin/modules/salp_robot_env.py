"""Import-path stand-in for the reference's ``salp_robot_env`` module
(src/salp_robot_env.py): :class:`grasp_lab_salp_amd.salp_robot_env.SalpRobotEnv`
under the reference's module name (see :mod:`grasp_lab_salp_amd.dropin`)."""
from grasp_lab_salp_amd.salp_robot_env import *          # noqa: F401,F403
from grasp_lab_salp_amd.salp_robot_env import __all__     # noqa: F401

__salp_dropin__ = True
