"""Run a reference training script unchanged on the MI355X simulator.

``python -m grasp_lab_salp_amd.dropin train_robot.py [args...]`` runs the
script as ``__main__`` with :data:`MODULE_DIR` first on ``sys.path``, ahead of
the script's own directory.  That directory holds ``robot.py`` and
``salp_robot_env.py``, which re-export :mod:`grasp_lab_salp_amd.robot` and
:mod:`grasp_lab_salp_amd.salp_robot_env`, so the reference's
``from robot import Robot, Nozzle`` / ``from salp_robot_env import SalpRobotEnv``
(src/train_robot.py:6-7, src/train_robot_recurrent_ppo.py:23-24) resolve to the
HIP-backed classes and every other import (``tensorboard_callback``, SB3, ...)
still resolves from the script's directory.  The entries are on ``sys.path``,
not aliases in ``sys.modules``, so SubprocVecEnv's spawn / forkserver workers,
which rebuild ``sys.path`` from the parent's, import the same shims.
"""
import os

MODULE_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "modules")
SHIMMED = ("robot", "salp_robot_env")

__all__ = ["MODULE_DIR", "SHIMMED", "run_script"]


def run_script(path, argv=()):
    """Run ``path`` as ``__main__`` with the shims first on ``sys.path``.

    Mirrors ``python path argv...``: ``sys.argv`` is ``[path, *argv]`` and the
    script's directory is on ``sys.path`` (after :data:`MODULE_DIR`).  Returns
    the script's globals.
    """
    import runpy
    import sys

    path = os.path.abspath(path)
    if not os.path.isfile(path):
        raise FileNotFoundError(path)
    package_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    for mod in SHIMMED:              # a reference module imported earlier would shadow the shim
        if mod in sys.modules and not getattr(sys.modules[mod], "__salp_dropin__", False):
            del sys.modules[mod]
    front = [MODULE_DIR, os.path.dirname(path)]
    sys.path[:] = front + [p for p in sys.path if p not in front]
    if package_root not in sys.path:     # the shims import grasp_lab_salp_amd
        sys.path.append(package_root)
    sys.argv = [path, *argv]
    return runpy.run_path(path, run_name="__main__")
