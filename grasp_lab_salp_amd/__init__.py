"""MI355X-native batched SALP simulator (HIP/CDNA4 kernels behind a C ABI).

Public entry points (imported lazily so that the ABI description can be used
without torch or a GPU):

* :class:`grasp_lab_salp_amd.batched_env.BatchedSalpEnv` — n envs on one GPU,
  torch tensors in and out.
* :class:`grasp_lab_salp_amd.salp_robot_env.SalpRobotEnv`,
  :class:`grasp_lab_salp_amd.robot.Robot`, :class:`grasp_lab_salp_amd.robot.Nozzle`
  — drop-in replacements for the reference classes (src/salp_robot_env.py,
  src/robot.py).
* :class:`grasp_lab_salp_amd.vec_env.SalpVecEnv` — SB3 VecEnv-shaped adapter.
"""
__version__ = "0.1.0"
