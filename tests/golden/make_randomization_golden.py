"""Samples of the reference's randomisation features, for distributional parity.

Runs ONLY in the build container (imports /root/reference/src through the
stand-ins of make_golden.py).  The reference draws from NumPy's global
MT19937 and the device from Philox, so these are compared as distributions
(tests/test_randomization.py), not bit for bit.  Stored: data only.

* ``coef_*``      Robot._randomize_parameters (src/robot.py:594-628), 4000 draws
* ``ou_force``, ``ou_torque``  OUDisturbance states (src/robot.py:210-242) as the
                  robot uses them (force z / torque x, y zeroed after each
                  sample, src/robot.py:796-800, 834-838): 2000 chains x 400 steps,
                  final state
* ``act_in``, ``act_out``  SalpRobotEnv._randomize_actions (src/salp_robot_env.py:
                  176-181) of fixed float32 rescaled actions, 4000 draws each
* ``obs_in``, ``obs_out``  _randomize_observations (:183-194) of a fixed float32
                  observation with entries of both signs, 4000 draws
* ``latency``     geometry.randomize_scalar_jit(0.05, 1.0) (:294-295), 4000 draws

Usage:  python tests/golden/make_randomization_golden.py
"""
import os

import numpy as np

from make_golden import CANON, _import_reference

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "randomization.npz")


def main():
    ref_robot, ref_env = _import_reference()
    import geometry  # noqa: F401  (the reference module, importable once robot is)
    np.random.seed(12345)
    c = CANON
    nozzle = ref_robot.Nozzle(length1=c["length1"], length2=c["length2"], length3=c["length3"],
                              area=c["area"], mass=c["nozzle_mass"])
    robot = ref_robot.Robot(dry_mass=c["dry_mass"], init_length=c["init_length"], init_width=c["init_width"],
                            max_contraction=c["max_contraction"], nozzle=nozzle)
    out = {}
    n = 4000
    keys = ["cd", "dfr", "dtr", "amf", "amrf", "amt", "amrt"]
    draws = {k: [] for k in keys}
    for _ in range(n):
        robot._randomize_parameters()
        draws["cd"].append(robot.discharge_coefficient)
        draws["dfr"].append(robot.drag_force_ratio)
        draws["dtr"].append(robot.drag_torque_ratio)
        draws["amf"].append(np.diag(robot.added_mass_coefficient_force))
        draws["amrf"].append(np.diag(robot.added_mass_rate_coefficient_force))
        draws["amt"].append(np.diag(robot.added_mass_coefficient_torque))
        draws["amrt"].append(np.diag(robot.added_mass_rate_coefficient_torque))
    for k in keys:
        out["coef_" + k] = np.asarray(draws[k], np.float64)
    # OU processes exactly as Robot uses them
    chains, steps = 2000, 400
    fo, to = [], []
    for _ in range(chains):
        f = ref_robot.OUDisturbance(size=3, mu=0.0, theta=2.0, sigma=0.05, dt=0.01)
        t = ref_robot.OUDisturbance(size=3, mu=0.0, theta=2.0, sigma=0.01, dt=0.01)
        for _ in range(steps):
            fn = f.sample()
            fn[-1] = 0
            tn = t.sample()
            tn[0:2] = 0
        fo.append(f.state.copy())
        to.append(t.state.copy())
    out["ou_force"] = np.asarray(fo)
    out["ou_torque"] = np.asarray(to)
    out["ou_steps"] = np.int64(steps)
    # env-side randomisation (methods only read self: call them unbound)
    env_cls = ref_env.SalpRobotEnv
    acts = np.array([[0.03, 5.0, 0.5], [0.045, 1.5, -1.2]], np.float32)
    out["act_in"] = acts
    out["act_out"] = np.asarray([[env_cls._randomize_actions(None, a) for _ in range(n)] for a in acts],
                                np.float64)
    obs = np.array([0.8, -0.6, 0.05, -0.02, -0.3, 1.2, 0.4, -0.9, 1.1, 0.2], np.float32)
    out["obs_in"] = obs
    out["obs_out"] = np.asarray([env_cls._randomize_observations(None, obs) for _ in range(n)], np.float64)
    out["latency"] = np.asarray([geometry.randomize_scalar_jit(0.05, 1.0) for _ in range(n)], np.float64)
    np.savez_compressed(OUT, **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
