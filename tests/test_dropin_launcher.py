"""``python -m grasp_lab_salp_amd.dropin``: a reference script runs with its
imports unchanged (VERDICT r5 missing #4; src/train_robot.py:6-7).

The script directory below holds decoy ``robot.py`` / ``salp_robot_env.py``
(standing in for the reference's own modules beside its scripts) and an
ordinary helper module: the launcher must bind the first two to the HIP-backed
classes, leave the helper importable, pass argv through, and keep the binding in
a spawned worker (SubprocVecEnv's start methods).  Only constructors run here:
they hold arguments and touch no device (grasp_lab_salp_amd/robot.py docstring).
"""
import json
import os
import subprocess
import sys
import textwrap

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent("""
    import json, multiprocessing as mp, sys
    from robot import Robot, Nozzle
    from salp_robot_env import SalpRobotEnv
    import helper

    def child(q):
        import robot, salp_robot_env
        q.put([robot.Robot.__module__, salp_robot_env.SalpRobotEnv.__module__])

    if __name__ == "__main__":
        nozzle = Nozzle(length1=0.05, length2=0.05, length3=0.05, area=0.00016, mass=1.0)
        robot = Robot(dry_mass=1.0, init_length=0.3, init_width=0.15, max_contraction=0.06, nozzle=nozzle)
        robot.nozzle.set_angles(angle1=0.0, angle2=0.0)
        robot.set_environment(density=1000)
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        p = ctx.Process(target=child, args=(q,))
        p.start()
        spawned = q.get(timeout=120)
        p.join(120)
        print("RESULT " + json.dumps({
            "robot": Robot.__module__, "nozzle": Nozzle.__module__, "env": SalpRobotEnv.__module__,
            "helper": helper.VALUE, "argv": sys.argv[1:], "spawned": spawned,
            "exitcode": p.exitcode,
        }))
""")


def test_dropin_runs_reference_script_unchanged(tmp_path):
    (tmp_path / "robot.py").write_text("raise ImportError('reference robot.py imported')\n")
    (tmp_path / "salp_robot_env.py").write_text("raise ImportError('reference salp_robot_env.py imported')\n")
    (tmp_path / "helper.py").write_text("VALUE = 'helper from the script directory'\n")
    script = tmp_path / "train_robot.py"
    script.write_text(SCRIPT)
    env = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
    out = subprocess.run([sys.executable, "-m", "grasp_lab_salp_amd.dropin", str(script), "--x", "1"],
                         cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("RESULT ")][-1]
    res = json.loads(line[len("RESULT "):])
    assert res["robot"] == res["nozzle"] == "grasp_lab_salp_amd.robot"
    assert res["env"] == "grasp_lab_salp_amd.salp_robot_env"
    assert res["helper"] == "helper from the script directory"
    assert res["argv"] == ["--x", "1"]
    assert res["spawned"] == ["grasp_lab_salp_amd.robot", "grasp_lab_salp_amd.salp_robot_env"]
    assert res["exitcode"] == 0


def test_dropin_usage():
    env = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
    out = subprocess.run([sys.executable, "-m", "grasp_lab_salp_amd.dropin"], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 2 and "usage" in out.stdout
