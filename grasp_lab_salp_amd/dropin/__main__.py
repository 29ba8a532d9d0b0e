"""``python -m grasp_lab_salp_amd.dropin SCRIPT [ARGS...]`` (see the package docstring)."""
import sys

from . import run_script


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    if not argv or argv[0] in ("-h", "--help"):
        print("usage: python -m grasp_lab_salp_amd.dropin SCRIPT [ARGS...]\n"
              "Runs a reference script unchanged with robot / salp_robot_env bound to the HIP simulator.")
        return 0 if argv else 2
    run_script(argv[0], argv[1:])
    return 0


if __name__ == "__main__":
    sys.exit(main())
