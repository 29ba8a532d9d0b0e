"""The C-ABI boundary: libsalp.so builds, loads without a GPU and exports
exactly the functions include/salp.h declares (no compute calls here)."""
import ctypes
import os
import re

import pytest

from grasp_lab_salp_amd import _abi, _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "salp.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(salp_[a-z_0-9]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from grasp_lab_salp_amd import build
    build.build()
    return _lib.load()


def test_header_and_binding_agree():
    assert declared_functions() == sorted(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol(lib):
    for name in declared_functions():
        assert hasattr(lib, name), name


def test_state_layout_matches(lib):
    assert lib.salp_num_fields() == _abi.NUM_FIELDS
    names = [lib.salp_field_name(i).decode() for i in range(_abi.NUM_FIELDS)]
    assert names == list(_abi.FIELDS)
    assert lib.salp_field_name(_abi.NUM_FIELDS) is None
    hdr = open(HEADER).read()
    assert f"#define SALP_INFO_DIM {_abi.INFO_DIM}" in hdr
    assert f"#define SALP_MAX_OBSTACLES {_abi.MAX_OBSTACLES}" in hdr
    assert f"#define SALP_MATH_SELFTEST_ROWS {_abi.MATH_SELFTEST_ROWS}" in hdr


def test_default_params_match_python(lib):
    p = _abi.SalpParams()
    lib.salp_default_params(ctypes.byref(p))
    assert p.as_dict() == _abi.default_params().as_dict()


def test_create_rejects_bad_arguments_without_touching_the_gpu(lib):
    h = ctypes.c_void_p()
    p = _abi.default_params(num_obstacles=9)
    assert lib.salp_create(ctypes.byref(p), 4, 0, 0, 0, ctypes.byref(h)) == -1
    assert b"num_obstacles" in lib.salp_last_error(None)
    p = _abi.default_params()
    assert lib.salp_create(ctypes.byref(p), 0, 0, 0, 0, ctypes.byref(h)) == -1
    assert lib.salp_step(None, None, None, None, None, None, 0, None, None, None) == -1


def _header_struct_fields(name):
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    body = re.search(r"typedef struct " + name + r"\s*\{(.*?)\}\s*" + name + ";", text, flags=re.S).group(1)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        decl = re.sub(r"\[[^\]]*\]", "", decl)   # array fields: their name
        first, *rest = decl.split(",")
        fields.append(re.findall(r"(\w+)\s*$", first.strip())[0])
        fields += [r.strip().lstrip("*").strip() for r in rest]
    return fields


@pytest.mark.parametrize("name,cls", [("SalpParams", _abi.SalpParams), ("SalpRolloutBuffers", _lib.SalpRolloutBuffers),
                                      ("SalpTraceBuffer", _lib.SalpTraceBuffer),
                                      ("SalpPolicyRollout", _lib.SalpPolicyRollout),
                                      ("SalpPpoMinibatch", _lib.SalpPpoMinibatch), ("SalpPpoAdam", _lib.SalpPpoAdam)])
def test_struct_layouts_match_header(name, cls):
    """The ctypes mirrors declare the header's fields in the header's order."""
    assert _header_struct_fields(name) == [f for f, _ in cls._fields_]


def test_abi_version(lib):
    assert lib.salp_abi_version() == _abi.ABI_VERSION
    assert f"#define SALP_ABI_VERSION {_abi.ABI_VERSION}" in open(HEADER).read()


def test_policy_layout_matches_header(tmp_path):
    """salp_collect's packed policy: the SALP_POLICY_* offsets of the header
    (compiled with gcc) equal grasp_lab_salp_amd._abi.POLICY_OFFSETS, which
    ppo.pack_policy writes."""
    import subprocess
    names = ["PI_W1", "PI_B1", "PI_W2", "PI_B2", "ACT_W", "ACT_B", "LOG_STD", "VF_W1", "VF_B1", "VF_W2", "VF_B2",
             "VAL_W", "VAL_B", "SIZE"]
    src = tmp_path / "p.c"
    src.write_text('#include <stdio.h>\n#include "salp.h"\nint main(void) {\n'
                   + "".join(f'    printf("%d\\n", (int)(SALP_POLICY_{n}));\n' for n in names) + "    return 0;\n}\n")
    exe = tmp_path / "p"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    want = [_abi.POLICY_OFFSETS[n.lower()][0] for n in names[:-1]] + [_abi.POLICY_SIZE]
    assert got == want
    assert _abi.POLICY_OFFSETS["pi_w1"][1] == _abi.POLICY_HIDDEN * _abi.OBS_DIM_MAX


def test_fused_ppo_step_layout(lib):
    """salp_ppo_mlp_*: the flat gradient holds the 13 policy tensors of
    include/salp.h SalpMlpTensor back to back (torch Linear shapes)."""
    for d in (6, 10, 14):
        sizes = [64 * d, 64, 64 * 64, 64, 3 * 64, 3, 3, 64 * d, 64, 64 * 64, 64, 64, 1]
        offs = [lib.salp_ppo_mlp_offset(d, t) for t in range(14)]
        assert offs == [sum(sizes[:t]) for t in range(14)]
        assert lib.salp_ppo_mlp_num_params(d) == sum(sizes)
        assert lib.salp_ppo_mlp_workspace_doubles(32768, d) > 0
    assert _lib.N_MLP_TENSORS == len(sizes)
    assert lib.salp_ppo_mlp_num_params(15) == -1 and lib.salp_ppo_mlp_offset(10, 14) == -1
    assert lib.salp_ppo_mlp_grads(None, None) == -1


@pytest.mark.parametrize("name,cls", [("SalpParams", _abi.SalpParams), ("SalpRolloutBuffers", _lib.SalpRolloutBuffers),
                                      ("SalpTraceBuffer", _lib.SalpTraceBuffer),
                                      ("SalpPolicyRollout", _lib.SalpPolicyRollout),
                                      ("SalpPpoMinibatch", _lib.SalpPpoMinibatch), ("SalpPpoAdam", _lib.SalpPpoAdam)])
def test_struct_offsets_match_the_c_compiler(name, cls, tmp_path):
    """The ctypes mirrors' field offsets and sizes equal what gcc lays out for
    the header's structs (a field appended, widened or reordered in one place
    only would hand the library shifted pointers)."""
    import subprocess
    fields = [f for f, _ in cls._fields_]
    src = tmp_path / "o.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "salp.h"\nint main(void) {\n'
                   + f'    printf("%zu\\n", sizeof({name}));\n'
                   + "".join(f'    printf("%zu\\n", offsetof({name}, {f}));\n' for f in fields) + "    return 0;\n}\n")
    exe = tmp_path / "o"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    want = [ctypes.sizeof(cls)] + [getattr(cls, f).offset for f in fields]
    assert got == want, (name, got, want)


def test_ppo_workspace_constants_match_header():
    text = open(HEADER).read()
    assert f"#define SALP_PPO_APPLY_WORKSPACE_DOUBLES {_lib.APPLY_WORKSPACE_DOUBLES}" in text
    assert f"#define SALP_PPO_ADV_PARTIAL_DOUBLES {_lib.ADV_PARTIAL_DOUBLES}" in text
