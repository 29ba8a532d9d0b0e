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
        first, *rest = decl.split(",")
        fields.append(re.findall(r"(\w+)\s*$", first.strip())[0])
        fields += [r.strip().lstrip("*").strip() for r in rest]
    return fields


@pytest.mark.parametrize("name,cls", [("SalpParams", _abi.SalpParams), ("SalpRolloutBuffers", _lib.SalpRolloutBuffers),
                                      ("SalpTraceBuffer", _lib.SalpTraceBuffer),
                                      ("SalpPolicyRollout", _lib.SalpPolicyRollout)])
def test_struct_layouts_match_header(name, cls):
    """The ctypes mirrors declare the header's fields in the header's order."""
    assert _header_struct_fields(name) == [f for f, _ in cls._fields_]


def test_abi_version(lib):
    assert lib.salp_abi_version() == _abi.ABI_VERSION
    assert f"#define SALP_ABI_VERSION {_abi.ABI_VERSION}" in open(HEADER).read()
