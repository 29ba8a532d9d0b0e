"""The kernel fingerprint that ties bench.py's PMC numbers to the library it
runs (grasp_lab_salp_amd/_codeobj.py, DESIGN.md §5 "Provenance"): read from
libsalp.so's offload bundle on the CPU, stable for one build, and a summary
with another fingerprint is reported as stale, not as measured."""
import json
import os
import sys

import pytest

from grasp_lab_salp_amd import _codeobj

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    from grasp_lab_salp_amd import build
    return build.build()


def test_rollout_kernel_fingerprint_is_found_and_stable(lib):
    names = _codeobj.kernel_symbols(lib, "k_rollout")
    assert any("k_rolloutILb0ELb0EE" in n for n in names)
    assert any("k_rollout_pairILb1EE" in n for n in names)
    a = _codeobj.kernel_sha(lib, _codeobj.ROLLOUT_KERNEL)
    assert a and len(a) == 16 and a == _codeobj.kernel_sha(lib, _codeobj.ROLLOUT_KERNEL)
    # another instance has another fingerprint; an ambiguous fragment has none
    assert _codeobj.kernel_sha(lib, "k_rolloutILb0ELb1EE") not in (None, a)
    assert _codeobj.kernel_sha(lib, "k_rollout") is None


def test_bench_reports_pmc_only_for_the_measured_build(lib, tmp_path, monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    sha = _codeobj.kernel_sha(lib, _codeobj.ROLLOUT_KERNEL)
    prof = tmp_path / "profiles"
    prof.mkdir()
    base = {"config": {"n_envs": 64, "tick_budget": 32, "chunk": 16},
            "per_dispatch": {}, "derived": {"hbm_bytes": 1.0, "fp64_flops": 2.0}}
    json.dump({**base, "kernel_sha16": "0" * 16}, open(prof / "r9a_pmc_summary.json", "w"))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    name, summ, why = bench.pmc_profile(64, 32, 16)
    assert name is None and summ is None and "r9a_pmc_summary.json" in why
    json.dump({**base, "kernel_sha16": sha}, open(prof / "r9b_pmc_summary.json", "w"))
    name, summ, why = bench.pmc_profile(64, 32, 16)
    assert name == "r9b_pmc_summary.json" and why is None and summ["derived"]["hbm_bytes"] == 1.0


def test_layout_mask_zeroes_only_pc_relative_literals():
    """_mask_layout zeroes the literals of the s_add_u32 / s_addc_u32 pair after
    an s_getpc_b64 (addresses that move with the rest of the library) and
    nothing else, so an instruction change still changes the fingerprint."""
    import struct
    getpc = 0xBE821C00                     # s_getpc_b64 s[2:3]
    add, addc = 0x8002FF02, 0x8203FF03     # s_add_u32 s2, s2, lit ; s_addc_u32 s3, s3, lit
    other = 0xD2800000                     # some VOP3 word
    words = [other, getpc, add, 0x1234, addc, 0x5, other, add, 0x777]
    code = struct.pack("<%dI" % len(words), *words)
    masked = struct.unpack("<%dI" % len(words), _codeobj._mask_layout(code))
    # the pair after getpc is masked; an s_add_u32 literal elsewhere is not
    assert masked == (other, getpc, add, 0, addc, 0, other, add, 0x777)
    moved = list(words)
    moved[3], moved[5] = 0x9999, 0x6
    assert _codeobj._mask_layout(struct.pack("<9I", *moved)) == _codeobj._mask_layout(code)
    changed = list(words)
    changed[6] = other + 1
    assert _codeobj._mask_layout(struct.pack("<9I", *changed)) != _codeobj._mask_layout(code)
