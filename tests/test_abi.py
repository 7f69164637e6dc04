"""CPU: the C-ABI library loads and exports every symbol include/invsim.h
declares, and the ctypes mirrors of the spec structs match the C layout.
No compute calls (no GPU here)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "invsim.h")


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(invsim_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from invsim import _capi
    lib = _capi.load_library()
    declared = _declared_functions()
    assert len(declared) >= 18
    missing = [f for f in declared if not hasattr(lib, f)]
    assert not missing, missing
    assert sorted(_capi.EXPORTS) == declared
    assert lib.invsim_abi_version() == 4


def test_library_is_gfx950_code_object():
    """The embedded HIP fat binary carries a gfx950 code object (and no other target)."""
    from invsim import _capi
    blob = open(_capi.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx90a", b"--gfx942", b"--gfx1100"):
        assert other not in blob


def test_spec_struct_layout_matches_header(tmp_path):
    """Compile a probe against include/invsim.h and compare sizeof/offsetof with ctypes."""
    from invsim import _capi
    probe = tmp_path / "probe.c"
    fields = {
        "invsim_newsvendor_spec": (_capi.NewsvendorSpec, [f for f, _ in _capi.NewsvendorSpec._fields_]),
        "invsim_invmgmt_spec": (_capi.InvMgmtSpec, [f for f, _ in _capi.InvMgmtSpec._fields_]),
        "invsim_netinvmgmt_spec": (_capi.NetInvMgmtSpec, [f for f, _ in _capi.NetInvMgmtSpec._fields_]),
        "invsim_policy": (_capi.PolicySpec, [f for f, _ in _capi.PolicySpec._fields_]),
    }
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for cname, (_, names) in fields.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for n in names:
            lines.append(f'printf("{cname} {n} %zu\\n", offsetof({cname}, {n}));')
    lines.append("return 0;}")
    probe.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(probe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    got = {}
    for ln in out:
        if ln:
            a, b, c = ln.split()
            got[(a, b)] = int(c)
    for cname, (cls, names) in fields.items():
        assert got[(cname, "size")] == C.sizeof(cls), cname
        for n in names:
            assert got[(cname, n)] == getattr(cls, n).offset, (cname, n)


def test_create_without_gpu_fails_cleanly():
    """No GPU in this container: create must fail with an error code, not crash."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from invsim import _capi
    lib = _capi.load_library()
    spec = _capi.NewsvendorSpec(5, 40, 4000.0, 2000.0, 100.0, 5.0, 10.0, 200.0, 1.0)
    h = C.c_void_p()
    rc = lib.invsim_create_newsvendor(C.byref(spec), 16, 0, 0, C.byref(h))
    assert rc != 0 and not h.value
    assert lib.invsim_last_error(None)


def test_validation_errors_mirror_reference_asserts():
    """Spec validation happens before any device call (inventory_management.py:144-167)."""
    import numpy as np
    from invsim import _capi
    lib = _capi.load_library()
    I0 = np.array([100, -1, 200], np.int64)
    f4 = np.ones(4, np.float32)
    c = np.array([100, 200, 230], np.int64)
    L = np.array([1, 5, 10], np.int64)
    spec = _capi.InvMgmtSpec(4, 30, 1, 1, 20.0, 0.97, I0.ctypes.data, f4.ctypes.data, f4.ctypes.data,
                             f4.ctypes.data, f4.ctypes.data, c.ctypes.data, L.ctypes.data, None)
    h = C.c_void_p()
    assert lib.invsim_create_invmgmt(C.byref(spec), 8, 0, 0, C.byref(h)) == -22
    assert b"Initial inventory cannot be negative" in lib.invsim_last_error(None)
    I0[1] = 150
    spec.alpha = 1.5
    assert lib.invsim_create_invmgmt(C.byref(spec), 8, 0, 0, C.byref(h)) == -22
    assert b"alpha" in lib.invsim_last_error(None)
    spec.alpha = 0.97
    # numpy's own argument checks for the demand samplers (inventory_management.py:173-182)
    for dist, kw, msg in [(2, dict(dist_n=10, dist_p=1.5), b"p > 1"), (2, dict(dist_n=-1, dist_p=0.5), b"n < 0"),
                          (3, dict(dist_low=5, dist_high=4), b"low >= high"), (4, dict(dist_p=0.0), b"p <= 0"),
                          (7, {}, b"dist must be one of")]:
        spec.dist = dist
        for k, v in kw.items():
            setattr(spec, k, v)
        assert lib.invsim_create_invmgmt(C.byref(spec), 8, 0, 0, C.byref(h)) == -22
        assert msg in lib.invsim_last_error(None)


def test_python_env_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from invsim import InvManagementBacklogEnv
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        InvManagementBacklogEnv(4)


def test_launch_switches_are_read_only_at_handle_creation():
    """the INVSIM_* A/B switches are read from the
    environment once, when a handle is created (capi.hip read_knobs into
    Common::kn), never on a launch path: `getenv` appears only in capi.hip's
    env_flag / read_knobs, and every switch the launchers use is a Knobs
    field."""
    import re
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "or-gym-inventory_amd", "csrc")
    hits = {}
    for name in sorted(os.listdir(csrc)):
        if name.endswith((".hip", ".hpp")):
            src = open(os.path.join(csrc, name)).read()
            for m in re.finditer(r"\bgetenv\s*\(", src):
                hits.setdefault(name, []).append(src.count("\n", 0, m.start()) + 1)
    assert list(hits) == ["capi.hip"], hits
    capi = open(os.path.join(csrc, "capi.hip")).read()
    a = capi.index("bool env_flag(")
    b = capi.index("void bind_common(")
    lines = [capi.count("\n", 0, i) + 1 for i in (a, b)]
    assert all(lines[0] <= ln < lines[1] for ln in hits["capi.hip"]), (hits, lines)
    assert "c.kn = read_knobs();" in capi[b:b + 200]
    kern = open(os.path.join(csrc, "kernels.hpp")).read()
    fields = set(re.findall(r"^\s+(?:bool|int8_t|int64_t) (\w+) = ", kern[kern.index("struct Knobs"):kern.index("struct Common")], re.M))
    reads = set(re.findall(r'"INVSIM_(\w+)"', capi[a:b]))
    assert {f.upper() for f in fields} == reads, (fields, reads)
