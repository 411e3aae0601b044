"""The C-ABI boundary: libgbp.so loads, exports every entry point that
include/gbp.h declares, and validates arguments before touching a device
(no compute here — the CPU container has no GPU)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from global_body_planner_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gbp.h")


def declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gbp_\w+)\s*\(", txt)) - {"gbp_terrain"})


def test_library_exports_every_declared_symbol():
    names = declared()
    assert len(names) >= 25
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (gbp_\w+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    assert sorted(L.EXPORTS) == names  # the Python binding covers the same surface


def test_exports_are_plain_c():
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    # no mangled C++ symbol leaks through the boundary except HIP's runtime glue
    assert "gbp_" not in "".join(l for l in out.splitlines() if "_Z" in l and "gbp" in l)


def test_load_version_and_status_strings():
    lib = L.load()
    assert lib.gbp_version() == 200
    assert lib.gbp_status_string(0) == b"ok"
    assert lib.gbp_status_string(-6) == b"no HIP device"
    assert lib.gbp_status_string(12345) == b"unknown status"


def test_argument_validation_without_device():
    lib = L.load()
    h = ctypes.c_void_p()
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    x = np.arange(4.0)
    z = np.zeros((4, 4))
    assert lib.gbp_terrain_create(0, 1, 4, P(x), P(x), P(z), None, None, None, 0, ctypes.byref(h)) \
        == -5  # GBP_E_SHAPE
    bad = np.array([0.0, 2.0, 1.0, 3.0])
    assert lib.gbp_terrain_create(0, 4, 4, P(bad), P(x), P(z), None, None, None, 0,
                                  ctypes.byref(h)) == -1  # non-ascending coordinates
    assert lib.gbp_terrain_create(0, 4, 4, P(x), P(x), None, None, None, None, 0,
                                  ctypes.byref(h)) == -1  # no heights
    assert lib.gbp_terrain_create(0, 4, 4, P(x), P(x), P(z), P(z), None, None, 0,
                                  ctypes.byref(h)) == -1  # partial slope layers
    assert lib.gbp_terrain_destroy(None) == -2
    assert lib.gbp_validate_pairs_dev(None, 1, None, None, None, 0, 0, None, None, None, None,
                                      None, None) == -2
    assert lib.gbp_nearest_batch_dev(-1, None, 0, None, None, None, None) == -1
    c = ctypes.c_int(7)
    rc = lib.gbp_device_count(ctypes.byref(c))
    import torch
    if not torch.cuda.is_available():
        assert rc == -6 and c.value == 0
        assert lib.gbp_terrain_create(0, 4, 4, P(x), P(x), P(z), None, None, None, 0,
                                      ctypes.byref(h)) == -6


def test_product_has_no_cpu_fallback(monkeypatch, tmp_path):
    """Without libgbp.so the engine raises instead of computing on the CPU."""
    monkeypatch.setattr(L, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(L, "_lib", None)
    with pytest.raises(FileNotFoundError):
        L.load()


def test_product_never_imports_the_oracle():
    pkg = os.path.join(ROOT, "global_body_planner_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in txt and "gbp_oracle" not in txt, f


def test_planner_library_exports_and_fails_without_device():
    """libgbp_planner.so (include/gbp_planner.h) exports the flat C entry
    gbp_plan_rrt_connect, no other unmangled symbol, and reports the engine's
    status instead of planning on the CPU when no device is present."""
    from global_body_planner_amd import planner
    out = subprocess.run(["nm", "-D", "--defined-only", planner.PLANNER_PATH], capture_output=True,
                         text=True, check=True).stdout
    c_syms = set(re.findall(r"\bT (gbp_\w+)", out))
    assert c_syms == {"gbp_plan_rrt_connect", "gbp_attempt_connect_batch",
                      "gbp_terrain_arrays_from_csv"}
    txt = open(os.path.join(ROOT, "include", "gbp_planner.h")).read()
    for name in c_syms:
        assert f"int {name}(" in txt
    # the C structs mirror the header layout: ... + max_time_opt (double) +
    # gbp_sampling (32) + fragile_eps_fm (8) + adaptive, nn_stats (4 + 4) +
    # max_halves, tree_capacity (8 + 8) + tree_v / tree_a / tree_parent / tree_g (4 x 2 x 8)
    # + stop_poll, stop_ctx (8 + 8) + the warm start: init_n, init_v, init_a,
    # init_parent (4 x 2 x 8), first_half, extend_base (8 + 8), stage_timing (4 + 4 padding)
    assert ctypes.sizeof(planner.PlanParams) == (4 * 3 + 4 + 8 * 6 + 8 * 16 + 8 + 8 + 8 + 8 + 8 +
                                                 32 + 8 + 8 + 8 + 8 + 64 + 16 + 64 + 16 + 8)
    # ... + stage_us[7], stage_halves (56 + 8)
    assert ctypes.sizeof(planner.PlanResult) == 312 + 64
    from global_body_planner_amd import engine
    assert ctypes.sizeof(engine.PlanStatus) == 216   # gbp_plan_status (static_assert in gbp_plan.hip)
    assert ctypes.sizeof(L.Sampling) == 32
    import torch
    if not torch.cuda.is_available():
        from global_body_planner_amd import terrain_data as td
        data = td.synth_rough(64)
        with pytest.raises(L.GbpError) as e:
            planner.plan_rrt_connect(data, np.zeros(8), np.zeros(8), batch=4, max_time=0.1)
        assert e.value.status == -6


def build_node_callsite(out, src="node_callsite.cpp"):
    """g++ the ROS-node call-site check against the reference's global names."""
    lib = os.path.join(ROOT, "global_body_planner_amd", "lib")
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "integration", src), "-L", lib,
                    "-lgbp_planner", "-lgbp", f"-Wl,-rpath,{lib}", "-o", str(out)], check=True)
    return str(out)


def test_node_config1_compiles(tmp_path):
    """The config-1 node twin (CSV ingest + buildRRTConnect) builds against the drop-in."""
    assert os.path.exists(build_node_callsite(tmp_path / "node_config1", src="node_config1.cpp"))


def test_node_callsite_compiles_links_and_refuses_cpu(tmp_path):
    """The call sites of global_body_planner.cpp compile unchanged against
    gbp_planner_compat.h and link against libgbp_planner.so; without a GPU the
    planner raises the engine's error instead of planning on the CPU."""
    exe = build_node_callsite(tmp_path / "node_callsite")
    import torch
    if not torch.cuda.is_available():
        r = subprocess.run([exe], capture_output=True, text=True)
        assert r.returncode != 0 and "no HIP device" in r.stderr
