"""CPU checks of the drop-in boundary: the HIP library builds, loads and exports
exactly the C ABI declared in include/livo.h; struct layouts agree between C
and the Python binding; errors come back as codes (no GPU needed, no compute).
"""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "livo.h")


def _declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(livo_\w+)\s*\(", txt, flags=re.M)))


def test_header_declares_abi():
    names = _declared()
    for n in ("livo_ctx_create", "livo_map_build", "livo_knn", "livo_scan_upload", "livo_h_share",
              "livo_iekf_update", "livo_iekf_update_batch"):
        assert n in names


def test_library_exports_every_declared_symbol(built):
    import livo_amd
    lib = C.CDLL(livo_amd.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    # and the Python binding covers the whole ABI
    assert set(_declared()) == set(livo_amd.SIGNATURES)
    out = subprocess.run(["nm", "-D", "--defined-only", livo_amd.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (livo_\w+)", out))
    assert exported == set(_declared())


def test_hip_code_object_is_gfx950(built):
    import livo_amd
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", livo_amd.LIB_PATH], capture_output=True,
                         text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(livo_amd.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_version_and_errors(built):
    import livo_amd
    L = livo_amd.load()
    hdr = open(HEADER).read()
    ver = int(re.search(r"#define LIVO_ABI_VERSION (\d+)", hdr).group(1))
    assert L.livo_abi_version() == ver
    for code in (0, -1, -2, -3, -4, -5, -6, -77):
        assert isinstance(L.livo_error_string(code), bytes)
    p = livo_amd.default_params()
    # reference defaults (laser_mapping.cpp:968-983, :518, :530, :552)
    assert p.laser_point_cov == 0.001 and p.max_iterations == 4
    assert abs(p.plane_threshold - 0.1) < 1e-7 and p.max_nn_sqdist == 5.0 and p.max_residual == 2.0
    assert list(p.R_LI) == [1, 0, 0, 0, 1, 0, 0, 0, 1] and list(p.t_LI) == [0, 0, 0]


def test_invalid_arguments_return_codes(built):
    import livo_amd
    L = livo_amd.load()
    assert L.livo_ctx_create(0, None, None) == -1  # LIVO_E_INVALID
    assert L.livo_ctx_destroy(None) == -1
    assert L.livo_params_default(None) == -1
    bad = livo_amd.default_params()
    bad.max_iterations = 99
    h = C.c_void_p()
    assert L.livo_ctx_create(0, C.byref(bad), C.byref(h)) == -1
    assert L.livo_map_build(None, None, 0, 0) == -1
    assert L.livo_sync(None) == -1
    t = C.c_int32(-1)
    assert L.livo_iekf_update_batch_submit(None, 0, None, None, None, C.byref(t)) == -1
    assert L.livo_iekf_update_batch_wait(None, 0, None, None) == -1
    assert L.livo_error_string(-8).startswith(b"batches in flight")  # LIVO_E_BUSY


def test_knn_calibration_fixture():
    """tests/golden/knn_calibration.json (tools/calibrate_knn.py): a timing calibration
    of the oracle's k-NN against BASELINE.md's survey timing of the reference
    ikd_Tree.cpp, one row per survey size; bench.py carries the 1M ratio."""
    import json
    cal = json.load(open(os.path.join(ROOT, "tests", "golden", "knn_calibration.json")))
    assert cal["pins_parity"] is False
    sizes = {r["map_points"]: r for r in cal["rows"]}
    assert set(sizes) == {100_000, 1_000_000, 10_000_000}
    for r in cal["rows"]:
        lo, hi = r["reference_us_per_query"]
        ratio = r["oracle_us_per_query"] / (0.5 * (lo + hi))
        assert abs(ratio - r["ratio_oracle_over_reference"]) < 1e-2 and 0.05 < ratio < 20


def test_no_gpu_fails_loudly(built):
    """Without a usable GPU every compute path reports LIVO_E_HIP: there is no CPU fallback."""
    import livo_amd
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except Exception:
        pass
    with pytest.raises(livo_amd.LivoError) as e:
        livo_amd.Context(0)
    assert e.value.code == -2


def test_struct_layouts_match_c(tmp_path):
    import livo_amd
    src = tmp_path / "sz.c"
    src.write_text('#include "livo.h"\n#include <stdio.h>\n#include <stddef.h>\nint main(void){printf("%zu %zu %zu %zu '
                   '%zu %zu %zu %zu\\n", sizeof(livo_params), sizeof(livo_state), sizeof(livo_iter_stats), '
                   'sizeof(livo_map_info), sizeof(livo_point_out), sizeof(livo_timings), '
                   'offsetof(livo_params, max_iterations), offsetof(livo_iter_stats, solution));return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    want = [C.sizeof(livo_amd.Params), C.sizeof(livo_amd.State), C.sizeof(livo_amd.IterStats),
            C.sizeof(livo_amd.MapInfo), C.sizeof(livo_amd.PointOut), C.sizeof(livo_amd.Timings),
            livo_amd.Params.max_iterations.offset, livo_amd.IterStats.solution.offset]
    assert got == want
    import oracle
    assert C.sizeof(oracle.OrcState) == C.sizeof(livo_amd.State)


def test_ikfom_struct_layouts_match_c(tmp_path):
    import livo_amd
    import oracle
    src = tmp_path / "ik.c"
    src.write_text('#include "livo.h"\n#include <stdio.h>\n#include <stddef.h>\nint main(void){printf("%zu %zu %zu '
                   '%zu %zu\\n", sizeof(livo_ikfom_state), sizeof(livo_ikfom_stats), offsetof(livo_ikfom_state, cov), '
                   'offsetof(livo_ikfom_stats, dx), offsetof(livo_ikfom_stats, res_mean));return 0;}\n')
    exe = tmp_path / "ik"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    want = [C.sizeof(livo_amd.IkfomState), C.sizeof(livo_amd.IkfomStats), livo_amd.IkfomState.cov.offset,
            livo_amd.IkfomStats.dx.offset, livo_amd.IkfomStats.res_mean.offset]
    assert got == want
    assert C.sizeof(oracle.OrcIkfomState) == C.sizeof(livo_amd.IkfomState)
    assert C.sizeof(oracle.OrcIkfomStats) == C.sizeof(livo_amd.IkfomStats)


def test_ivox_abi_layouts_and_args(tmp_path, built):
    import livo_amd
    src = tmp_path / "iv.c"
    src.write_text('#include "livo.h"\n#include <stdio.h>\n#include <stddef.h>\nint main(void){printf("%zu %zu %zu '
                   '%d %d %d\\n", sizeof(livo_ivox_params), sizeof(livo_ivox_info), offsetof(livo_ivox_params, '
                   'capacity), LIVO_BACKEND_IKDTREE, LIVO_BACKEND_IVOX, LIVO_E_CAPACITY);return 0;}\n')
    exe = tmp_path / "iv"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert got == [C.sizeof(livo_amd.IvoxParams), C.sizeof(livo_amd.IvoxInfo), livo_amd.IvoxParams.capacity.offset,
                   livo_amd.BACKEND_IKDTREE, livo_amd.BACKEND_IVOX, -7]
    L = livo_amd.load()
    p = livo_amd.IvoxParams()
    assert L.livo_ivox_params_default(C.byref(p)) == 0
    # reference defaults: ivox_grid_resolution 0.2, NEARBY18 (laser_mapping.cpp:1021-1035), capacity 1e6
    assert abs(p.resolution - 0.2) < 1e-7 and p.nearby_type == 18 and p.capacity == 1_000_000
    assert L.livo_ivox_params_default(None) == -1
    assert L.livo_ivox_init(None, None) == -1
    assert L.livo_ctx_set_backend(None, 1) == -1
    assert L.livo_ivox_add_points(None, None, 0, 0) == -1
    assert L.livo_map_incremental(None, 0, None, 0.5, 1, None, None) == -1
    assert L.livo_scan_inherit_neighbors(None, 0, 0) == -1
    assert b"capacity" in L.livo_error_string(-7)
