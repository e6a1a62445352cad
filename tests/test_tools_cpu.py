"""CPU: the measurement tooling that bench.py's roofline fields depend on.

bench.py reads the committed PMC summaries (profiles/r01_pmc_*.json) by
kernel name.  The kernels are templates on their rows per thread (rows_a_for /
rows_b_for), so rocprofv3 reports e.g. `void k_shared_secret<4>`; the summary
tool must map the full-batch instances to the names bench.py looks up."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _pmc_summary():
    spec = importlib.util.spec_from_file_location("pmc_summary", os.path.join(ROOT, "tools", "pmc_summary.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_kernel_names():
    k = _pmc_summary().kernel_key
    assert k("void k_shared_secret<4>(unsigned int const*, unsigned int const*, unsigned int)") == "k_shared_secret"
    assert k("void k_shared_secret<1>(unsigned int const*)") == "k_shared_secret<1>"
    assert k("void k_match<false, 6>(unsigned int const*, unsigned int)") == "void k_match<false>"
    assert k("void k_match<true, 6>(x)") == "void k_match<true>"
    assert k("void k_match<false, 2>(x)") == "void k_match<false, 2>"
    assert k("k_layout_probe(unsigned int const*)") == "k_layout_probe"
    assert k("void k_scan_multi<26>(MultiBatch const*, unsigned int)") == "k_scan_multi"
    assert k("void k_scan_multi<26, true>(cudasp::MultiBatch const*, unsigned int)") == "k_scan_multi"


def test_committed_profiles_have_bench_keys():
    """The summaries bench.py reads by default carry the counters it uses."""
    sq = json.load(open(os.path.join(ROOT, "profiles", "r01_pmc_sq_counters.json")))["per_kernel"]
    for name in ("k_shared_secret", "void k_match<false>"):
        assert sq[name]["SQ_INSTS_VALU"] > 0, name
    hbm = json.load(open(os.path.join(ROOT, "profiles", "r01_pmc_k_shared_secret.json")))
    assert hbm["hbm_bytes_per_launch"] > 0
    per = hbm["per_kernel"]
    assert per["k_shared_secret"]["FETCH_SIZE_KiB_per_launch"] > 0
    assert per["k_layout_probe"]["FETCH_SIZE_KiB_per_launch"] > 0


def _lib_path():
    return os.path.join(ROOT, "duckdb-cudasp-extension_amd", "libcudasp_amd.so")


def _codeobj():
    spec = importlib.util.spec_from_file_location("codeobj", os.path.join(ROOT, "tools", "codeobj.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_code_stamp_names_one_kernel():
    """tools/codeobj.py finds the bench's timed kernel in the library's gfx950
    code object, and the stamp is a function of its machine code only."""
    import pytest
    co = _codeobj()
    if not os.path.exists(_lib_path()):
        pytest.skip("library not built")
    a = co.kernel_stamp(_lib_path(), co.multi_pattern(26))
    assert a["symbol"].startswith("_Z12k_scan_multiILi26ELb1EE") and a["code_bytes"] > 10000
    assert co.kernel_stamp(_lib_path(), co.multi_pattern(26)) == a
    b = co.kernel_stamp(_lib_path(), co.multi_pattern(22))
    assert b["sha256"] != a["sha256"]
    with pytest.raises(ValueError):
        co.kernel_stamp(_lib_path(), r"^_Z12k_scan_multi")  # several instances


def test_committed_counters_match_the_built_kernel():
    """bench.py reads roofline traffic and VALU counts only from summaries
    stamped with the loaded kernel's machine code.  The tree must carry such
    summaries for the default shapes (config 4, config 3, the config-5 shape)
    and the ladder-mix ceiling: a change to k_scan_multi<26,true> without new
    PMC passes (tools/recipes/pmc.sh) fails here instead of reporting stale
    counters."""
    import glob
    import json
    import pytest
    co = _codeobj()
    if not os.path.exists(_lib_path()):
        pytest.skip("library not built")
    want = co.kernel_stamp(_lib_path(), co.multi_pattern(26))["sha256"]
    for name in ("pmc_hbm_multi", "pmc_sq_multi_L0_k2_w26", "pmc_sq_multi_L1_k2_w26", "pmc_sq_multi_L16_k1-15_w26",
                 "valu_ceiling"):
        stamps = []
        for p in glob.glob(os.path.join(ROOT, "profiles", "r0*_%s.json" % name)):
            d = json.load(open(p))
            stamps.append(((d.get("code_stamp") or {}).get("k_scan_multi") or {}).get("sha256"))
        assert want in stamps, (name, want, stamps)


def test_committed_multi_profiles_have_bench_keys():
    """The newest summaries bench.py reads with --launch multi (the default):
    k_scan_multi's VALU count and GRBM cycles per launch with its rows, and
    its HBM traffic per row."""
    sq = json.load(open(os.path.join(ROOT, "profiles", "r06_pmc_sq_multi_L0_k2_w26.json")))
    k = sq["per_kernel"]["k_scan_multi"]
    assert k["SQ_INSTS_VALU"] > 0 and k["GRBM_GUI_ACTIVE"] > 0 and sq["multi_rows_per_launch"] == 32_700_000
    hbm = json.load(open(os.path.join(ROOT, "profiles", "r06_pmc_hbm_multi.json")))
    assert hbm["multi_hbm_bytes_per_row"] > 0 and hbm["probe_hbm_bytes_per_row"] > 0


def test_stage_a_kernels_keep_three_blocks_per_cu():
    """The stage-A kernels run three 256-thread blocks per CU (CUDASP_WAVES_A,
    the persistent grids are sized for it): each block's LDS (the odd-multiple
    table's y, LdsY; the stream kernel's own) must fit a third of gfx950's
    160 KB, and its VGPRs a third of 512 per SIMD lane.  Read from the built
    code object's kernel descriptors, so a larger CUDASP_*_LDS_Y cannot lower
    the occupancy unnoticed."""
    import struct
    import pytest
    co = _codeobj()
    if not os.path.exists(_lib_path()):
        pytest.skip("library not built")
    elf = co.code_objects(_lib_path())[0][1]
    syms, secs = co.symbols(elf)
    seen = 0
    for name, (val, size, typ, shndx) in syms.items():
        if not name.endswith(".kd") or not any(k in name for k in ("k_scan_multi", "k_scan_stream", "k_shared_secret")):
            continue
        kd = co._bytes_at(elf, secs, shndx, val, 64)
        lds, = struct.unpack_from("<I", kd, 0)
        rsrc1, = struct.unpack_from("<I", kd, 48)
        vgprs = ((rsrc1 & 0x3F) + 1) * 8  # gfx950: granules of 8, AGPRs included
        assert 3 * lds <= 160 * 1024, (name, lds)
        assert 3 * vgprs <= 512, (name, vgprs)
        seen += 1
    assert seen >= 8
