"""bench.py's roofline plumbing on the CPU: the PMC summary is used only for the exact config, kernel and
library build it was measured on, and the committed summary is keyed the way bench.py looks it up."""
import importlib.util
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_pmc_summary_matched_on_config_kernel_and_library(tmp_path):
    b = bench()
    k = "rt::persistent_df_kernel<false, false, 23>"
    d = {"config": b.pmc_key("C3", 64), "kernel": f"void {k}(rt::KParams, rt::JobSrc)", "lib_sha": "abc",
         "hbm_bytes_per_launch": 123.0, "note": "n"}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps(d))
    assert b.load_pmc("C3v64", k, "abc", str(p))[0] == 123.0
    assert b.load_pmc("C3v16", k, "abc", str(p))[0] is None  # another batch size
    assert b.load_pmc("C3v64", "rt::persistent_df_kernel<false, false, 0>", "abc", str(p))[0] is None
    assert b.load_pmc("C3v64", k, "def", str(p))[0] is None  # another library build
    assert b.load_pmc("C3v64", k, "abc", str(tmp_path / "missing.json"))[0] is None


def test_committed_summary_is_keyed_for_the_default_bench():
    b = bench()
    d = json.load(open(os.path.join(REPO, "profiles", "pmc_latest.json")))
    assert d["config"] == b.pmc_key("C3", b.DEFAULT_VIEWS)
    # the bench's render kernel (the opaque-scene kernel for C3 since round 3), its plain (non-counting) build
    assert any(k in d["kernel"] for k in ("persistent_opaque_kernel<false", "persistent_df_kernel<false"))
    assert d["hbm_bytes_per_launch"] > 0
