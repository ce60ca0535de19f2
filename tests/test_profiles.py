"""The committed traffic profiles describe this tree's kernels: bench.py falls back to
profiles/pmc_traffic*.json for roofline.traffic only when its live PMC leg cannot run, and
then only when the profile's csrc_sha matches the library sources; this test keeps every
committed profile HEAD-stamped (a csrc/ change without a re-measurement fails here)."""
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scripts"))


def test_traffic_profiles_match_the_library_sources():
    from pmc_traffic import csrc_sha
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_traffic*.json")))
    assert paths, "no committed traffic profile"
    sha = csrc_sha()
    for p in paths:
        t = json.load(open(p))
        assert t.get("csrc_sha") == sha, (f"{os.path.basename(p)} was measured on other library sources "
                                          f"({t.get('csrc_sha')} vs {sha}): re-measure (scripts/traffic_from_bench.py)")
        assert t["conv_engine_bytes_per_step"] > 0


def test_per_call_traffic_table_matches_the_aggregate():
    """The committed per-conv-call traffic table (profiles/pmc_layers.md, scripts/pmc_layers.py)
    is of the same library sources as the aggregate profiles/pmc_traffic.json: both carry this
    tree's csrc_sha."""
    from pmc_traffic import csrc_sha
    path = os.path.join(REPO, "profiles", "pmc_layers.md")
    assert os.path.exists(path), "no committed per-call traffic table"
    text = open(path).read()
    agg = json.load(open(os.path.join(REPO, "profiles", "pmc_traffic.json")))
    assert f"csrc_sha {csrc_sha()}" in text, "profiles/pmc_layers.md was measured on other library sources"
    assert agg.get("csrc_sha") == csrc_sha()
    assert "| net | layer | op |" in text
