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
