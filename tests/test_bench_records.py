"""bench.py's committed-counter loaders pick the HEADLINE records by name.

Round 5's loader kept the lexicographically last `profiles/pmc_*.json`, which became
`pmc_tiles_r05.json` (another benchmark's record, keyed "B" not "batch"), so the bench
line's `roofline.traffic` and `backward_leg.traffic` went null.
"""
import json
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]

import bench  # noqa: E402

PROFILES = os.path.join(ROOT, "profiles")


def test_traffic_resolves_to_the_headline_record_beside_the_tiles_record():
    assert os.path.exists(os.path.join(PROFILES, "pmc_tiles_r05.json"))
    rec, src = bench.load_pmc_traffic(PROFILES, 4096, 100)
    assert rec is not None, src
    # the newest headline record (round 5 or later); round 5's figures, when it is the newest
    newest = max(int(f[5:-5]) for f in os.listdir(PROFILES) if bench._HEADLINE_RECORD.match(f)
                 and f.startswith("pmc_"))
    assert src == f"profiles/pmc_r{newest:02d}.json"
    if newest == 5:
        assert rec["hbm_bytes_per_fused_launch"] == pytest.approx(530.7e6, rel=1e-3)
        assert rec["hbm_bytes_per_backward_launch"] == pytest.approx(240.1e6, rel=1e-3)
    # algorithmic bytes of one fused launch at B = 4096: 531.8 MB; the counters agree within 1 %
    c = bench.algorithmic_counts(100)
    alg = (c["bw_bytes"] + c["fw_bytes"]) * 4096
    assert rec["hbm_bytes_per_fused_launch"] == pytest.approx(alg, rel=0.01)


def test_loader_orders_rounds_numerically_and_ignores_other_benches(tmp_path):
    d = tmp_path / "profiles"
    d.mkdir()
    good = {"batch": 4096, "T": 100, "hbm_bytes_per_backward_launch": 2.0, "hbm_bytes_per_fused_launch": 3.0}
    (d / "pmc_r09.json").write_text(json.dumps(dict(good, hbm_bytes_per_fused_launch=9.0)))
    (d / "pmc_r10.json").write_text(json.dumps(good))          # r10 > r09 numerically
    (d / "pmc_tiles_r99.json").write_text(json.dumps({"B": 1}))
    (d / "pmc_r10_v2.json").write_text(json.dumps({"B": 1}))
    (d / "mfma_r03.json").write_text(json.dumps({"fused": {"MfmaUtil": 1}}))
    (d / "mfma_tiles_r04.json").write_text(json.dumps({"fused": {"MfmaUtil": 2}}))
    rec, src = bench.load_pmc_traffic(str(d), 4096, 100)
    assert src == "profiles/pmc_r10.json" and rec["hbm_bytes_per_fused_launch"] == 3.0
    assert bench.load_mfma_pmc(str(d))["fused"]["MfmaUtil"] == 1
    # another batch: no traffic, and the reason names the record
    rec, src = bench.load_pmc_traffic(str(d), 8192, 100)
    assert rec is None and "pmc_r10.json" in src and "batch=8192" in src


def test_malformed_headline_record_fails_loudly(tmp_path):
    d = tmp_path / "profiles"
    d.mkdir()
    (d / "pmc_r11.json").write_text(json.dumps({"B": 4096, "T": 100}))
    with pytest.raises(ValueError, match="lacks"):
        bench.load_pmc_traffic(str(d), 4096, 100)
    shutil.rmtree(d)
    assert bench.load_pmc_traffic(str(d), 4096, 100) == (None, "no profiles/pmc_rNN.json")
