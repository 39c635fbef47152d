"""tools/pmc_summary.py (CPU): which rocprofv3 kernel names count as the training E-step launch, and
that a summary naming no E-step kernel is refused rather than written as an empty traffic entry."""
import csv
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)

import pmc_summary as P  # noqa: E402

# names as rocprofv3 reports them (after short()), from profiles/r04*_pmc.json and r02 / r03 profiles
TRAINING = [
    "k_estep_rows64<RShape<13, 5, 6>, true, false>",
    "k_estep_rows64_long<RShape<13, 8, 8>, true, false>",
    "k_estep_grid<GShape<2, 26, 6, 2>, true, false, true>",
    "k_estep_grid<GShape<2, 26, 6, 2>, true, false, false>",
    "k_estep_grid_long<GShape<2, 26, 8, 1>, true, false>",
    "k_estep_wide_mc<double, 1, 64, true>",
    "k_estep_wide_tc<double, 2, 24, true>",
    "k_estep_grid64<DShape<13, 5>, true, false, true>",
    "k_estep<double, true, false>",
    "k_estep_wide<float, 4, 32, true, false>",
]
NOT_TRAINING = [
    "k_estep_rows64<RShape<13, 5, 6>, false, true>",   # the bound's E-step
    "k_estep_grid<GShape<2, 26, 6, 2>, false, false, true>",  # inference
    "k_estep_wide_mc<double, 1, 64, false>",
    "k_sstats<double, 8>",
    "k_lambda_eeb<double, 4, true>",
]


@pytest.mark.parametrize("name", TRAINING)
def test_training_estep_names_match(name):
    assert P.ESTEP.search(name), name


@pytest.mark.parametrize("name", NOT_TRAINING)
def test_other_kernels_do_not_match(name):
    assert not P.ESTEP.search(name), name


def _write(path, rows, counter):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for kn, v in rows:
            w.writerow({"Kernel_Name": f"void {kn}(int)", "Counter_Name": counter, "Counter_Value": v})


def test_summary_without_an_estep_kernel_is_refused(tmp_path, monkeypatch):
    d = tmp_path / "prof"
    os.makedirs(d / "stats")
    (d / "stats" / "stats_kernel_stats.csv").write_text("Name,Calls\n")
    rows = [("k_sstats<double, 8>", 10.0), ("k_lambda_eeb<double, 4, true>", 5.0)]
    _write(str(d / "fetch" / "fetch_counter_collection.csv"), rows, "FETCH_SIZE")
    _write(str(d / "write" / "write_counter_collection.csv"), rows, "WRITE_SIZE")
    monkeypatch.setattr(P, "ROOT", str(tmp_path))
    monkeypatch.setattr(sys, "argv", ["pmc_summary.py", str(d), "--tag", "t"])
    with pytest.raises(SystemExit) as e:
        P.main()
    assert "refusing" in str(e.value)
    assert not (tmp_path / "profiles" / "pmc_traffic.json").exists()
