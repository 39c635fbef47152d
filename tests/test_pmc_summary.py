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
    "k_estep_rows64_pers<RShape<13, 5, 6>, true, false>",
    "k_estep_grid_pers<GShape<2, 26, 6, 2>, true, false, false>",
    "k_estep_grid<GShape<2, 26, 6, 2>, true, false, true>",
    "k_estep_grid<GShape<2, 26, 6, 2>, true, false, false>",
    "k_estep_grid_long<GShape<2, 26, 8, 1>, true, false>",
    "k_estep_wide_mc<double, 1, 64, true>",
    "k_estep_wide_tc<double, 2, 24, true>",
    "k_estep_grid64<DShape<13, 5>, true, false, true>",
    "k_estep<double, true, false>",
    "k_estep_wide<float, 4, 32, true, false>",
    "k_estep_tgrid64<13, true>",
]
NOT_TRAINING = [
    "k_estep_rows64<RShape<13, 5, 6>, false, true>",   # the bound's E-step
    "k_estep_rows64_pers<RShape<13, 5, 6>, false, false>",  # inference on the resident grid
    "k_estep_grid<GShape<2, 26, 6, 2>, false, false, true>",  # inference
    "k_estep_wide_mc<double, 1, 64, false>",
    "k_estep_tgrid64<13, false>",
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


def test_steady_window_keeps_the_last_dispatches(tmp_path):
    """--steady: only the last fraction of each kernel's dispatches (the timed minibatches) is averaged,
    both in the kernel-trace stats table and in the counter passes (config 4's average
    included the cold launches)."""
    trace = tmp_path / "t.csv"
    with open(trace, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for i in range(10):  # 5 cold launches of 1000 ns, then 5 of 100 ns
            w.writerow({"Dispatch_Id": i + 1, "Kernel_Name": "k_estep", "Start_Timestamp": 0,
                        "End_Timestamp": 1000 if i < 5 else 100})
    out = tmp_path / "s.csv"
    P.steady_stats(str(trace), str(out), 0.5)
    (row,) = list(csv.DictReader(open(out)))
    assert int(float(row["Calls"])) == 5 and float(row["AverageNs"]) == 100.0
    rows = [{"Dispatch_Id": str(i), "v": i} for i in (3, 1, 2, 4)]
    assert [r["v"] for r in P._last(rows, 0.5)] == [3, 4]
    assert P.WINDOW.search("k_sstats<double, 2>") and P.WINDOW.search("k_estep_rows64<RShape<13, 5, 6>, true, false>")
    assert not P.WINDOW.search("k_lambda_eeb<double, 2, true>") and not P.WINDOW.search("k_sample")
