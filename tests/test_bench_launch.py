"""CPU: bench.py's launch modes.

`python bench.py --gpus N` with no launcher must drive N devices from one process through stc_group
(the reference's own deployment: one JVM on Spark local[*], LDATraining.scala:7) and report what ran;
under torchrun (WORLD_SIZE set) every rank drives its own GPU.  No GPU here: the device count and the
group are mocked, so only the bench's host logic runs.
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "spark-text-clustering_amd"))

import bench  # noqa: E402


def test_launch_mode():
    assert bench.launch_mode(1, {}) == ("single", 1, 0, 0)
    assert bench.launch_mode(8, {}) == ("group", 8, 0, 0)
    assert bench.launch_mode(2, {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"}) == ("ranks", 2, 1, 1)
    assert bench.launch_mode(1, {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})[0] == "ranks"
    # --launch group: one stc_group even at N = 1 (its RCCL communicator under STC_GROUP_RCCL=1)
    assert bench.launch_mode(1, {}, True) == ("group", 1, 0, 0)


class FakeGroup:
    """stands in for stc.LdaGroup: records the devices and the corpus split, counts next() calls"""
    made = []

    def __init__(self, devices, k, vocab_size, **kw):
        self.devices, self.k, self.V = list(devices), k, vocab_size
        self.steps = 0
        self.rows = 0
        FakeGroup.made.append(self)

    def set_corpus(self, corpus):
        self.rows = corpus.num_rows
        self.nnz = corpus.nnz

    def init_random(self, seed):
        pass

    def set_topics(self, t):
        pass

    def next(self, stats=True):
        self.steps += 1

    def synchronize(self):
        pass

    def enable_timing(self, on=True):
        pass

    def transport(self):
        return "rccl" if len(self.devices) > 1 else "none"

    def counters(self):
        n = len(self.devices)
        return [{"docs": 10 * self.steps, "entries": 1000 * self.steps, "inner_iters": 50 * self.steps,
                 "cap_hits": 0, "kernels": {"k_estep_rows64": self.steps, "k_estep": 0}} for _ in range(n)]

    def phase_times(self):
        return [{"sample": 0.1, "estep": 1.0 + i, "sstats": 0.2, "allreduce": 0.3, "mstep": 0.1, "steps": 5}
                for i in range(len(self.devices))]


def _run_bench(monkeypatch, capsys, argv, n_dev):
    import stc

    FakeGroup.made.clear()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(stc.Context, "device_count", staticmethod(lambda: n_dev))
    monkeypatch.setattr(stc, "LdaGroup", FakeGroup)
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    bench.main()
    out = capsys.readouterr().out.strip().splitlines()
    return json.loads(out[-1])


def test_gpus_n_without_launcher_drives_a_group(monkeypatch, capsys):
    line = _run_bench(monkeypatch, capsys, ["--gpus", "2", "--steps", "3", "--warmup", "1", "--docs", "2000",
                                            "--tokens", "20", "--vocab", "4096", "--k", "8", "--workers", "1",
                                            "--no-hbm-copy"], n_dev=2)
    (g,) = FakeGroup.made
    assert g.devices == [0, 1]
    assert g.rows == 2000  # strong scaling: the whole corpus, sharded by the group
    assert line["n_gpus"] == 2
    assert line["config"]["parallelism"] == "group2"
    assert line["config"]["baseline_config"] == "configs[2]"
    assert line["cpu_baseline"] is None and line["secondary"] == []
    # value = docs of all members / wall time; the roofline uses member 0's K6 window (E-step + sstats)
    assert line["value"] > 0
    assert line["config"]["phase_ms"]["estep_slowest_member"] == 2.0
    assert line["roofline"]["kernel_ms_per_launch"] == pytest.approx(1.2)
    split = line["roofline"]["phase_split"]
    assert split["estep"]["ms"] == 1.0 and split["sstats"]["ms"] == 0.2
    # the split's bytes add up to the window's
    assert split["estep"]["algorithmic_bytes"] + split["sstats"]["algorithmic_bytes"] == pytest.approx(
        line["roofline"]["algorithmic_bytes_per_launch"])
    assert line["parity"].startswith("north-star bars met")  # the fp64 headline
    # the kernel named is the one the library counted as launched in the timed steps
    assert line["roofline"]["kernel"].startswith("k_estep_rows64_pers")


def test_kernel_name_comes_from_the_launch_counters():
    assert bench.kernel_name({"k_estep_wide": 20}).startswith("k_estep_wide (")
    n = bench.kernel_name({"k_estep_tgrid64": 19, "k_estep_wide": 1, "team_fallback": 1})
    assert n.startswith("k_estep_tgrid64") and "team_fallback" in n
    assert bench.kernel_name({}) == "no E-step launch in the timed steps"
    # mixed: the fp32 pass names the step, the fp64 re-solve is listed beside it
    m = bench.kernel_name({"k_estep_rows64": 10, "k_estep_grid": 10, "mixed_resolves": 10, "mixed_docs": 6300})
    assert m.startswith("k_estep_grid_pers") and "mixed_docs" in m


def test_group_launch_at_one_gpu(monkeypatch, capsys):
    """--launch group at N = 1: the group path (group1) on device 0, reported as such."""
    line = _run_bench(monkeypatch, capsys, ["--launch", "group", "--steps", "2", "--warmup", "0", "--docs", "800",
                                            "--tokens", "10", "--vocab", "1024", "--k", "4", "--workers", "1",
                                            "--no-hbm-copy", "--no-cpu-baseline"], n_dev=1)
    (g,) = FakeGroup.made
    assert g.devices == [0] and line["n_gpus"] == 1 and line["config"]["parallelism"] == "group1"


def test_gpus_n_fails_loudly_when_fewer_devices_are_visible(monkeypatch, capsys):
    with pytest.raises(SystemExit, match="only 1 device"):
        _run_bench(monkeypatch, capsys, ["--gpus", "4", "--steps", "1", "--warmup", "0", "--docs", "500",
                                         "--tokens", "10", "--vocab", "1024", "--k", "4", "--workers", "1",
                                         "--no-hbm-copy"], n_dev=1)


def test_weak_group_corpus_is_one_shard_per_member(monkeypatch, capsys):
    line = _run_bench(monkeypatch, capsys, ["--gpus", "2", "--scaling", "weak", "--steps", "1", "--warmup", "0",
                                            "--docs", "600", "--tokens", "10", "--vocab", "1024", "--k", "4",
                                            "--workers", "1", "--no-hbm-copy"], n_dev=3)
    (g,) = FakeGroup.made
    assert g.rows == 1200 and line["scaling"] == "weak" and line["n_gpus"] == 2


def test_traffic_is_null_with_a_reason_unless_measured_on_these_sources(tmp_path, monkeypatch):
    class A:
        docs, k, vocab, tokens, fraction = 1000000, 100, 1 << 18, 200, 0.05

    wl = {"docs": A.docs, "tokens": A.tokens, "vocab": A.vocab, "k": A.k, "fraction": A.fraction,
          "corpus": "zipf", "dtype": "f64"}
    p = tmp_path / "pmc.json"
    monkeypatch.setattr(bench, "PMC_SUMMARY", str(p))
    p.write_text(json.dumps({"entries": [{"workload": wl, "estep_kernel": [], "estep_kernel_bytes_per_launch": 0.0}]}))
    b, why = bench.pmc_traffic(A, "f64", "zipf")
    assert b is None and "no E-step kernel" in why
    p.write_text(json.dumps({"entries": [{"workload": wl, "estep_kernel": ["k"], "estep_kernel_bytes_per_launch": 4.6e9,
                                          "estep_sources_sha": "0" * 16}]}))
    b, why = bench.pmc_traffic(A, "f64", "zipf")
    assert b is None and "other E-step sources" in why
    p.write_text(json.dumps({"entries": [{"workload": wl, "estep_kernel": ["k"], "estep_kernel_bytes_per_launch": 4.6e9,
                                          "estep_sources_sha": bench.estep_sources_sha()}]}))
    t = bench.pmc_traffic(A, "f64", "zipf")[0]
    assert t["kernel"] == 4.6e9 and t["window"] is None  # no window / phase bytes in this entry
    p.write_text(json.dumps({"entries": [{"workload": wl, "estep_kernel": ["k"], "estep_kernel_bytes_per_launch": 4.6e9,
                                          "k6_window_bytes_per_step": 6.1e9,
                                          "estep_sources_sha": bench.estep_sources_sha()}]}))
    t = bench.pmc_traffic(A, "f64", "zipf")[0]
    assert t == {"kernel": 4.6e9, "window": 6.1e9} and np.isfinite(t["window"])


def test_featurisation_traffic_is_bound_to_its_sources(tmp_path, monkeypatch):
    """The featurisation line's `traffic` comes from the committed PMC summary only when it was measured on
    this tree's featurisation sources (bench.FEAT_SOURCES); otherwise null with the reason."""
    p = tmp_path / "feat_pmc.json"
    monkeypatch.setattr(bench, "FEAT_PMC", str(p))
    t, why = bench.feat_traffic()
    assert t is None and "no featurisation PMC" in why
    stages = {"hashing_tf": {"bytes_per_call": 4.4e9}, "idf_fit": {"bytes_per_call": 0.8e9},
              "idf_transform": {"bytes_per_call": 3.3e9}}
    p.write_text(json.dumps({"feat_sources_sha": "0" * 16, "stages": stages}))
    t, why = bench.feat_traffic()
    assert t is None and "other featurisation sources" in why
    p.write_text(json.dumps({"feat_sources_sha": bench.feat_sources_sha(), "stages": stages}))
    t, _ = bench.feat_traffic()
    assert t == {"hashing_tf": 4.4e9, "idf_fit": 0.8e9, "idf_transform": 3.3e9}
    # the committed summary matches this tree
    monkeypatch.undo()
    assert bench.feat_traffic()[0] is not None
