"""bench.py's triad-ceiling helpers (CPU): the live quick-mode parse, the
committed file's fallback, and the line's fields they feed
(roofline.ceiling_measured / frac_of_ceiling)."""
import os
import stat

import bench


def test_ceiling_of_picks_the_best_triad_form_and_the_pure_streams():
    rows = [
        {"form": "read2 U2", "wg_per_cu": 1, "gbs_avg": 7000.0},
        {"form": "read2 U2", "wg_per_cu": 2, "gbs_avg": 7300.0},
        {"form": "write1 U4", "wg_per_cu": 1, "gbs_avg": 6200.0},
        {"form": "triad U1", "wg_per_cu": 1, "gbs_avg": 6100.0},
        {"form": "triad U1", "wg_per_cu": 2, "gbs_avg": 6400.0},
        {"form": "triadL D4 nt", "wg_per_cu": 1, "gbs_avg": 6350.0},
        {"bogus": 1},
    ]
    c = bench._ceiling_of(rows, "src")
    assert c["gbs"] == 6400.0 and c["form"] == "triad U1, 2 WG/CU"
    assert c["read2_gbs"] == 7300.0 and c["write1_gbs"] == 6200.0
    assert c["forms_measured"] == 3 and c["source"] == "src"
    assert bench._ceiling_of([{"form": "read2 U2", "wg_per_cu": 1, "gbs_avg": 1.0}], "x") is None


def test_committed_ceiling_file_loads():
    c = bench.load_triad_ceiling()
    assert c is not None and 5000.0 < c["gbs"] < 8000.0 and "another box" in c["source"]


def test_live_ceiling_parses_the_quick_mode_output(tmp_path, monkeypatch):
    # a stand-in for the microbenchmark binary: prints quick-mode lines
    ub = tmp_path / "scripts" / "ubench"
    ub.mkdir(parents=True)
    exe = ub / "ub_triad_ceiling.bin"
    exe.write_text("#!/bin/sh\n"
                   "[ \"$1\" = quick ] || exit 9\n"
                   "echo 'noise'\n"
                   "echo '{\"form\": \"triad U1\", \"wg_per_cu\": 2, \"avg_ms\": 0.5, \"gbs_avg\": 6440.5, \"gbs_best\": 6500.0}'\n"
                   "echo '{\"form\": \"read2 U2\", \"wg_per_cu\": 1, \"avg_ms\": 0.3, \"gbs_avg\": 7100.0, \"gbs_best\": 7200.0}'\n")
    exe.chmod(exe.stat().st_mode | stat.S_IXUSR)
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    c = bench.measure_triad_ceiling_live()
    assert c["gbs"] == 6440.5 and c["read2_gbs"] == 7100.0 and c["source"].startswith("live:")


def test_live_ceiling_is_none_without_the_binary_or_on_failure(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.measure_triad_ceiling_live() is None
    ub = tmp_path / "scripts" / "ubench"
    ub.mkdir(parents=True)
    exe = ub / "ub_triad_ceiling.bin"
    exe.write_text("#!/bin/sh\nexit 3\n")
    exe.chmod(exe.stat().st_mode | stat.S_IXUSR)
    assert bench.measure_triad_ceiling_live() is None
    assert os.path.exists(str(exe))
