"""tools/plot_results.py (A34 analogue) over the committed profiles."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_plots_and_summary(tmp_path):
    import plot_results

    data = plot_results.load(os.path.join(ROOT, "profiles"))
    assert data["allops"] and data["bench"] is not None
    plot_results.main(["--profiles", os.path.join(ROOT, "profiles"), "--out", str(tmp_path), "--fmt", "png"])
    rows = (tmp_path / "summary.csv").read_text().splitlines()
    assert rows[0].startswith("benchmark,")
    assert any(r.startswith("lr_query,") for r in rows)
    for name in ("allops.png", "lr_timeline.png"):
        assert (tmp_path / name).stat().st_size > 1000
