"""DESIGN.md §5's and README.md's measured values trace to the committed bench
lines in profiles/ (VERDICT r4 #7, r5 #6): each DESIGN table row's value
equals its line's `value` (in k Mpx/s, one decimal; OF two decimals) and its
per-run spread the line's `timing.value_per_run` range; every bench line a
README row names carries that line's value. CPU only: reads text and JSON."""
import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ROWS = [   # (row label prefix in DESIGN §5, profiles line, decimals)
    ("**FD 1080p, configs[1] (headline)**", "r6_bench_fd_1080p.json", 1),
    ("FD 1080p, configs[1], the operating points' box", "r6_bench_fd_1080p_box_b.json", 1),
    ("FD 4K, configs[2]", "r6_bench_fd_4k.json", 1),
    ("FD 1080p noisy", "r6_bench_fd_noisy.json", 1),
    ("FD 1080p, NV12 decoder surfaces in place", "r6_bench_fd_nv12_input.json", 1),
    ("FD 1080p, I420 decoder surfaces in place", "r6_bench_fd_i420_input.json", 1),
    ("FD 1080p, I420 outputs", "r6_bench_fd_i420_output.json", 1),
    ("FD 1080p, NV12 in place → I420 outputs", "r6_bench_fd_nv12_input_i420_output.json", 1),
    ("FD 1080p, the reference's `__main__` kwargs", "r6_bench_fd_b8_k10_r0.3.json", 1),
    ("OF 1080p, configs[4]", "r6_bench_of_1080p.json", 2),
    ("OF 1080p, NV12 in place", "r6_bench_of_nv12_input.json", 2),
]


def _section5():
    text = open(os.path.join(ROOT, "DESIGN.md"), encoding="utf-8").read()
    a = text.index("## 5. Measured")
    return text[a:text.index("## 6.", a)]


def _k(v, dec):
    return f"{v / 1000:.{dec}f}"


@pytest.mark.parametrize("label,fname,dec", ROWS)
def test_design_table_traces_to_profiles(label, fname, dec):
    sec = _section5()
    row = next((ln for ln in sec.splitlines() if ln.startswith("| " + label)), None)
    assert row is not None, f"DESIGN §5 has no row {label!r}"
    cells = [c.strip() for c in row.strip("|").split("|")]
    d = json.load(open(os.path.join(ROOT, "profiles", fname)))
    nums = re.findall(r"\d+\.\d+", cells[1])
    assert nums and nums[0] == _k(d["value"], dec), f"{label}: {cells[1]} vs {d['value']}"
    runs = d["timing"]["value_per_run"]
    lo, hi = re.findall(r"\d+\.\d+", cells[2])[:2]
    assert (lo, hi) == (_k(min(runs), dec), _k(max(runs), dec)), f"{label}: spread {cells[2]} vs {runs}"


def test_design_batch_curve_traces_to_profiles():
    sec = _section5()
    for fname in ("r6_bench_fd_per_frame.json", "r6_bench_fd_batch8.json", "r6_bench_fd_batch32.json",
                  "r6_bench_fd_batch128.json", "r6_bench_fd_out_ring1.json", "r6_bench_fd_1080p_box_b.json"):
        row = next(ln for ln in sec.splitlines() if ln.startswith("|") and fname in ln)
        d = json.load(open(os.path.join(ROOT, "profiles", fname)))
        assert _k(d["value"], 1) in row, f"{fname}: {row}"


def test_readme_table_traces_to_profiles():
    text = open(os.path.join(ROOT, "README.md"), encoding="utf-8").read()
    rows = [ln for ln in text.splitlines() if ln.startswith("| ") and "_bench_" in ln]
    assert len(rows) >= 4
    seen = 0
    for row in rows:
        for fname in re.findall(r"r\d+_bench_[\w.]+?\.json", row):
            d = json.load(open(os.path.join(ROOT, "profiles", fname)))
            dec = 2 if "_of_" in fname else 1
            assert _k(d["value"], dec) in row, f"README: {fname} value {d['value']} not in {row!r}"
            seen += 1
    assert seen >= 7
    # the performance table quotes this round's closing refresh
    assert "r5_bench" not in text and "r4_bench" not in text
