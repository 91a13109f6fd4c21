"""bench.py's printed line stays parseable by the driver: strict JSON under bench.LINE_MAX bytes, built by
bench.compact_line from a full (detail) record.  Round 4's 27.4 KB line came back `parsed: null`; the full
record now goes to --detail-out and the line carries only the contract keys, a lean roofline /
cpu_baseline and the per-leg summary.  Fed from a recorded detail file (profiles/r05_bench_detail.json
when present) and from round 4's record inflated with every leg this round adds, at full size."""
import copy
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEAD_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
             "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "summary")


def _from_r04():
    """Round 4's recorded full line recast as a detail record, plus hash / Merkle / device-set legs with
    every field the new code writes (long names, all legs present: the worst case for the line's size)."""
    with open(os.path.join(ROOT, "profiles", "r04_bench_default.json")) as f:
        d = json.load(f)
    full = copy.deepcopy(d)
    full["head_name"] = "c2"
    full["head"] = {"value": d["value"], "ms_per_step": d["ms_per_step"], "roofline": d["roofline"]}
    full["detail_path"] = "gpurun_out/bench_detail.json"
    pmc = {"valu_issue": 0.61234, "valu_per_unit": 1.2345e7, "source": "profiles/r05_pmc_legs.json",
           "same_kernel_source": True, "traffic": 1.234e8}
    rf = {"bound": "int-valu", "frac": 0.61234, "useful_ops_per_s": 3.1e13, "useful_frac": 0.8312,
          "peak_ops_per_s": bench.PEAK_ALU_PER_S, "units": 123456, "traffic": 1.234e8, "pmc": pmc,
          "algorithmic_bytes": 123456789}
    full["hashes"] = {name: {"hashes_per_s": 1.23456e9, "ms": 0.81234, "reps": 300, "messages": n, "bytes_each": ln,
                             "GB_per_s": 123.456, "roofline": rf}
                      for name, _, n, ln in bench.HASH_SPECS}
    for n, h, w in bench.MERKLE_SPECS:
        m = full["merkle"][bench.merkle_name(n, h, w)]
        m["roofline"] = dict(rf)
    full["devset"] = {"devices": [0, 1, 2, 3, 4, 5, 6, 7],
                      "c4": {"tx_s": 1.2345e8, "ms_per_step": 81.234, "steps": 13, "matches_single_device": True},
                      "c5": {"tx_s": 1.2345e8, "ms_per_step": 101.23, "steps": 11, "matches_single_device": True}}
    return full


def _records():
    out = [("r04+new legs", _from_r04())]
    p = os.path.join(ROOT, "profiles", "r05_bench_detail.json")
    if os.path.exists(p):
        with open(p) as f:
            out.append(("r05 detail", json.load(f)))
    return out


@pytest.mark.parametrize("which", range(len(_records())))
def test_line_is_strict_json_under_the_limit(which):
    name, full = _records()[which]
    line = bench.compact_line(full)
    text = bench.dumps_line(line)
    assert len(text) < bench.LINE_MAX, (name, len(text))
    back = json.loads(text, parse_constant=lambda c: pytest.fail("non-strict constant %s" % c))
    for k in HEAD_KEYS:
        assert k in back, (name, k)
    assert list(back)[-1] == "summary"  # the last key survives a tail-only record
    rf = back["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "useful_8d", "kernel", "kernel_ms", "traffic", "valu_issue"):
        assert k in rf, (name, k)
    assert 0 < rf["frac"] <= 1
    cb = back["cpu_baseline"]
    for k in ("value", "kind", "cores", "full_host_estimate"):
        assert k in cb, (name, k)
    assert "\n" not in text
    assert back["value"] == pytest.approx(full["value"])


def test_line_refuses_nan():
    full = _from_r04()
    full["head"]["roofline"]["kernel_ms"] = float("nan")
    with pytest.raises(ValueError):
        bench.dumps_line(bench.compact_line(full))


def test_roofline_fracs_of_recorded_legs_do_not_exceed_one():
    """Every leg's reported roofline `frac` (the executed-issue fraction) is <= 1 in a recorded detail
    file; the SURVEY 8(d) op-count figure is carried separately as useful_frac / frac_8d."""
    p = os.path.join(ROOT, "profiles", "r05_bench_detail.json")
    if not os.path.exists(p):
        pytest.skip("no round-5 detail record yet")
    with open(p) as f:
        full = json.load(f)
    fracs = [full["head"]["roofline"]["frac"]] + [v["roofline"]["frac"] for v in full.get("legs", {}).values()]
    for grp in ("hashes", "merkle"):
        fracs += [v["roofline"]["frac"] for v in (full.get(grp) or {}).values()
                  if isinstance(v, dict) and "roofline" in v]
    assert all(f is None or 0 < f <= 1 for f in fracs), fracs


def test_line_survives_failed_extra_legs():
    """An extra rank-0 leg that raised is recorded as {"error": ...} (bench._safe): the line still parses,
    lists the failed legs under summary.errors, and keeps every other leg; a failed CPU baseline leaves
    cpu_baseline null."""
    full = copy.deepcopy(_records()[-1][1])
    for k in ("devset", "pcie_inclusive", "interface", "merkle", "cpu_baseline"):
        full[k] = {"error": "RuntimeError: boom " + "x" * 300, "leg": k}
    text = bench.dumps_line(bench.compact_line(full))
    back = json.loads(text)
    assert back["cpu_baseline"] is None
    assert set(back["summary"]["errors"]) == {"devset", "pcie_inclusive", "interface", "merkle", "cpu_baseline"}
    assert all(len(v) <= 200 for v in back["summary"]["errors"].values())
    assert "hashes[h/s,frac,useful]" in back["summary"] and back["value"] == full["value"]
    assert len(text) < bench.LINE_MAX


def test_safe_returns_error_record(capsys):
    assert bench._safe("x", lambda: {"ok": 1}) == {"ok": 1}
    r = bench._safe("x", lambda: 1 / 0)
    assert r["leg"] == "x" and r["error"].startswith("ZeroDivisionError")
    assert "Traceback" in capsys.readouterr().err
