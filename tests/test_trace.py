"""Tracing: host ranges recorded and exported as Chrome trace JSON."""
import json

from analyzer_amd.utils import trace


def test_trace_ranges_and_chrome_export(tmp_path, monkeypatch):
    from analyzer_amd.runtime.rerate import RerateSpec, run

    monkeypatch.setenv("ANA_TRACE", "1")
    trace.clear()
    run(RerateSpec(total_matches=600, players=50, window=200, seed=3), "cpu",
        checkpoint_dir=str(tmp_path / "ck"), checkpoint_every=1)
    names = [e["name"] for e in trace.events()]
    assert names.count("rate") == 3 and names.count("checkpoint") == 3
    n = trace.dump_chrome_trace(str(tmp_path / "t.json"))
    doc = json.load(open(str(tmp_path / "t.json")))
    assert n == len(doc["traceEvents"]) and all(e["ph"] == "X" and e["dur"] >= 0 for e in doc["traceEvents"])


def test_trace_disabled_records_nothing(monkeypatch):
    monkeypatch.delenv("ANA_TRACE", raising=False)
    trace.clear()
    with trace.trace_range("x"):
        pass
    assert trace.events() == []
