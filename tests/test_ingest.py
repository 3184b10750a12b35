"""Native record-file ingest (C++ reader thread + SPSC ring) and the overlapped
file -> device -> host pipeline."""
import pytest
import torch

from analyzer_amd.ops.rate import BatchRater
from analyzer_amd.ops.synth import RosterSpec, StreamSpec, make_roster, make_stream
from analyzer_amd.runtime.ingest import FileSource, rate_file, write_records


def _data(M=1000, K=3, P=60):
    return make_stream(StreamSpec(team_size=K, seed=4, p_afk=0.05), M, P, K=K), K, P


@pytest.mark.parametrize("window,slots", [(128, 2), (1000, 3), (333, 4), (5000, 2)])
def test_reader_windows_reassemble_the_file(tmp_path, window, slots):
    rec, K, P = _data()
    path = str(tmp_path / "s.rec")
    write_records(path, rec, K)
    src = FileSource(path, window, "cpu", slots=slots)
    assert src.K == K and src.num_windows == -(-1000 // window)
    parts = list(src)
    assert [b for b, _ in parts] == list(range(0, 1000, window))
    assert torch.equal(torch.cat([r for _, r in parts]), rec)


def test_bad_file_is_rejected(tmp_path):
    from analyzer_amd.ops.native import native

    p = tmp_path / "x.rec"
    p.write_bytes(b"not a record file at all, definitely not" * 2)
    with pytest.raises(RuntimeError):
        native().RecordReader(str(p), 10, 2, False)


def test_rate_file_equals_direct_rating(tmp_path):
    rec, K, P = _data(M=900)
    path = str(tmp_path / "s.rec")
    write_records(path, rec, K)
    roster = make_roster(RosterSpec(num_players=P, seed=2))
    direct = roster.clone()
    ref = BatchRater().rate(direct, rec, K)
    got = {}
    n = rate_file(path, roster, 200, on_result=lambda base, host: got.__setitem__(base, host))
    assert n == 5 and sorted(got) == [0, 200, 400, 600, 800]
    s_mu = torch.cat([got[b]["s_mu"] for b in sorted(got)])
    assert torch.equal(s_mu.nan_to_num(-7), ref.s_mu.nan_to_num(-7))
    assert torch.equal(roster.state.nan_to_num(-7), direct.state.nan_to_num(-7))


def test_several_windows_held_at_once(tmp_path):
    from analyzer_amd.ops.native import native

    rec, K, P = _data(M=100)
    path = str(tmp_path / "s.rec")
    write_records(path, rec, K)
    r = native().RecordReader(path, 10, 3, False)
    a, b = r.acquire(), r.acquire()
    assert a[0] != b[0] and (a[1], b[1]) == (0, 10)
    assert torch.equal(a[2], rec[:10]) and torch.equal(b[2], rec[10:20])
    with pytest.raises(Exception):
        r.release(b[0])  # out of order
    r.release(a[0])
    r.release(b[0])
    rest = []
    while (w := r.acquire()) is not None:
        rest.append(w[1])
        r.release(w[0])
    assert rest == list(range(20, 100, 10))
