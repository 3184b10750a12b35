"""API-parity gate: the reference's own unit tests
(/root/reference/worker_test.py, 4 tests of ``rater``) run unchanged against
this repository's drop-in ``rater.py``.  The reference tree is read-only and
may be absent (e.g. on a GPU box); the test is skipped then."""
import importlib.util
import os

import pytest

REF_TEST = "/root/reference/worker_test.py"


def _load():
    spec = importlib.util.spec_from_file_location("reference_worker_test", REF_TEST)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # imports `rater` -> this repo's rater.py
    return mod


@pytest.mark.skipif(not os.path.exists(REF_TEST), reason="reference tree not mounted")
@pytest.mark.parametrize("name", ["test_get_trueskill_seed", "test_rate_match",
                                  "test_rate_match_returning", "test_rate_match_afk"])
def test_reference_worker_test(name):
    mod = _load()
    import rater

    assert os.path.dirname(os.path.abspath(rater.__file__)) == os.path.dirname(
        os.path.dirname(os.path.abspath(__file__))), "must test this repo's rater.py"
    getattr(mod.TestRater(), name)()
