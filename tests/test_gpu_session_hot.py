"""The session-window parity tests again with FW_SESS_HOT=4: every key with >= 4 records in a batch is walked
by k_sess_walk_hot (one wave per key, its slots held in lanes, 64 records loaded at a time) instead of
k_sess_walk's thread per key — the same oracle comparisons, bit-exact (fw_session.hip)."""
import pytest

from test_gpu_session import (hip, oracle_engine, test_session_capacity_error,  # noqa: F401
                              test_session_double_sums_exact, test_session_extreme_timestamps,
                              test_session_first_arrival_f1, test_session_golden_fixture,
                              test_session_hot_keys_and_batches, test_session_many_in_flight, test_session_max_by,
                              test_session_parity_double, test_session_parity_int)

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _hot_walk(monkeypatch):
    monkeypatch.setenv("FW_SESS_HOT", "4")
