"""The hybrid parser's share update (krr_amd.core.runner._rebalance): toward equal finishing
times of the device and host sides, damped and bounded, whatever the rates were."""
from krr_amd.core.runner import _rebalance


def test_moves_toward_the_slower_side_and_is_bounded():
    assert _rebalance(0.2, 50e-3, 50e-3) == 0.2
    assert _rebalance(0.2, 50e-3, 100e-3) < 0.2          # host slower: less to the host
    assert _rebalance(0.2, 100e-3, 50e-3) > 0.2          # device slower: more to the host
    assert _rebalance(0.2, 1.0, 1e-6) == 0.25            # at most 25% per call
    assert _rebalance(0.2, 1e-6, 1.0) == 0.2 * 0.8
    assert _rebalance(0.021, 1e-3, 1.0) == 0.02          # within [0.02, 0.8]
    assert _rebalance(0.79, 1.0, 1e-3) == 0.8


def test_settles_where_the_times_meet():
    """A model host whose two sides cost a * share and b * (1 - share) seconds: the share
    settles at b / (a + b)."""
    a, b, s = 0.4, 0.06, 0.5
    for _ in range(40):
        s = _rebalance(s, b * (1 - s), a * s)
    assert abs(s - b / (a + b)) < 0.01
