"""Device placement of the sharded body path (advisor round 3, high): a rank packs its bodies
and runs its kernel pass on ONE device — LOCAL_RANK's unless the caller names one — never
the packer's default GPU 0 for the pack and LOCAL_RANK's GPU for the kernel.  CPU test: the
pack and the kernel pass are stood in for by recorders."""
import pytest

from krr_amd.core import distributed
from krr_amd.core.runner import BatchedRunner
from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings


def _runner(monkeypatch, local: int):
    r = BatchedRunner(SimpleStrategy(SimpleStrategySettings()))
    seen = {}
    monkeypatch.setattr(distributed, "local_device", lambda: local)
    monkeypatch.setattr(r, "pack_bodies_device",
                        lambda cpu, mem, threads=0, device=None: seen.setdefault("pack", device) or "fleet")
    monkeypatch.setattr(r, "recommend_shard",
                        lambda fleet, group=None, dst=0, device=None: seen.setdefault("run", device))
    return r, seen


@pytest.mark.parametrize("local", [0, 3])
def test_bodies_shard_packs_and_runs_on_local_rank_device(monkeypatch, local):
    r, seen = _runner(monkeypatch, local)
    r.recommend_bodies_shard([[b"x"]], [[b"y"]], parser="device")
    assert seen == {"pack": local, "run": local}


def test_bodies_shard_explicit_device_wins(monkeypatch):
    r, seen = _runner(monkeypatch, 3)
    r.recommend_bodies_shard([[b"x"]], [[b"y"]], parser="device", device=5)
    assert seen == {"pack": 5, "run": 5}
