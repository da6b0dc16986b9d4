"""Multi-rank path on CPU: sharding + RCCL-style result gather, world_size 2 over gloo.

The per-rank compute is stood in for by the CPU oracle (test infrastructure);
what is under test is shard_bounds / pack_records / gather_records /
unpack_records — the N > 1 path bench.py runs over RCCL on the GPU box.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from krr_amd.core.distributed import gather_records, pack_records, record_counts, shard_bounds, unpack_records
from oracle import oracle


def test_shard_bounds_cover_and_balance():
    rng = np.random.default_rng(0)
    w = rng.integers(0, 20000, size=1001)
    for world in (1, 2, 3, 8, 16):
        b = shard_bounds(w, world)
        assert b[0][0] == 0 and b[-1][1] == w.size
        assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
        loads = [int(w[lo:hi].sum()) for lo, hi in b]
        assert max(loads) - min(loads) <= 2 * int(w.max()) + 1
    assert shard_bounds([], 4) == [(0, 0)] * 4
    assert shard_bounds([0, 0, 0, 0], 2) == [(0, 2), (2, 4)]


def _fleet(seed=1):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 3000, size=57)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    cpu = rng.gamma(2.0, 0.05, size=int(offs[-1]))
    mem = np.floor(rng.normal(2e8, 2e7, size=int(offs[-1])))
    return offs, cpu, mem


def _compute(offs, cpu, mem, lo, hi):
    o = offs[lo:hi + 1] - offs[lo]
    c = cpu[offs[lo]:offs[hi]]
    m = mem[offs[lo]:offs[hi]]
    cv, cn, cf = oracle.percentile(c, o, 2, 99, 1, 0.99)
    mv, mn, mf = oracle.seg_max(m, o)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dt)
    return {"cpu_value": t(cv, torch.float64), "cpu_count": t(cn, torch.int64),
            "cpu_flags": t(cf.astype(np.int32), torch.int32), "mem_value": t(mv, torch.float64),
            "mem_count": t(mn, torch.int64), "mem_flags": t(mf.astype(np.int32), torch.int32)}


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        offs, cpu, mem = _fleet()
        lo, hi = shard_bounds(np.diff(offs), world)[rank]
        rec = pack_records(_compute(offs, cpu, mem, lo, hi))
        out = gather_records(rec, dst=0)
        # the pipelined form bench.py uses: counts exchanged once, gather in flight
        # while the caller already overwrites its record buffer
        counts = record_counts(rec.shape[0], rec.device)
        pend = gather_records(rec, dst=0, counts=counts, async_op=True)
        rec.fill_(-1)
        out2 = pend.wait()
        # copy_local=False (bench.py's RCCL form with alternating record buffers):
        # an unpadded shard is sent from the caller's buffer, which stays untouched
        rec = pack_records(_compute(offs, cpu, mem, lo, hi))
        out3 = gather_records(rec, dst=0, counts=counts, async_op=True, copy_local=False).wait()
        # equal shard sizes: the receive buffer itself is the fleet (no trim copy)
        eq = torch.full((7, 4), rank, dtype=torch.int64)
        out4 = gather_records(eq, dst=0, counts=[7] * world, async_op=True, copy_local=False).wait()
        empty = gather_records(eq[:0], dst=0)
        if rank == 0:
            assert torch.equal(out2, out) and torch.equal(out3, out)
            assert out4.shape == (7 * world, 4)
            assert torch.equal(out4[:, 0], torch.arange(world).repeat_interleave(7))
            assert empty.shape == (0, 4)
            q.put(unpack_records(out))
        else:
            assert out is None and out2 is None and out3 is None and out4 is None and empty is None
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_gather_reassembles_fleet_in_order(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    offs, cpu, mem = _fleet()
    want = _compute(offs, cpu, mem, 0, offs.size - 1)
    for k, v in want.items():
        w = v.numpy()
        g = got[k]
        if w.dtype == np.float64:
            assert np.array_equal(g.view(np.uint64), w.view(np.uint64)) or np.array_equal(g, w, equal_nan=True), k
        else:
            assert np.array_equal(g.astype(np.int64), w.astype(np.int64)), k


def test_record_roundtrip_keeps_bits_and_flags():
    d = {"cpu_value": torch.tensor([float("nan"), -0.0, 1.5], dtype=torch.float64),
         "cpu_count": torch.tensor([0, 3, 2**40], dtype=torch.int64),
         "cpu_flags": torch.tensor([4, 0, 1], dtype=torch.int32),
         "mem_value": torch.tensor([2e8, float("inf"), 0.0], dtype=torch.float64),
         "mem_count": torch.tensor([1, 2, 3], dtype=torch.int64),
         "mem_flags": torch.tensor([0, 2, 4], dtype=torch.int32)}
    u = unpack_records(pack_records(d))
    assert np.signbit(u["cpu_value"][1]) and np.isnan(u["cpu_value"][0])
    assert u["cpu_count"].tolist() == [0, 3, 2**40] and u["cpu_flags"].tolist() == [4, 0, 1]
    assert u["mem_flags"].tolist() == [0, 2, 4] and np.isinf(u["mem_value"][1])


# ---------------------------------------------------------------------------
# BatchedRunner's multi-GPU mode (shard -> one pass per rank -> gather -> round on rank 0),
# two gloo ranks as fresh interpreters; the per-rank kernel pass is the oracle stand-in.
# ---------------------------------------------------------------------------
import json  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "config1_reference.json")) as _fh:
    CONFIG1 = json.load(_fh)


def run_sharded_workers(world, compute, entry, path, tmp_path, timeout=300):
    """Start `world` ranks of tests/_sharded_worker.py (gloo); rank 0's rows."""
    port = _free_port()
    out = tmp_path / f"rows_{compute}_{entry}_{path}_{world}.json"
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_sharded_worker.py"), "--compute", compute,
                                       "--entry", entry, "--path", path, "--out", str(out)], env=env))
    codes = []
    for p in procs:
        try:
            codes.append(p.wait(timeout=timeout))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert codes == [0] * world, codes
    with open(out) as fh:
        doc = json.load(fh)
    assert doc["world"] == world
    return doc["rows"]


def expected_rows(path):
    return [[w["rounded"]["cpu_request"], w["rounded"]["mem_request"], w["rounded"]["mem_limit"]]
            for w in CONFIG1["results"][path]]


@pytest.mark.parametrize("entry,path", [("packed", "cli_99_5"), ("loader", "cli_99_5"), ("packed", "default_int"),
                                        ("bodies", "cli_99_5")])
def test_sharded_runner_matches_reference_fixture(entry, path, tmp_path):
    """recommend_packed_sharded / gather_objects_recommendations_sharded on 2 ranks give the
    reference's own config-1 strings (tests/golden/config1_reference.json) for every object."""
    assert run_sharded_workers(2, "oracle", entry, path, tmp_path) == expected_rows(path)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_runner_resolves_exact_history(world, tmp_path):
    """HistoryData with non-canonical Decimals ('0.10', 25-digit values, float
    collisions) through recommend_packed_sharded: the sample objects each rank resolves reach
    rank 0, so N ranks answer as the reference (tests/golden/simple_strategy_exact.json)."""
    with open(os.path.join(HERE, "golden", "simple_strategy_exact.json")) as fh:
        doc = json.load(fh)
    want = [[c["results"]["cli_99_5"]["rounded"][k] for k in ("cpu_request", "mem_request", "mem_limit")]
            for c in doc["cases"] if "rounded" in c["results"]["cli_99_5"]]
    got = run_sharded_workers(world, "oracle", "exact", "cli_99_5", tmp_path)
    assert got == want


def test_sharded_runner_three_ranks_equals_one(tmp_path):
    assert run_sharded_workers(3, "oracle", "packed", "cli_99_5", tmp_path) == \
        run_sharded_workers(1, "oracle", "packed", "cli_99_5", tmp_path)


def test_slice_fleet_and_balanced_bounds():
    from krr_amd.core.distributed import fleet_shard_bounds, slice_fleet
    from krr_amd.core.packing import PackedFleet, PackedSeries

    offs, cpu, mem = _fleet()
    fleet = PackedFleet(PackedSeries(cpu, offs, int(np.diff(offs).max())),
                        PackedSeries(mem, offs.copy(), int(np.diff(offs).max())))
    for world in (1, 2, 5):
        b = fleet_shard_bounds(fleet, world)
        parts = [slice_fleet(fleet, lo, hi) for lo, hi in b]
        assert sum(p.n_objects for p in parts) == fleet.n_objects
        assert np.array_equal(np.concatenate([p.cpu.values for p in parts]), cpu)
        for (lo, hi), p in zip(b, parts):
            assert p.cpu.offsets[0] == 0 and np.array_equal(np.diff(p.cpu.offsets), np.diff(offs[lo:hi + 1]))
            assert p.cpu.max_len == (int(np.diff(offs[lo:hi + 1]).max()) if hi > lo else 0)


def test_subclass_overriding_run_is_not_batched():
    """a SimpleStrategy subclass that overrides only run() keeps its run()."""
    from krr_amd.core.abstract.strategies import supports_batch, supports_packed
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

    class Mine(SimpleStrategy):
        def run(self, history_data, object_data):
            return {}

    class Batched(SimpleStrategy):
        def run_batch(self, histories, objects=None):
            return []

    st = SimpleStrategySettings()
    assert supports_batch(SimpleStrategy(st)) and supports_packed(SimpleStrategy(st))
    assert not supports_batch(Mine(st)) and not supports_packed(Mine(st))
    assert supports_batch(Batched(st))
