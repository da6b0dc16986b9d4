"""The host runtime's persistent worker pool (krr_pack.cpp parallel_for) in a forked child:
the child gets none of the parent's worker threads, so it must start its own pool instead of
waiting on tickets nobody takes (a hang without the atfork reset)."""
import multiprocessing as mp

import pytest

from krr_amd.core.prom_native import pack_query_range_bodies

BODY = b'{"status":"success","data":{"resultType":"matrix","result":[{"metric":{},"values":[[1,"0.5"],[2,"1.5"]]}]}}'


def _pack_in_child(q):
    ps = pack_query_range_bodies([[BODY]] * 64, threads=4)
    q.put(float(ps.values.sum()))


def test_packer_pool_survives_fork():
    pack_query_range_bodies([[BODY]] * 64, threads=4)  # the parent's pool has workers now
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    p = ctx.Process(target=_pack_in_child, args=(q,))
    p.start()
    p.join(60)
    if p.is_alive():
        p.kill()
        pytest.fail("the forked child hung in parallel_for")
    assert p.exitcode == 0 and q.get(timeout=5) == 64 * 2.0
