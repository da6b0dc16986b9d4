"""Host diagnostics the bench line reports beside the grouped e2e (NUMA placement of pages,
transparent huge pages of a buffer, the cgroup CPU quota and throttling)."""
import numpy as np

from krr_amd.utils.numa import mapping_info, page_nodes


def test_page_nodes_counts_sampled_pages():
    a = np.ones(1 << 22, dtype=np.uint8)  # touched: every page is resident
    got = page_nodes(a.ctypes.data, a.nbytes, samples=16)
    if got is None:  # not x86_64 / the query refused: nothing to check
        return
    assert sum(got.values()) == 16
    assert all(k >= 0 for k in got)  # resident pages report their node, not -errno
    assert page_nodes(a.ctypes.data, 0) is None


def test_mapping_info_covers_the_buffer():
    a = np.ones(1 << 24, dtype=np.uint8)
    info = mapping_info(a.ctypes.data, a.nbytes)
    assert info is not None and info["mappings"] >= 1
    assert info["Size"] * 1024 >= a.nbytes and info["Rss"] * 1024 >= a.nbytes
    assert 0 <= info.get("AnonHugePages", 0) <= info["Size"]


def test_cgroup_cpu_reads_counters_or_nothing():
    import bench

    cg = bench.cgroup_cpu()
    assert isinstance(cg, dict)
    for k in ("nr_periods", "nr_throttled"):
        if k in cg:
            assert isinstance(cg[k], int) and cg[k] >= 0
