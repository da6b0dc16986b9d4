"""krr_amd.utils.numa: the cpulist parser and a binding that never leaves the allowed CPUs."""
import os

from krr_amd.utils import numa


def test_cpulist():
    assert numa._parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert numa._parse_cpulist("") == set()


def test_local_cpus_within_the_affinity(monkeypatch):
    monkeypatch.setattr(numa, "gpu_numa_node", lambda device=0: 0)
    cpus = numa.gpu_local_cpus(0)
    if cpus is not None:  # a host with sysfs NUMA nodes
        assert cpus <= os.sched_getaffinity(0)
    monkeypatch.setattr(numa, "gpu_numa_node", lambda device=0: None)
    assert numa.gpu_local_cpus(0) is None and numa.bind_local(0) is None
