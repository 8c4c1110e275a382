"""Host ingress sizing and NUMA placement of the multi-device engine (VERDICT r04 "Next 4";
substrafl_amd.multi_device.host_placement): pack workers per GPU from the CPUs the process may
use, bound to the GPU's NUMA node read from sysfs.  CPU only: a fake sysfs tree."""

from substrafl_amd import multi_device as md


def test_pack_threads_per_gpu_follows_the_host():
    assert md.pack_threads_per_gpu(256, 8) == 32  # the 8-GPU node: 32 per GPU (was 2)
    assert md.pack_threads_per_gpu(128, 8) == 16
    assert md.pack_threads_per_gpu(16, 8) == 2
    assert md.pack_threads_per_gpu(8, 8) == 2  # never below 2
    assert md.pack_threads_per_gpu(512, 2) == md.PACK_THREADS_CAP  # capped
    assert md.pack_threads_per_gpu(16, 1) == 16


def test_cpulist_parsing():
    assert md._cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert md._cpulist("") == []


def _fake_sysfs(tmp_path, gpus, nodes):
    pci, node = tmp_path / "pci", tmp_path / "node"
    for bus, n in gpus.items():
        (pci / bus).mkdir(parents=True)
        (pci / bus / "numa_node").write_text(f"{n}\n")
    for n, cpus in nodes.items():
        (node / f"node{n}").mkdir(parents=True)
        (node / f"node{n}" / "cpulist").write_text(cpus + "\n")
    return str(pci), str(node)


def test_host_placement_binds_each_gpu_to_its_node(tmp_path):
    gpus = {f"0000:{0x05 + 0x10 * i:02x}:00.0": (0 if i < 4 else 1) for i in range(8)}
    pci, node = _fake_sysfs(tmp_path, gpus, {0: "0-63,128-191", 1: "64-127,192-255"})
    place = md.host_placement(list(gpus), allowed=range(256), pci_sysfs=pci, node_sysfs=node)
    assert [p["numa_node"] for p in place] == [0, 0, 0, 0, 1, 1, 1, 1]
    assert all(p["threads"] == 32 for p in place)
    assert place[0]["cpus"] == list(range(0, 64)) + list(range(128, 192))
    assert place[7]["cpus"] == list(range(64, 128)) + list(range(192, 256))
    # a cgroup that allows only part of the host: the threads follow it, the binding is intersected
    place = md.host_placement(list(gpus), allowed=range(0, 32), pci_sysfs=pci, node_sysfs=node)
    assert all(p["threads"] == 4 for p in place)
    assert place[0]["cpus"] == list(range(32)) and place[7]["cpus"] == []  # node 1: none allowed -> unbound
    # explicit thread count wins
    assert md.host_placement(list(gpus)[:1], pack_threads=6, allowed=range(8), pci_sysfs=pci,
                             node_sysfs=node)[0]["threads"] == 6


def test_unknown_node_leaves_the_workers_unbound(tmp_path):
    pci, node = _fake_sysfs(tmp_path, {"0000:05:00.0": -1}, {0: "0-7"})
    (p,) = md.host_placement(["0000:05:00.0", ], allowed=range(8), pci_sysfs=pci, node_sysfs=node)
    assert p["numa_node"] is None and p["cpus"] == [] and p["threads"] == 8
    (p,) = md.host_placement(["0000:99:00.0"], allowed=range(8), pci_sysfs=pci, node_sysfs=node)
    assert p["numa_node"] is None and p["cpus"] == []
