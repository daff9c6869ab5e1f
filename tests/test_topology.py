"""xGMI/NUMA/partition-aware placement (gpumounter_amd/hw/topology.py)."""
import itertools

from hypothesis import given, settings
from hypothesis import strategies as st

from gpumounter_amd.hw import topology
from gpumounter_amd.models.device import AmdGpu, LinkMatrix


def node(n=8, hives=None, numa=None, bus=None):
    gpus = []
    for i in range(n):
        gpus.append(AmdGpu(index=i, uuid=f"u{i}", bdf=f"0000:{(bus or {}).get(i, 0x10 * (i + 1)):02x}:00.{i % 8 if bus else 0}",
                           render_minor=128 + i, card_minor=i,
                           xgmi_hive_id=(hives or {}).get(i, 0xABC),
                           numa_node=(numa or {}).get(i, 0 if i < n // 2 else 1)))
    links = LinkMatrix(n=n)
    links.types = [[0 if a == b else (2 if gpus[a].xgmi_hive_id == gpus[b].xgmi_hive_id else 1)
                    for b in range(n)] for a in range(n)]
    links.hops = [[0 if a == b else (1 if links.types[a][b] == 2 else 3) for b in range(n)]
                  for a in range(n)]
    links.weights = [[0 if a == b else (15 if links.types[a][b] == 2 else 72) for b in range(n)]
                     for a in range(n)]
    return gpus, links


def test_small_sets_stay_on_one_numa_node():
    gpus, links = node()
    for n in (1, 2, 3, 4):
        p = topology.choose(gpus, n, links)
        assert p.numa_nodes == 1 and p.non_xgmi_pairs == 0 and len(p.chosen) == n


def test_full_node_and_insufficient():
    gpus, links = node()
    p = topology.choose(gpus, 8, links)
    assert sorted(p.chosen) == list(range(8)) and p.numa_nodes == 2
    assert topology.choose(gpus[:3], 4, links) is None


def test_grow_one_at_a_time_fills_numa_node_first():
    gpus, links = node()
    attached = []
    order = []
    for _ in range(8):
        free = [g for g in gpus if g not in attached]
        p = topology.choose(free, 1, links, attached=attached)
        g = next(x for x in gpus if x.index == p.chosen[0])
        attached.append(g)
        order.append(g.numa_node)
    assert order == [0, 0, 0, 0, 1, 1, 1, 1]


def test_prefers_one_hive_over_numa_locality():
    # two hives of 4; the free set offers a 2+2 split with shared NUMA or a same-hive pair
    hives = {i: (0xA if i < 4 else 0xB) for i in range(8)}
    numa = {0: 0, 1: 1, 2: 1, 3: 1, 4: 0, 5: 0, 6: 1, 7: 1}
    gpus, links = node(hives=hives, numa=numa)
    free = [gpus[0], gpus[4], gpus[1]]
    p = topology.choose(free, 2, links)
    assert sorted(p.chosen) == [0, 1]          # same hive (different NUMA) beats 0+4 (same NUMA)
    assert p.hives == 1 and p.non_xgmi_pairs == 0


def test_attached_gpus_pull_new_ones_into_their_hive():
    hives = {i: (0xA if i < 4 else 0xB) for i in range(8)}
    gpus, links = node(hives=hives)
    p = topology.choose([gpus[1], gpus[5]], 1, links, attached=[gpus[4]])
    assert p.chosen == [5]


def test_cpx_partitions_of_one_package_are_colocated():
    # 4 packages × 2 partitions: partitions share domain:bus
    bus = {i: 0x10 * (i // 2 + 1) for i in range(8)}
    gpus, links = node(bus=bus, numa={i: 0 for i in range(8)})
    p = topology.choose(gpus[1:], 2, links)
    pk = {gpus[i].physical_id for i in p.chosen}
    assert len(pk) == 1


def test_first_fit_policy_is_topology_blind():
    gpus, links = node()
    free = [gpus[3], gpus[4], gpus[5]]
    assert topology.choose(free, 2, links, policy="first-fit").chosen == [3, 4]
    assert topology.choose(free, 2, links).chosen in ([4, 5],)


def test_greedy_path_for_large_inventories():
    gpus, links = node(n=64, numa={i: i // 16 for i in range(64)})
    p = topology.choose(gpus, 8, links)
    assert len(set(p.chosen)) == 8 and p.numa_nodes == 1


@settings(max_examples=50, deadline=None)
@given(st.sets(st.integers(0, 7), min_size=1), st.integers(1, 8))
def test_choice_is_valid_subset(free_idx, n):
    gpus, links = node()
    free = [gpus[i] for i in sorted(free_idx)]
    p = topology.choose(free, n, links)
    if n > len(free):
        assert p is None
        return
    assert len(p.chosen) == n == len(set(p.chosen))
    assert set(p.chosen) <= free_idx
    # optimality on the small exhaustive space: no other subset scores strictly better
    table = {g.index: g for g in gpus}
    best = min(topology.score_set(table, links, list(c))[0]
               for c in itertools.combinations(sorted(free_idx), n))
    assert p.score == best


def test_describe_reports_all_pairs_xgmi():
    gpus, links = node()
    d = topology.describe(gpus, links)
    assert d["all_pairs_xgmi"] and d["numa_nodes"] == 2
