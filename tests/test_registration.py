"""On-demand registration of ordinary CUDA tensors (DeviceGroup._register_call /
_map_slot): which slots a new allocation set invalidates, LRU reuse, and that the
slot table is a pure function of the keys every rank holds (so all ranks map the
same slots).  Host-only: the methods run on stand-in objects, no GPU needed."""
from collections import OrderedDict
from types import SimpleNamespace

from collective_communication_mpi_amd.device import DeviceGroup, stale_keys


def alloc(handle, base, size, gen=0):
    return (handle, base, size, gen)


def test_stale_keys_overlap_rules():
    a0 = alloc(b"h0", 0x1000, 0x1000)
    b0 = alloc(b"k0", 0x9000, 0x1000)
    old = (a0, b0)
    # same allocations: not stale
    assert stale_keys([old], (a0, b0)) == []
    # rank 0 reallocated the same range (new handle / generation): stale
    assert stale_keys([old], (alloc(b"h1", 0x1000, 0x1000, 1), b0)) == [old]
    # partial overlap on rank 1 with a different allocation: stale
    assert stale_keys([old], (a0, alloc(b"k9", 0x9800, 0x4000))) == [old]
    # disjoint new allocations on every rank: the old slot stays valid
    assert stale_keys([old], (alloc(b"h2", 0x4000, 0x1000), alloc(b"k2", 0xc000, 0x100))) == []
    # a rank that reuses its allocation while another rank's differs: only true overlaps count
    assert stale_keys([old], (a0, alloc(b"k3", 0x20000, 0x1000))) == []


class FakeDC:
    def __init__(self):
        self.slots = {}
        self.cleared = []
        self.next = 1

    def set_segment(self, s, base, size, handles, offs, keys):
        if s < 0:
            s = self.next
            self.next += 1
        self.slots[s] = (base, size, tuple(keys))
        return s

    def clear_segment(self, s):
        self.cleared.append(s)
        self.slots.pop(s, None)


def group(rank=0, size=2, slots=2):
    syncs = []
    torch = SimpleNamespace(cuda=SimpleNamespace(synchronize=lambda *_: syncs.append(1)))
    return SimpleNamespace(rank=rank, size=size, reg_slots=slots, _dyn=OrderedDict(), _free_slots=[], dc=FakeDC(),
                           torch=torch, device=None, registrations=0, _syncs=syncs, _pinned=set())


def test_map_slot_lru_and_stale_reuse():
    g = group(slots=2)
    k1 = (alloc(b"a", 0x1000, 0x100), alloc(b"b", 0x1000, 0x100))
    k2 = (alloc(b"c", 0x2000, 0x100), alloc(b"d", 0x2000, 0x100))
    k3 = (alloc(b"e", 0x3000, 0x100), alloc(b"f", 0x3000, 0x100))
    DeviceGroup._map_slot(g, k1)
    DeviceGroup._map_slot(g, k2)
    assert list(g._dyn.values()) == [1, 2] and g._syncs == []  # fresh slots need no device sync
    g._dyn.move_to_end(k1)                                         # k1 used again: k2 is least recent
    DeviceGroup._map_slot(g, k3)
    assert k2 not in g._dyn and g._dyn[k3] == 2 and len(g._syncs) == 1
    # the allocation of k1 on rank 1 is freed and its range reallocated: k1's slot is
    # cleared and reused for the new set, before any LRU eviction
    k1b = (alloc(b"a", 0x1000, 0x100), alloc(b"b2", 0x1000, 0x200, 1))
    DeviceGroup._map_slot(g, k1b)
    assert k1 not in g._dyn and g._dyn[k1b] == 1 and g.dc.cleared == [1]
    assert g.registrations == 4


def test_slot_tables_identical_on_every_rank():
    """Two ranks replaying the same key sequence end with the same slot table."""
    keys = [(alloc(b"a%d" % i, 0x1000 * (i % 3), 0x800, i // 3), alloc(b"b%d" % i, 0x1000 * (i % 2), 0x800, 0))
            for i in range(9)]
    tables = []
    for rank in (0, 1):
        g = group(rank=rank, slots=3)
        for k in keys:
            if k in g._dyn:
                g._dyn.move_to_end(k)
            else:
                DeviceGroup._map_slot(g, k)
        tables.append(dict(g._dyn))
    assert tables[0] == tables[1]


def test_pinned_slots_survive_eviction_and_refuse_remap():
    """a slot a captured HIP graph resolves is pinned -- LRU eviction
    skips it, every slot pinned grows the table, and remapping its range raises."""
    import pytest

    g = group(slots=2)
    k1 = (alloc(b"a", 0x1000, 0x100), alloc(b"b", 0x1000, 0x100))
    k2 = (alloc(b"c", 0x2000, 0x100), alloc(b"d", 0x2000, 0x100))
    k3 = (alloc(b"e", 0x3000, 0x100), alloc(b"f", 0x3000, 0x100))
    k4 = (alloc(b"g", 0x4000, 0x100), alloc(b"h", 0x4000, 0x100))
    DeviceGroup._map_slot(g, k1)
    DeviceGroup._map_slot(g, k2)
    g._pinned.add(k1)                       # captured while least recently used
    DeviceGroup._map_slot(g, k3)            # evicts k2, not the pinned k1
    assert k1 in g._dyn and k2 not in g._dyn and g._dyn[k3] == 2
    g._pinned.add(k3)
    DeviceGroup._map_slot(g, k4)            # every slot pinned: a new one
    assert g._dyn[k4] == 3 and k1 in g._dyn and k3 in g._dyn
    k1b = (alloc(b"a2", 0x1000, 0x100, 7), alloc(b"b", 0x1000, 0x100))
    with pytest.raises(RuntimeError, match="captured HIP graph"):
        DeviceGroup._map_slot(g, k1b)       # k1's range reallocated under a live graph
    assert g._dyn[k1] == 1 and g.dc.cleared == []
    DeviceGroup.unpin_captured(g)
    DeviceGroup._map_slot(g, k1b)           # after unpin the stale slot is reused
    assert k1 not in g._dyn and g._dyn[k1b] == 1


def test_slots_of_the_current_call_are_not_evicted():
    """A collective on two new allocations with one evictable slot left: mapping the second
    must not evict the first (both are resolved by this call's kernel)."""
    g = group(slots=2)
    x = (alloc(b"x", 0x1000, 0x100), alloc(b"x1", 0x1000, 0x100))
    y = (alloc(b"y", 0x2000, 0x100), alloc(b"y1", 0x2000, 0x100))
    g._pinned.update({x})
    DeviceGroup._map_slot(g, x)
    a = (alloc(b"a", 0x3000, 0x100), alloc(b"a1", 0x3000, 0x100))
    b = (alloc(b"b", 0x4000, 0x100), alloc(b"b1", 0x4000, 0x100))
    DeviceGroup._map_slot(g, y)
    DeviceGroup._map_slot(g, a, keep={a})          # evicts y (LRU, unpinned)
    DeviceGroup._map_slot(g, b, keep={a, b})       # a is this call's: a new slot instead
    assert a in g._dyn and b in g._dyn and x in g._dyn and y not in g._dyn
