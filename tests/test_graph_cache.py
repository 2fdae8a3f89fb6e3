"""Host logic of the captured-chain cache (ops._GraphCache): LRU order and
the eviction wait (an evicted Gram chain's entry synchronizes its fetch
event before its pinned table can be reused).  CPU only: the event is a
stand-in class patched over torch.cuda.Event."""
import torch

from federatedscope_amd import ops


class _Ev:
    def __init__(self):
        self.waits = 0

    def synchronize(self):
        self.waits += 1


def _entry(ev):
    # the pairgram entry's shape: (graph, buf, tab, (pinned, event), keep)
    return (None, None, None, (None, ev), ())


def test_eviction_waits_for_fetch(monkeypatch):
    monkeypatch.setattr(torch.cuda, 'Event', _Ev)
    c = ops._GraphCache()
    evs = [_Ev() for _ in range(c.MAX_ENTRIES + 3)]
    for i, ev in enumerate(evs):
        c.put(('k', i), _entry(ev))
    assert len(c.entries) == c.MAX_ENTRIES
    assert [e.waits for e in evs[:3]] == [1, 1, 1]
    assert all(e.waits == 0 for e in evs[3:])
    assert c.lookup(('k', 0)) is None
    assert c.lookup(('k', 3)) is not None


def test_lookup_refreshes_lru(monkeypatch):
    monkeypatch.setattr(torch.cuda, 'Event', _Ev)
    c = ops._GraphCache()
    evs = [_Ev() for _ in range(c.MAX_ENTRIES)]
    for i, ev in enumerate(evs):
        c.put(('k', i), _entry(ev))
    assert c.lookup(('k', 0)) is not None      # now most recent
    extra = _Ev()
    c.put(('k', 'new'), _entry(extra))
    assert c.lookup(('k', 0)) is not None
    assert c.lookup(('k', 1)) is None
    assert evs[1].waits == 1 and evs[0].waits == 0


def test_entries_without_fetch_evict_plainly():
    c = ops._GraphCache()
    for i in range(c.MAX_ENTRIES + 2):
        c.put(('k', i), (None, None))
    assert len(c.entries) == c.MAX_ENTRIES
