"""TailTable (engine/native/tail.py) task tables on the CPU: the partition of a table whose tiles
exceed one launch keeps the task order, drops a wait whose producers ran in an earlier launch,
and counts ``need`` over the launch's own producers."""
import torch

from distributed_char_rnn_amd.engine.native import tail as T

W = T.TAIL_WORDS


def _tasks(tab):
    return [tab.words[i * W:(i + 1) * W] for i in range(len(tab.ops))]


def _table():
    tab = T.TailTable(16)
    part = torch.zeros(2, 640, 256)           # 10 x 4 = 40 tiles
    dew = torch.zeros(72, 2048)
    tab.sum(torch.zeros(4, 72, 2048), dew, norm=False, sig=0)     # producer: 2 x 32 = 64 tiles
    tab.sum(part, torch.zeros(640, 256), norm=True)
    E, Wx = torch.zeros(65, 512), torch.zeros(512, 2048)
    tab.mm(torch.zeros(512, 2048), E, (1, 512), dew, (2048, 1), 65, norm=True, wait=0)
    tab.mm(torch.zeros(65, 512), dew, (2048, 1), Wx, (1, 2048), 2048, norm=True, wait=0,
           slabs=torch.zeros(4, 65, 512), slab_sig=1)
    return tab


def test_partition_whole_table_is_itself():
    tab = _table()
    assert tab.partition(10 ** 6) == [tab]


def test_partition_splits_and_rewires_waits():
    tab = _table()
    full = _tasks(tab)
    parts = tab.partition(300)
    assert len(parts) > 1
    assert all(sum(p.tiles) <= 300 for p in parts)
    got = [t for p in parts for t in _tasks(p)]
    assert len(got) == len(full)
    for a, b in zip(got, full):
        # same task in the same order; only wait / need (words 4, 5) may change
        assert a[:4] == b[:4] and a[6:] == b[6:]
    for p in parts:
        produced = {}
        for t, nt in zip(_tasks(p), p.tiles):
            op, wait, need, sig = t[0], t[4], t[5], t[6]
            if wait >= 0:
                assert need == produced.get(wait, 0) > 0
            if sig >= 0:
                produced[sig] = produced.get(sig, 0) + nt
    # the first launch holds the dEW producer; a waiting MM in a later launch waits for nothing
    first = _tasks(parts[0])
    assert first[0][6] == 0
    for p in parts[1:]:
        for t in _tasks(p):
            if t[0] == T.MM and t[4] == 0:
                raise AssertionError("waits on a producer of an earlier launch")
