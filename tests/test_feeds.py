"""Work feeds of the enrichment engine (dmcp/enrich/feeds.py): the GPU
worker's MultiFeed deals several projects' classes round-robin and forgets a
project once its stream ended AND its queue drained (a long-lived worker
must not keep every project's README and queue)."""
from dmcp.enrich.feeds import IterFeed, MultiFeed, QueueFeed


def test_multifeed_round_robin_and_drop_after_drain():
    f = MultiFeed()
    f.begin(1, "readme one")
    f.begin(2, "readme two")
    f.put(1, [("a", "A"), ("b", "B"), ("c", "C")])
    f.put(2, [("x", "X")])
    f.end(1)  # ended with items still queued (the pool's usual order)
    f.end(2)
    assert f.sessions() == 2
    got = f.take(2)
    assert [k for k, _, _ in got] == [(1, "a"), (2, "x")] and got[0][2] == "readme one"
    assert f.sessions() == 1  # session 2 drained after its end: dropped
    assert [k for k, _, _ in f.take(10)] == [(1, "b"), (1, "c")]
    assert f.sessions() == 0 and not f._readme and not f._order and not f._ended
    f.put(1, [("late", "L")])  # items for a dropped session are ignored
    assert f.take(5) == []


def test_multifeed_end_before_items_and_shutdown():
    f = MultiFeed()
    f.begin(7, None)
    f.end(7)  # nothing queued: dropped at once
    assert f.sessions() == 0
    f.begin(8, "r")
    f.put(8, [("k", "K")])
    assert not f.done
    f.shutdown()
    assert not f.done  # queued work first
    assert f.take(1, wait=True)[0][0] == (8, "k")
    assert f.done


def test_many_sessions_do_not_accumulate():
    f = MultiFeed()
    for sid in range(200):
        f.begin(sid, "x" * 1000)
        f.put(sid, [(i, i) for i in range(3)])
        f.end(sid)
        f.take(3)
    assert f.sessions() == 0


def test_iter_and_queue_feeds():
    it = IterFeed(iter([(1, "a"), (2, "b")]))
    assert it.take(5) == [(1, "a"), (2, "b")] and it.done
    q = QueueFeed()
    q.put([(1, "a")])
    q.close()
    assert q.take(3, wait=True) == [(1, "a")] and q.done
