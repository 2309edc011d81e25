"""CPU tests of ilqr_amd.cache (the workspaces the functional API keeps per shape):
reuse, exclusive check-out under concurrency, LRU bound. Fake workspaces, no GPU."""
import threading
import time

from ilqr_amd import cache


class Fake:
    made = 0

    def __init__(self):
        Fake.made += 1
        self.closed = False
        self.busy = 0

    def close(self):
        self.closed = True


def test_reuse_and_clear():
    cache.clear()
    Fake.made = 0
    for _ in range(5):
        with cache.workspace(("k", 1), Fake) as s:
            assert not s.closed
    assert Fake.made == 1 and cache.size() == 1
    cache.clear()
    assert s.closed and cache.size() == 0


def test_concurrent_callers_never_share():
    cache.clear()
    Fake.made = 0
    errors = []

    def work():
        for _ in range(50):
            with cache.workspace(("shape",), Fake) as s:
                s.busy += 1
                if s.busy != 1:
                    errors.append("shared")
                time.sleep(0.0005)
                s.busy -= 1
    ts = [threading.Thread(target=work) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors
    assert cache.size() == 1            # the surplus workspaces were closed on check-in
    assert 1 <= Fake.made <= 4
    cache.clear()


def test_lru_bound_closes_evicted():
    cache.clear()
    made = []

    def mk():
        f = Fake()
        made.append(f)
        return f
    for k in range(cache.MAX_CACHED + 3):
        with cache.workspace(("k", k), mk):
            pass
    assert cache.size() == cache.MAX_CACHED
    assert [f.closed for f in made[:3]] == [True] * 3 and not any(f.closed for f in made[3:])
    with cache.workspace(("k", 3), mk):   # a hit moves it to the back
        pass
    assert len(made) == cache.MAX_CACHED + 3
    cache.clear()
