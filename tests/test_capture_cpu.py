"""rollout.capture_graph / replay_graph keep Python's cyclic collector off while a decode step is captured and while
its replays are enqueued, and restore it afterwards — after a normal return and after an exception (round-5 GPU-suite
abort: a collection inside a capture destroyed an unreachable CUDAGraph, a HIP call the capturing stream forbids).
torch.cuda is mocked: no device needed."""
import contextlib
import gc

import pytest

from dots.rl_amd import rollout


class _FakeGraph:
    log = []

    def capture_begin(self, pool=None):
        self.log.append(("begin", gc.isenabled()))

    def capture_end(self):
        self.log.append(("end", gc.isenabled()))

    def replay(self):
        self.log.append(("replay", gc.isenabled()))


@pytest.fixture
def fake_cuda(monkeypatch):
    cuda = rollout.torch.cuda
    monkeypatch.setattr(cuda, "synchronize", lambda *a, **k: None)
    monkeypatch.setattr(cuda, "Stream", lambda *a, **k: object())
    monkeypatch.setattr(cuda, "stream", lambda s: contextlib.nullcontext())
    monkeypatch.setattr(cuda, "CUDAGraph", _FakeGraph)
    monkeypatch.setattr(rollout, "_CAPTURE_STREAM", None)
    _FakeGraph.log = []
    was = gc.isenabled()
    gc.enable()
    yield _FakeGraph.log
    if not was:
        gc.disable()


def test_capture_runs_the_body_with_collection_off_and_restores_it(fake_cuda):
    seen = []
    g = rollout.capture_graph(lambda: seen.append(gc.isenabled()), pool=None)
    assert seen == [False]
    assert fake_cuda == [("begin", False), ("end", False)]
    assert gc.isenabled()
    rollout.replay_graph(g, 3)
    assert fake_cuda[2:] == [("replay", False)] * 3
    assert gc.isenabled()


def test_capture_restores_collection_after_an_exception(fake_cuda):
    def body():
        assert not gc.isenabled()
        raise RuntimeError("boom")

    with pytest.raises(RuntimeError, match="boom"):
        rollout.capture_graph(body, pool=None)
    assert fake_cuda == [("begin", False), ("end", False)]  # capture_end still ran
    assert gc.isenabled()


def test_capture_leaves_a_disabled_collector_disabled(fake_cuda):
    gc.disable()
    try:
        rollout.capture_graph(lambda: None, pool=None)
        assert not gc.isenabled()
        with pytest.raises(ValueError):
            with rollout.gc_paused():
                raise ValueError
        assert not gc.isenabled()
    finally:
        gc.enable()


def test_replay_restores_collection_after_an_exception(fake_cuda):
    class Bad:
        def replay(self):
            assert not gc.isenabled()
            raise RuntimeError("replay failed")

    with pytest.raises(RuntimeError):
        rollout.replay_graph(Bad(), 2)
    assert gc.isenabled()
