"""Host logic of the sampler draw plan (base/sampling.py draw_plan): recorded requests, one
launch for the whole plan from the second iteration, fallback when a request leaves the plan.
The launch itself is replaced by a recorder (the device draw is covered by
tests/test_gpu_sampler.py::test_draw_plan_one_launch_per_iteration)."""
import torch

from base import sampling as S


def _key(n, dim=2, dev=None):
    return (dim, ((n, (-1.0,) * dim, (1.0,) * dim),), dev)


def test_draw_plan_bookkeeping(monkeypatch):
    launches = []
    monkeypatch.setattr(S, "_launch_boxes", lambda reqs, dim, dev: launches.append([o.shape for o, _ in reqs]))

    class Owner:
        pass

    owner, dev = Owner(), torch.device("cpu")
    keys = [_key(100), _key(8), _key(6)]
    with S.draw_plan(owner) as p:  # iteration 0: nothing recorded yet, every request draws alone
        assert [p.take(k, dev) for k in keys] == [None, None, None]
    assert owner._insr_draw_plan == keys and launches == []
    for _ in range(2):  # later iterations: the first request draws the whole plan in one launch
        launches.clear()
        with S.draw_plan(owner) as p:
            outs = [p.take(k, dev) for k in keys]
        assert launches == [[(100, 2), (8, 2), (6, 2)]]
        assert [tuple(o.shape) for o in outs] == [(100, 2), (8, 2), (6, 2)]
        assert len({o.data_ptr() for o in outs}) == 3
    launches.clear()
    with S.draw_plan(owner) as p:  # off the plan at request 1: it and every later one draw alone
        assert p.take(keys[0], dev) is not None
        assert p.take(_key(9), dev) is None
        assert p.take(keys[2], dev) is None
    assert owner._insr_draw_plan == [keys[0], _key(9), keys[2]]
    launches.clear()
    with S.draw_plan(owner) as p:  # a different first request: no plan this iteration
        assert p.take(_key(50), dev) is None
    assert launches == [] and S.draw_plan.active is None


def test_draw_plan_needs_one_dim_and_box_budget(monkeypatch):
    monkeypatch.setattr(S, "_launch_boxes", lambda reqs, dim, dev: None)

    class Owner:
        pass

    dev = torch.device("cpu")
    for keys in ([_key(10, 2), _key(10, 3)],                       # mixed dims: one launch cannot hold both
                 [_key(10)] * 9,                                    # more boxes than INSR_MAX_BOXES
                 [_key(10)]):                                       # a single request: nothing to batch
        owner = Owner()
        with S.draw_plan(owner) as p:
            for k in keys:
                p.take(k, dev)
        with S.draw_plan(owner) as p:
            assert all(p.take(k, dev) is None for k in keys)
