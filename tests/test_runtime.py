"""Actor runtime (the Ray-core subset): actors, refs, resources, GPU pinning,
simulated multi-node rank mapping, queue, failure detection."""
import os
import time

import pytest

from ray_lightning_accelerators_amd import runtime as ray
from ray_lightning_accelerators_amd.accelerators.ray_ddp import RayAccelerator, RayExecutor


@pytest.fixture
def rt():
    ray.init(num_cpus=4, num_gpus=0)
    yield
    ray.shutdown()


@ray.remote
class Counter:
    def __init__(self, start=0):
        self.n = start

    def inc(self, k=1):
        self.n += k
        return self.n

    def env(self, key):
        return os.environ.get(key)

    def pid(self):
        return os.getpid()

    def fail(self):
        raise ValueError("boom")

    def die(self):
        os._exit(3)

    def nested_get(self, box):
        return ray.get(box[0]) * 2

    def make_child(self):
        c = Counter.remote(100)
        return ray.get(c.inc.remote())


def test_actor_calls_are_ordered(rt):
    c = Counter.remote(5)
    refs = [c.inc.remote() for _ in range(20)]
    assert ray.get(refs) == list(range(6, 26))


def test_put_get_and_toplevel_deref(rt):
    c = Counter.remote()
    r = ray.put(7)
    assert ray.get(c.inc.remote(r)) == 7


def test_nested_ref_via_shared_file(rt):
    c = Counter.remote()
    r = ray.put(21)
    assert ray.get(c.nested_get.remote([r])) == 42


def test_exception_type_preserved(rt):
    c = Counter.remote()
    with pytest.raises(ValueError, match="boom"):
        ray.get(c.fail.remote())


def test_wait(rt):
    c = Counter.remote()
    refs = [c.inc.remote() for _ in range(3)]
    ready, not_ready = ray.wait(refs, num_returns=3, timeout=30)
    assert len(ready) == 3 and not not_ready


def test_resources_and_kill(rt):
    a = Counter.options(num_cpus=2).remote()
    ray.get(a.inc.remote())
    assert ray.available_resources()["CPU"] == 2.0
    ray.kill(a)
    time.sleep(0.3)
    assert ray.available_resources()["CPU"] == 4.0
    assert [v["State"] for v in ray.actors().values()] == ["DEAD"]


def test_worker_death_detected(rt):
    a = Counter.remote()
    ray.get(a.inc.remote())
    with pytest.raises(ray.ActorDiedError):
        ray.get(a.die.remote(), timeout=30)
    time.sleep(0.5)
    assert [v["State"] for v in ray.actors().values()] == ["DEAD"]


def test_nested_actor_dies_with_owner(rt):
    a = Counter.remote()
    assert ray.get(a.make_child.remote()) == 101
    assert sum(v["State"] == "ALIVE" for v in ray.actors().values()) == 2
    ray.kill(a)
    time.sleep(1.5)
    assert all(v["State"] == "DEAD" for v in ray.actors().values())


def test_pending_until_resources_free(rt):
    big = Counter.options(num_cpus=4).remote()
    ray.get(big.inc.remote())
    waiting = Counter.options(num_cpus=1).remote()
    ref = waiting.inc.remote()
    ready, _ = ray.wait([ref], timeout=1.0)
    assert not ready  # cannot be scheduled yet
    ray.kill(big)
    assert ray.get(ref, timeout=60) == 1


def test_gpu_pinning_env():
    """GPU actors get one device each via HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES."""
    ray.init(num_cpus=4, num_gpus=0, _nodes=[{"ip": "127.0.0.1", "num_cpus": 4, "num_gpus": 2,
                                              "gpu_ids": ["0", "1"]}])
    try:
        ws = [Counter.options(num_gpus=1).remote() for _ in range(2)]
        vis = sorted(ray.get([w.env.remote("HIP_VISIBLE_DEVICES") for w in ws]))
        cvis = sorted(ray.get([w.env.remote("CUDA_VISIBLE_DEVICES") for w in ws]))
        assert vis == ["0", "1"] and cvis == ["0", "1"]
        assert ray.available_resources()["GPU"] == 0.0
        cpu_only = Counter.remote()
        assert ray.get(cpu_only.env.remote("HIP_VISIBLE_DEVICES")) == ""
    finally:
        ray.shutdown()


def test_multi_node_local_ranks():
    """Fake node IPs: local ranks restart at 0 on every node (reference ray_ddp.py:132-143)."""
    ray.init(_nodes=[{"ip": "10.0.0.1", "num_cpus": 2}, {"ip": "10.0.0.2", "num_cpus": 2}])
    try:
        acc = RayAccelerator(num_workers=4)
        acc.workers = [acc._create_worker() for _ in range(4)]
        ips = ray.get([w.get_node_ip.remote() for w in acc.workers])
        assert sorted(ips) == ["10.0.0.1", "10.0.0.1", "10.0.0.2", "10.0.0.2"]
        local = acc.get_local_ranks()
        per_node = {}
        for ip, lr in zip(ips, local):
            per_node.setdefault(ip, []).append(lr)
        assert all(sorted(v) == [0, 1] for v in per_node.values())
        for w in acc.workers:
            ray.kill(w)
    finally:
        ray.shutdown()


def test_queue(rt):
    q = ray.Queue(actor_options={"num_cpus": 0})
    assert ray.available_resources()["CPU"] == 4.0
    for i in range(5):
        q.put(i)
    assert q.size() == 5
    assert q.drain() == [0, 1, 2, 3, 4]
    with pytest.raises(ray.Empty):
        q.get_nowait()
    q.shutdown()


def test_remote_function(rt):
    @ray.remote
    def add(a, b):
        return a + b

    assert ray.get(add.remote(2, 3)) == 5


def test_session_guards():
    from ray_lightning_accelerators_amd import session

    with pytest.raises(ValueError):
        session.get_actor_rank()
    session.init_session(rank=3, queue=None)
    try:
        assert session.get_actor_rank() == 3
        with pytest.raises(ValueError):
            session.put_queue("x")
        with pytest.raises(ValueError):
            session.init_session(rank=0, queue=None)
    finally:
        session.shutdown_session()


def test_executor_accelerator_pickling_drops_handles(rt):
    import cloudpickle

    acc = RayAccelerator(num_workers=1)
    acc.workers = [RayExecutor.remote()]
    clone = cloudpickle.loads(cloudpickle.dumps(acc))
    assert clone.workers == []
    ray.kill(acc.workers[0])


@ray.remote
class _Probe:
    def info(self):
        import sys

        return {"torch_preloaded": "torch" in sys.modules, "vis": os.environ.get("HIP_VISIBLE_DEVICES"),
                "actor": os.environ.get("RLA_ACTOR_ID"), "cwd": os.getcwd(), "pid": os.getpid(),
                "omp": os.environ.get("OMP_NUM_THREADS")}


def test_prestarted_worker_pool_assigns_actor_env():
    """Actors start on pre-started pool workers (torch already imported, no GPU
    touched) and still get their own GPU pinning, actor id, cwd and thread count."""
    ray.init(num_cpus=4, num_gpus=0, _nodes=[{"ip": "127.0.0.1", "num_cpus": 4, "num_gpus": 2,
                                               "gpu_ids": ["0", "1"]}])
    try:
        time.sleep(8.0)  # the head pre-starts RLA_WORKER_POOL (default: 2 for 4 CPUs) workers at init
        t0 = time.perf_counter()
        a = _Probe.options(num_cpus=2, num_gpus=1).remote()
        b = _Probe.options(num_cpus=1, num_gpus=1).remote()
        ia, ib = ray.get([a.info.remote(), b.info.remote()])
        dt = time.perf_counter() - t0
        assert ia["torch_preloaded"] and ib["torch_preloaded"], (ia, ib)
        assert {ia["vis"], ib["vis"]} == {"0", "1"}
        assert ia["actor"] != ib["actor"] and ia["pid"] != ib["pid"]
        assert ia["omp"] == "2" and ib["omp"] == "1"
        assert ia["cwd"] == os.getcwd()
        assert dt < 5.0, dt  # no interpreter + torch start on the critical path
        # the pool refills: a third actor is also served from it
        time.sleep(8.0)
        c = _Probe.options(num_cpus=1).remote()
        ic = ray.get(c.info.remote())
        assert ic["torch_preloaded"] and ic["vis"] == "", ic
    finally:
        ray.shutdown()


@ray.remote
class _Recyclable:
    def __init__(self, tag):
        self.tag = tag

    def info(self):
        import sys

        return {"pid": os.getpid(), "actor": os.environ.get("RLA_ACTOR_ID"), "tag": self.tag,
                "vis": os.environ.get("HIP_VISIBLE_DEVICES"), "mark": os.environ.get("RLA_TEST_MARK"),
                "parked_before": getattr(sys.modules["builtins"], "_rla_test_parked", 0)}

    def set_env(self, k, v):
        os.environ[k] = v

    def __rla_park__(self):
        import builtins

        builtins._rla_test_parked = getattr(builtins, "_rla_test_parked", 0) + 1


def test_recycled_worker_takes_next_actor_same_gpu():
    """A reusable actor's kill parks its process (after the instance's __rla_park__
    reset); the next actor with the same key and GPU token runs in it with a fresh
    environment and instance; stale handles see the old actor as dead."""
    ray.init(num_cpus=4, _nodes=[{"ip": "127.0.0.1", "num_cpus": 4, "num_gpus": 1, "gpu_ids": ["0"]}])
    try:
        a = _Recyclable.options(num_gpus=1, _reuse="k").remote("first")
        ia = ray.get(a.info.remote())
        ray.get(a.set_env.remote("RLA_TEST_MARK", "leak"))
        ray.kill(a)
        table = ray.actors()
        assert table[ia["actor"]]["State"] == "DEAD"
        assert ray.available_resources().get("GPU") == 1.0
        time.sleep(0.5)
        b = _Recyclable.options(num_gpus=1, _reuse="k").remote("second")
        ib = ray.get(b.info.remote())
        assert ib["pid"] == ia["pid"] and ib["actor"] != ia["actor"], (ia, ib)
        assert ib["tag"] == "second" and ib["vis"] == "0"
        assert ib["mark"] is None  # the environment is the new actor's, not the old one's
        assert ib["parked_before"] == 1  # the reset hook ran once
        with pytest.raises(Exception):
            ray.get(a.info.remote(), timeout=10)  # the old handle's actor is gone
        # another key never gets the parked process
        ray.kill(b)
        time.sleep(0.5)
        c = _Recyclable.options(num_gpus=1, _reuse="other").remote("third")
        assert ray.get(c.info.remote())["pid"] != ia["pid"]
        ray.kill(c)
        # a plain (non-reusable) actor's kill ends its process
        d = _Recyclable.options(num_gpus=1).remote("fourth")
        pd = ray.get(d.info.remote())["pid"]
        ray.kill(d)
        time.sleep(0.3)
        with pytest.raises(ProcessLookupError):
            os.kill(pd, 0)
    finally:
        ray.shutdown()
