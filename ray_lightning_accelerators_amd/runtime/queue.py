"""Actor-hosted FIFO queue (reference util.py:16-85 / ray.util.queue).

The queue actor is created with ``num_cpus=0`` by the accelerators so it fits
inside a Tune trial's reservation (reference ray_ddp.py:173-176).  Calls are
served by a small thread pool so a blocking ``get`` cannot starve ``put``.
"""
from __future__ import annotations

import queue as _q
import time
from typing import Any, Dict, List, Optional

from . import client


class Empty(Exception):
    pass


class Full(Exception):
    pass


class _QueueActor:
    def __init__(self, maxsize: int = 0):
        self.maxsize = maxsize
        self.q: _q.Queue = _q.Queue(maxsize)

    def qsize(self) -> int:
        return self.q.qsize()

    def empty(self) -> bool:
        return self.q.empty()

    def full(self) -> bool:
        return self.q.full()

    def put(self, item: Any, timeout: Optional[float] = None) -> None:
        try:
            self.q.put(item, timeout=timeout)
        except _q.Full:
            raise Full

    def get(self, timeout: Optional[float] = None) -> Any:
        try:
            return self.q.get(timeout=timeout)
        except _q.Empty:
            raise Empty

    def put_nowait(self, item: Any) -> None:
        try:
            self.q.put_nowait(item)
        except _q.Full:
            raise Full

    def put_nowait_batch(self, items: List[Any]) -> None:
        if self.maxsize > 0 and len(items) + self.q.qsize() > self.maxsize:
            raise Full(f"Cannot add {len(items)} items to queue of size {self.q.qsize()} and maxsize {self.maxsize}")
        for it in items:
            self.q.put_nowait(it)

    def get_nowait(self) -> Any:
        try:
            return self.q.get_nowait()
        except _q.Empty:
            raise Empty

    def get_nowait_batch(self, num_items: int) -> List[Any]:
        if num_items > self.q.qsize():
            raise Empty(f"Cannot get {num_items} items from queue of size {self.q.qsize()}")
        return [self.q.get_nowait() for _ in range(num_items)]

    def drain(self) -> List[Any]:
        out = []
        while True:
            try:
                out.append(self.q.get_nowait())
            except _q.Empty:
                return out

    def get_blocking_batch(self, timeout: float) -> List[Any]:
        """Block up to ``timeout`` for the first item, then drain (no client busy-spin)."""
        try:
            first = self.q.get(timeout=timeout)
        except _q.Empty:
            return []
        return [first] + self.drain()


QUEUE_REUSE_KEY = "rla-queue"


class Queue:
    def __init__(self, maxsize: int = 0, actor_options: Optional[Dict] = None) -> None:
        actor_options = dict(actor_options or {})
        actor_options.setdefault("num_cpus", 0)
        actor_options.setdefault("max_concurrency", 8)
        from ..config import get_config

        if get_config().reuse_workers:
            actor_options.setdefault("_reuse", QUEUE_REUSE_KEY)  # recycled, not restarted
        self.maxsize = maxsize
        self.actor = client.ActorClass(_QueueActor).options(**actor_options).remote(maxsize)

    def __len__(self) -> int:
        return self.size()

    def size(self) -> int:
        return client.get(self.actor.qsize.remote())

    def qsize(self) -> int:
        return self.size()

    def empty(self) -> bool:
        return client.get(self.actor.empty.remote())

    def full(self) -> bool:
        return client.get(self.actor.full.remote())

    def put(self, item: Any, block: bool = True, timeout: Optional[float] = None) -> None:
        if not block:
            return client.get(self.actor.put_nowait.remote(item))
        return client.get(self.actor.put.remote(item, timeout))

    def put_async(self, item: Any):
        return self.actor.put.remote(item, None)

    def get(self, block: bool = True, timeout: Optional[float] = None) -> Any:
        if not block:
            return client.get(self.actor.get_nowait.remote())
        return client.get(self.actor.get.remote(timeout))

    def put_nowait(self, item: Any) -> None:
        return self.put(item, block=False)

    def put_nowait_batch(self, items: List[Any]) -> None:
        return client.get(self.actor.put_nowait_batch.remote(list(items)))

    def get_nowait(self) -> Any:
        return self.get(block=False)

    def get_nowait_batch(self, num_items: int) -> List[Any]:
        return client.get(self.actor.get_nowait_batch.remote(num_items))

    def drain(self) -> List[Any]:
        return client.get(self.actor.drain.remote())

    def get_blocking_batch(self, timeout: float) -> List[Any]:
        return client.get(self.actor.get_blocking_batch.remote(timeout))

    def shutdown(self, force: bool = False, grace_period_s: int = 5) -> None:
        if self.actor is not None:
            client.kill(self.actor)
        self.actor = None
