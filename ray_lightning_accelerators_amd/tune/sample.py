"""Search-space primitives (the ``ray.tune`` sampling API used by the reference:
``tune.choice``, ``tune.loguniform`` -- examples/ray_ddp_example.py:84-89)."""
from __future__ import annotations

import copy
import itertools
import math
import random
from typing import Any, Callable, Dict, List, Sequence


class Domain:
    def sample(self, rng: random.Random, spec: Dict[str, Any]) -> Any:
        raise NotImplementedError


class Categorical(Domain):
    def __init__(self, categories: Sequence[Any]):
        self.categories = list(categories)

    def sample(self, rng, spec):
        return rng.choice(self.categories)

    def __repr__(self):
        return f"choice({self.categories})"


class Float(Domain):
    def __init__(self, lower: float, upper: float, log: bool = False, q: float = None):
        self.lower, self.upper, self.log, self.q = float(lower), float(upper), log, q

    def sample(self, rng, spec):
        if self.log:
            v = math.exp(rng.uniform(math.log(self.lower), math.log(self.upper)))
        else:
            v = rng.uniform(self.lower, self.upper)
        if self.q:
            v = round(v / self.q) * self.q
        return v


class Integer(Domain):
    def __init__(self, lower: int, upper: int, log: bool = False):
        self.lower, self.upper, self.log = int(lower), int(upper), log

    def sample(self, rng, spec):
        if self.log:
            return int(math.exp(rng.uniform(math.log(self.lower), math.log(self.upper))))
        return rng.randrange(self.lower, self.upper)


class Function(Domain):
    def __init__(self, fn: Callable):
        self.fn = fn

    def sample(self, rng, spec):
        try:
            return self.fn(spec)
        except TypeError:
            return self.fn()


class GridSearch:
    def __init__(self, values: Sequence[Any]):
        self.values = list(values)


def choice(categories: Sequence[Any]) -> Categorical:
    return Categorical(categories)


def uniform(lower: float, upper: float) -> Float:
    return Float(lower, upper)


def quniform(lower: float, upper: float, q: float) -> Float:
    return Float(lower, upper, q=q)


def loguniform(lower: float, upper: float, base: float = 10) -> Float:
    return Float(lower, upper, log=True)


def randint(lower: int, upper: int) -> Integer:
    return Integer(lower, upper)


def lograndint(lower: int, upper: int) -> Integer:
    return Integer(lower, upper, log=True)


def randn(mean: float = 0.0, sd: float = 1.0) -> Function:
    return Function(lambda spec=None: random.gauss(mean, sd))


def sample_from(fn: Callable) -> Function:
    return Function(fn)


def grid_search(values: Sequence[Any]) -> Dict[str, List[Any]]:
    return {"grid_search": list(values)}


def _walk(cfg: Any, path=()):
    if isinstance(cfg, dict):
        if set(cfg.keys()) == {"grid_search"}:
            yield path, GridSearch(cfg["grid_search"])
            return
        for k, v in cfg.items():
            yield from _walk(v, path + (k,))
    elif isinstance(cfg, (Domain, GridSearch)):
        yield path, cfg


def _set(cfg: Dict, path, value) -> None:
    d = cfg
    for k in path[:-1]:
        d = d[k]
    d[path[-1]] = value


def generate_variants(config: Dict[str, Any], num_samples: int, seed: int = None) -> List[Dict[str, Any]]:
    """BasicVariantGenerator semantics: grid axes are crossed, random domains
    are re-sampled for every (sample, grid point)."""
    rng = random.Random(seed)
    leaves = list(_walk(config or {}))
    grids = [(p, g.values) for p, g in leaves if isinstance(g, GridSearch)]
    rands = [(p, d) for p, d in leaves if isinstance(d, Domain)]
    out = []
    for _ in range(num_samples):
        for combo in itertools.product(*[vals for _, vals in grids]) if grids else [()]:
            cfg = copy.deepcopy(config or {})
            for (p, _), v in zip(grids, combo):
                _set(cfg, p, v)
            for p, d in rands:
                _set(cfg, p, d.sample(rng, cfg))
            out.append(cfg)
    return out
