"""Sampler orders as tensors, and device-resident dataset discovery.

The Trainer injects ``DistributedSampler`` into every loader
(reference ``ray_ddp.py:280-295``).  When a dataset can live
on the GPU (``SyntheticImageNet``, ``TensorDataset``, the synthetic MNIST
arrays), the fused / graph-captured training steps do not iterate the loader at
all: they rebuild the sampler's epoch order with tensor ops (bit-identical to
iterating it), upload it once per epoch and gather each batch on the device.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch.utils.data import DistributedSampler, RandomSampler, SequentialSampler, Subset, TensorDataset


def deterministic_sampler(sampler) -> bool:
    """True when every epoch iterates the sampler in the same order."""
    if isinstance(sampler, DistributedSampler):
        return not sampler.shuffle
    return isinstance(sampler, SequentialSampler)


def sampler_order(sampler) -> torch.Tensor:
    """The sampler's epoch order as an int64 tensor.  DistributedSampler /
    RandomSampler(no replacement) / SequentialSampler orders are rebuilt with
    tensor ops (bit-identical to iterating them: same generator draws), not a
    55K-element Python list per epoch; anything else is iterated."""
    if isinstance(sampler, DistributedSampler):
        n = len(sampler.dataset)
        if sampler.shuffle:
            g = torch.Generator()
            g.manual_seed(sampler.seed + sampler.epoch)
            idx = torch.randperm(n, generator=g)
        else:
            idx = torch.arange(n)
        total = sampler.total_size
        if not sampler.drop_last:
            pad = total - n
            if pad > 0:
                idx = torch.cat([idx, idx.repeat(-(-pad // n))[:pad]])
        else:
            idx = idx[:total]
        return idx[sampler.rank:total:sampler.num_replicas].contiguous()
    if isinstance(sampler, SequentialSampler):
        return torch.arange(len(sampler.data_source))
    if type(sampler) is RandomSampler and not sampler.replacement:
        # torch.utils.data.RandomSampler.__iter__ without replacement: the same
        # global-RNG seed draw (when no generator is set) and the same randperm calls
        n = len(sampler.data_source)
        if sampler.generator is None:
            seed = int(torch.empty((), dtype=torch.int64).random_().item())
            generator = torch.Generator()
            generator.manual_seed(seed)
        else:
            generator = sampler.generator
        m = sampler.num_samples
        parts = [torch.randperm(n, generator=generator) for _ in range(m // n)]
        parts.append(torch.randperm(n, generator=generator)[: m % n])
        return torch.cat(parts)
    return torch.as_tensor(list(iter(sampler)), dtype=torch.int64)


def loader_order(dl) -> torch.Tensor:
    """The index order ONE ``iter(dl)`` walks, making the same global-RNG draws:
    the loader iterator's base-seed draw (``_BaseDataLoaderIter.__init__``) comes
    before the sampler's own (a shuffling ``RandomSampler`` then draws its seed)."""
    torch.empty((), dtype=torch.int64).random_(generator=dl.generator)
    return sampler_order(dl.sampler)


def unwrap_subsets(dataset) -> Tuple[object, Optional[torch.Tensor]]:
    """(base dataset, index map or None) through a chain of ``Subset`` wrappers."""
    idx_map = None
    ds = dataset
    while isinstance(ds, Subset):
        ind = torch.as_tensor(ds.indices, dtype=torch.int64)
        idx_map = ind if idx_map is None else ind[idx_map]
        ds = ds.dataset
    return ds, idx_map


def resident_tensors(dataset, device: torch.device) -> Optional[Tuple[List[torch.Tensor], Optional[torch.Tensor]]]:
    """Device copies of a dataset whose batches are row gathers of a few tensors,
    as ``default_collate`` would stack them, plus the Subset index map.

    Two kinds qualify: a dataset that implements ``resident_tensors(device)``
    (returning the stacked columns of every item, e.g. ``SyntheticImageNet``), and
    ``TensorDataset``.  Anything else (per-item transforms, random augmentation)
    returns None and keeps its DataLoader."""
    base, idx_map = unwrap_subsets(dataset)
    fn = getattr(base, "resident_tensors", None)
    if callable(fn):
        cols = fn(device)
    elif isinstance(base, TensorDataset):
        cols = [t.to(device) for t in base.tensors]
    else:
        return None
    if cols is None:
        return None
    return list(cols), idx_map


def gather_rows(t: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """``t[idx]`` along dim 0, keeping a channels_last image tensor channels_last
    (the gather runs on the dense NHWC view: one contiguous copy per row)."""
    if t.dim() == 4 and not t.is_contiguous() and t.is_contiguous(memory_format=torch.channels_last):
        return t.permute(0, 2, 3, 1).index_select(0, idx).permute(0, 3, 1, 2)
    return t.index_select(0, idx)
