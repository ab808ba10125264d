"""Host-side helpers of the GRPO/PPO loops (index streams, batching, prompt
truncation).  Pure host logic; the numeric per-token work is in `..ops`.
Each function cites the reference symbol whose behaviour it keeps."""
from __future__ import annotations

from typing import Optional, Sequence

import torch


class RepeatSampler:
    """grpo_trainer.py:97-192 — each index repeated `mini_repeat_count` times,
    `batch_size` unique indices per chunk, each chunk emitted `repeat_count`
    times, tail chunk dropped, order from a local seeded torch.Generator."""

    def __init__(self, data_source, mini_repeat_count: int, batch_size: int = 1, repeat_count: int = 1,
                 shuffle: bool = True, seed: Optional[int] = None):
        self.num_samples = len(data_source)
        self.mini_repeat_count, self.batch_size, self.repeat_count = mini_repeat_count, batch_size, repeat_count
        self.shuffle, self.seed = shuffle, seed
        if shuffle:
            self.generator = torch.Generator()
            if seed is not None:
                self.generator.manual_seed(seed)

    def __iter__(self):
        order = (torch.randperm(self.num_samples, generator=self.generator).tolist() if self.shuffle
                 else list(range(self.num_samples)))
        full = self.num_samples // self.batch_size
        for c in range(full):
            chunk = order[c * self.batch_size:(c + 1) * self.batch_size]
            for _ in range(self.repeat_count):
                for idx in chunk:
                    for _ in range(self.mini_repeat_count):
                        yield idx

    def __len__(self):
        return (self.num_samples // self.batch_size) * self.batch_size * self.mini_repeat_count * self.repeat_count


def generation_batch_indices(n: int, num_generations: int, generation_batch_size: int, local_batch_size: int,
                             rank: int, seed: Optional[int], shuffle: bool = True, epochs: Optional[int] = None):
    """This rank's dataset indices of every global generation batch.

    The reference feeds `RepeatSampler(mini_repeat_count=G, batch_size=gbs/G,
    repeat_count=num_iterations*steps_per_generation)` (grpo_trainer.py:1096-1130)
    through accelerate's per-process batch sharding: rank r receives the r-th
    contiguous local chunk of each global generation batch, and the repeats are
    consumed without regenerating (`_prepare_inputs` :1411-1444).  Here the
    repeats are collapsed and each yielded list is one local generation batch
    (whole groups of G: local_batch_size is a multiple of G).  One sampler (one
    generator) serves every epoch, as the reference's dataloader re-iterates
    the same RepeatSampler: each epoch draws a fresh permutation."""
    sampler = RepeatSampler(range(n), mini_repeat_count=num_generations,
                            batch_size=generation_batch_size // num_generations, repeat_count=1,
                            shuffle=shuffle, seed=seed)
    ep = 0
    while epochs is None or ep < epochs:
        idx = list(sampler)
        for s in range(0, len(idx) - generation_batch_size + 1, generation_batch_size):
            yield idx[s + rank * local_batch_size:s + (rank + 1) * local_batch_size]
        ep += 1


def truncate_with_protected_tokens(ids: torch.Tensor, mask: torch.Tensor, target_length: int,
                                   protected_tokens: Sequence[int]):
    """grpo_trainer.py:367-421, vectorised: keep every protected id plus the
    rightmost non-protected ids so each row has `target_length` tokens.  No
    per-token host sync (the reference does one `.item()` per prompt token)."""
    B, L = ids.shape
    if L <= target_length and not protected_tokens:
        return ids, mask
    prot = torch.zeros_like(ids, dtype=torch.bool)
    if protected_tokens:
        prot = torch.isin(ids, torch.tensor(list(protected_tokens), device=ids.device, dtype=ids.dtype))
    n_prot = prot.sum(1)
    need = target_length - n_prot
    if bool((need < 0).any()):
        raise ValueError(f"target_length ({target_length}) is too small for the protected tokens "
                         f"({int(n_prot.max())} tokens). Please increase target length to at least "
                         f"{int(n_prot.max())} or disable truncation.")
    nonp = (~prot).long()
    from_right = nonp.flip(1).cumsum(1).flip(1)  # 1-based rank from the right among non-protected
    keep = prot | ((~prot) & (from_right <= need.unsqueeze(1)))
    counts = keep.sum(1)
    if bool((counts != counts[0]).any()):
        raise ValueError("rows shorter than target_length cannot be truncated to a common width")
    w = int(counts[0])
    return ids[keep].view(B, w), mask[keep].view(B, w)


def pad(tensors: Sequence[torch.Tensor], padding_value: int = 0, padding_side: str = "right",
        pad_to_multiple_of: Optional[int] = None) -> torch.Tensor:
    """trl/trainer/utils.py:245-308: one [n, *max_shape] tensor holding the
    ragged inputs; the leading (sequence) dim is padded on `padding_side` and
    rounded up to `pad_to_multiple_of`, trailing dims are filled from 0."""
    if padding_side not in ("left", "right"):
        raise ValueError("padding_side must be 'left' or 'right'")
    nd = tensors[0].dim()
    size = [max(int(t.shape[d]) for t in tensors) for d in range(nd)]
    if pad_to_multiple_of:
        size[0] = -(-size[0] // pad_to_multiple_of) * pad_to_multiple_of
    out = tensors[0].new_full([len(tensors), *size], padding_value)
    for i, t in enumerate(tensors):
        lead = size[0] - t.shape[0] if padding_side == "left" else 0
        out[(i, slice(lead, lead + t.shape[0])) + tuple(slice(0, s) for s in t.shape[1:])] = t
    return out


def left_pad(seqs: Sequence[Sequence[int]], pad_id: int, device=None):
    """Left-pad token lists → (ids [B, P] int64, mask [B, P] int32)."""
    P = max((len(s) for s in seqs), default=0)
    ids = torch.full((len(seqs), P), pad_id, dtype=torch.int64)
    mask = torch.zeros((len(seqs), P), dtype=torch.int32)
    for i, s in enumerate(seqs):
        if len(s):
            ids[i, P - len(s):] = torch.as_tensor(list(s), dtype=torch.int64)
            mask[i, P - len(s):] = 1
    return ids.to(device), mask.to(device)


def split_tensor_dict(d: dict, num_chunks: int) -> list[dict]:
    """grpo_trainer.py:214-241."""
    first = next(v for v in d.values() if v is not None)
    n = first.shape[0] // num_chunks
    return [{k: (None if v is None else v[i * n:(i + 1) * n]) for k, v in d.items()} for i in range(num_chunks)]


def shuffle_sequence_dict(d: dict, generator: Optional[torch.Generator] = None) -> dict:
    """grpo_trainer.py:244-271 — one permutation applied to every entry."""
    n = len(next(v for v in d.values() if v is not None))
    perm = torch.randperm(n, generator=generator)

    def take(v):
        if v is None:
            return None
        if isinstance(v, torch.Tensor):
            return v[perm.to(v.device)]
        return [v[int(i)] for i in perm]

    return {k: take(v) for k, v in d.items()}


def nanstd(t: torch.Tensor) -> torch.Tensor:
    """grpo_trainer.py:196-211."""
    keep = t[~torch.isnan(t)]
    n = keep.numel()
    var = ((keep - keep.mean()) ** 2).mean() * (n / (n - 1))
    return torch.sqrt(var)


def pad_left_cat(tensors: Sequence[torch.Tensor], value) -> torch.Tensor:
    """Concatenate [b_i, P_i] tensors along dim 0, left-padding to max P."""
    P = max(t.shape[1] for t in tensors)
    out = []
    for t in tensors:
        if t.shape[1] < P:
            pad = torch.full((t.shape[0], P - t.shape[1]), value, dtype=t.dtype, device=t.device)
            t = torch.cat([pad, t], 1)
        out.append(t)
    return torch.cat(out, 0)


def linear_lr(step: int, total: int, base: float, warmup: int = 0) -> float:
    """transformers get_linear_schedule_with_warmup (the Trainer default)."""
    if warmup and step < warmup:
        return base * step / max(1, warmup)
    return base * max(0.0, (total - step) / max(1, total - warmup))


def get_high_entropy_mask(entropies: torch.Tensor, mask: torch.Tensor, threshold: float) -> torch.Tensor:
    """grpo_trainer.py:341-364 — tokens whose entropy >= the `threshold` quantile of
    the non-pad entropies (on device; torch.quantile's linear interpolation)."""
    valid = entropies[mask.bool()].float()
    if valid.numel() == 0:
        return torch.zeros_like(entropies, dtype=torch.bool)
    thr = torch.quantile(valid, threshold)
    return ((entropies * mask.float()) >= thr) & mask.bool()
