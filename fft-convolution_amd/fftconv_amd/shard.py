"""Channel sharding across GPUs (one process per GPU).

Channels are fully independent convolvers (the reference is one instance per
channel, src/fft_convolver.rs:86-102), so a node-level batch of C channels is
split into contiguous per-rank blocks with no data-path exchange.  Synthetic
IRs and dry blocks are seeded by *global* channel id, so a channel's output is
bit-identical whatever the world size.  The only collective is the optional
dry-block broadcast for the "one source, many IRs" case (`broadcast_dry`).
"""
from __future__ import annotations

import numpy as np

IR_SEED = 1234
DRY_SEED = 4321


def channel_range(rank: int, world: int, channels_per_rank: int) -> range:
    """Global channel ids owned by `rank` (weak scaling: fixed channels per GPU)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    lo = rank * channels_per_rank
    return range(lo, lo + channels_per_rank)


def split_channels(total: int, world: int, rank: int) -> range:
    """Strong-scaling split of `total` channels into near-equal contiguous shards."""
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return range(lo, hi)


def synth_irs(channels: range, length: int) -> np.ndarray:
    """White-noise IR per global channel: U[-1,1)/sqrt(L), seed IR_SEED + channel."""
    out = np.empty((len(channels), length), np.float32)
    scale = 1.0 / np.sqrt(max(length, 1))
    for k, c in enumerate(channels):
        out[k] = np.random.default_rng(IR_SEED + c).uniform(-1.0, 1.0, length) * scale
    return out


def synth_dry(channels: range, nblocks: int, block: int) -> np.ndarray:
    """White-noise dry input U[-1,1) per global channel, [nblocks][channels][block]."""
    out = np.empty((nblocks, len(channels), block), np.float32)
    for k, c in enumerate(channels):
        out[:, k, :] = np.random.default_rng(DRY_SEED + c).uniform(-1.0, 1.0, (nblocks, block))
    return out


def synth_shared_dry(nblocks: int, block: int) -> np.ndarray:
    """One dry source for every channel (rank 0 generates, then broadcasts)."""
    return np.random.default_rng(DRY_SEED).uniform(-1.0, 1.0, (nblocks, block)).astype(np.float32)


def broadcast_dry(dist, tensor, src: int = 0):
    """The one collective of the path: rank 0's dry block to every rank
    (RCCL over xGMI on GPUs, gloo in the CPU tests).  In-place."""
    dist.broadcast(tensor, src=src)
    return tensor
